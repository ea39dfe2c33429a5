"""Per-launch time of the conv / weight-gradient kernels of the LAST training step, joined with
the shapes TrainGraph logged (YOLOX_AMD_TRAIN_LOG=path python bench.py --workload train ...).
Usage: python tools/train_shapes.py run_kernel_trace.csv launch_log.json"""
import csv
import json
import sys
from collections import defaultdict

FAMILIES = ("conv_igemm", "conv_glds", "conv_rows", "conv_r3", "conv_pw", "conv_ws", "conv_wgrad", "wgrad_f32<", "wgrad9t_f32",
            "wgrad9t_h", "wgrad1t_h", "dgrad_s2f", "dgrad_s2h")
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
log = json.load(open(sys.argv[2]))
per_step = len(log["launches"]) // log["steps"]
last = log["launches"][-per_step:]
convs = [r for r in rows if any(f in r["Kernel_Name"] for f in FAMILIES)]
tail = convs[-per_step:]
agg = defaultdict(lambda: [0.0, 0, ""])
tot = 0.0
for (kind, k, s, cin, cout, ih, iw, oh, ow, b, tile, nsrc, up, acc), r in zip(last, tail):
    us = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    tot += us
    what = "dgrad-dil" if kind == "dgrad" and up == 2 else kind
    key = f"{what:9s} k{k}s{s} {cin:4d}->{cout:4d} @{oh}x{ow} b{b}"
    a = agg[key]
    a[0] += us
    a[1] += 1
    a[2] = r["Kernel_Name"].split("(")[0].replace("void yxh::", "")[:60]
flops_note = "us"
print(f"last step: {len(tail)} conv/wgrad launches, {tot:.0f} us")
for key, (us, n, kern) in sorted(agg.items(), key=lambda kv: -kv[1][0]):
    print(f"{us:8.1f} us {n:3d}x  {key}  {kern}")
