"""Per-forward wall spans from a rocprofv3 kernel trace of bench.py: a forward starts at a
stem launch and ends at the last conv / head launch before the next post-processing
kernel.  Usage: python tools/forward_spans.py run_kernel_trace.csv"""
import csv
import sys
from collections import defaultdict

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
FWD = ("stem_", "conv_", "head_pred", "spp_maxpool", "focus_pack")
spans, cur, busy = [], None, defaultdict(float)
for r in rows:
    name = r["Kernel_Name"]
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    if "stem_" in name:
        if cur:
            spans.append(cur)
        cur = [s, e, 0.0, 0]
    elif cur and any(k in name for k in FWD):
        cur[1] = max(cur[1], e)
    if cur and any(k in name for k in FWD):
        cur[2] += e - s
        cur[3] += 1
        busy[name.split("<")[0].replace("void ", "")] += e - s
if cur:
    spans.append(cur)
spans = spans[2:]  # drop the autotune / warm-up forwards
n = len(spans)
print(f"{n} forwards: span {sum(x[1] - x[0] for x in spans) / n / 1e3:.1f} us, kernel sum "
      f"{sum(x[2] for x in spans) / n / 1e3:.1f} us, {spans[-1][3]} launches")
tot = sum(busy.values())
for k, v in sorted(busy.items(), key=lambda x: -x[1]):
    print(f"  {v / tot * 100:5.1f}%  {k}")
