"""Per-kernel time over the last N steps of a rocprofv3 kernel trace, steps delimited by a
marker kernel (default sgd_ema_step, the last launch of a train step).
Usage: python tools/trace_window.py run_kernel_trace.csv [N] [MARKER]"""
import csv
import sys
from collections import defaultdict

path = sys.argv[1]
n = int(sys.argv[2]) if len(sys.argv) > 2 else 5
marker = sys.argv[3] if len(sys.argv) > 3 else "sgd_ema_step"
rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
ends = [i for i, r in enumerate(rows) if marker in r["Kernel_Name"]]
lo, hi = ends[-n - 1] + 1, ends[-1] + 1
win = rows[lo:hi]
t0, t1 = int(win[0]["Start_Timestamp"]), int(win[-1]["End_Timestamp"])
per = defaultdict(lambda: [0.0, 0])
for r in win:
    d = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    per[r["Kernel_Name"]][0] += d
    per[r["Kernel_Name"]][1] += 1
busy = sum(v[0] for v in per.values())
print(f"{n} steps: span {(t1 - t0) / n / 1e3:.1f} us/step, kernel busy {busy / n / 1e3:.1f} us/step, "
      f"{len(win) // n} launches/step")
fam = defaultdict(float)
for k, (d, c) in per.items():
    fam[k.split("<")[0].replace("void ", "")] += d
for k, d in sorted(fam.items(), key=lambda x: -x[1])[:25]:
    print(f"  {d / n / 1e3:9.1f} us/step  {k[:90]}")
