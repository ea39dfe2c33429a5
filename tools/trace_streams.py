"""Per-queue (stream) busy time over the last N steps of a rocprofv3 kernel trace, and the top
kernels of each queue: which stream bounds a step whose side stream overlaps the main one.
Usage: python tools/trace_streams.py run_kernel_trace.csv [N] [MARKER]"""
import csv
import sys
from collections import defaultdict

path = sys.argv[1]
n = int(sys.argv[2]) if len(sys.argv) > 2 else 3
marker = sys.argv[3] if len(sys.argv) > 3 else "sgd_ema_step"
rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
ends = [i for i, r in enumerate(rows) if marker in r["Kernel_Name"]]
win = rows[ends[-n - 1] + 1:ends[-1] + 1]
t0, t1 = int(win[0]["Start_Timestamp"]), int(win[-1]["End_Timestamp"])
print(f"{n} steps, span {(t1 - t0) / n / 1e3:.1f} us/step")
byq = defaultdict(list)
for r in win:
    byq[r["Queue_Id"]].append(r)
for q, rs in sorted(byq.items(), key=lambda x: -len(x[1])):
    busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rs)
    # union of intervals on this queue (kernels of one queue may overlap)
    iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rs)
    cov, cs, ce = 0, iv[0][0], iv[0][1]
    for s, e in iv[1:]:
        if s > ce:
            cov += ce - cs
            cs, ce = s, e
        else:
            ce = max(ce, e)
    cov += ce - cs
    print(f"queue {q}: {len(rs) // n} launches/step, busy {busy / n / 1e3:.1f} us/step, covered {cov / n / 1e3:.1f} us/step")
    fam = defaultdict(float)
    for r in rs:
        fam[r["Kernel_Name"].split("<")[0].replace("void ", "").replace("_ZN3yxh", "")[:60]] += \
            int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    for k, d in sorted(fam.items(), key=lambda x: -x[1])[:12]:
        print(f"    {d / n / 1e3:9.1f} us/step  {k}")
