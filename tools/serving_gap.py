#!/usr/bin/env python3
"""The serving step beyond the forward, from a rocprofv3 --kernel-trace CSV of bench.py: for every
pair of consecutive forwards (a forward starts at its stem launch), the time from the end of the
forward's last kernel to the start of the next forward's stem, and the NMS kernels (pp_*) that ran
in that window or beside the next forward, with their mean durations.

Usage: python tools/serving_gap.py run_kernel_trace.csv [skip_first_forwards]"""
import csv
import statistics
import sys
from collections import defaultdict

FWD = ("stem_", "conv_", "head_pred", "spp_maxpool", "focus_pack", "dwconv")


def main():
    rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
    skip = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    ks = [(r["Kernel_Name"], int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows]
    starts = [i for i, (n, _, _) in enumerate(ks) if "stem_" in n]
    gaps, fwd, per = [], [], defaultdict(list)
    for a, b in zip(starts[skip:], starts[skip + 1:]):
        seg = ks[a:b]
        f_end = max(e for n, s, e in seg if any(k in n for k in FWD))
        gaps.append((ks[b][1] - f_end) / 1e3)
        fwd.append((f_end - ks[a][1]) / 1e3)
        for n, s, e in seg:
            if "pp_" in n:
                per[n.split("(")[0].replace("void ", "")].append((e - s) / 1e3)
    if not gaps:
        sys.exit("fewer than two timed forwards in the trace")
    print(f"{len(gaps)} forward pairs: forward span {statistics.mean(fwd):.1f} us, end of forward -> next stem "
          f"{statistics.mean(gaps):.1f} us (min {min(gaps):.1f}, max {max(gaps):.1f}); step = "
          f"{statistics.mean(fwd) + statistics.mean(gaps):.1f} us")
    for n, v in sorted(per.items(), key=lambda kv: -sum(kv[1])):
        print(f"  {n:40s} x{len(v) / len(gaps):.1f} per step  mean {statistics.mean(v):6.1f} us")


if __name__ == "__main__":
    main()
