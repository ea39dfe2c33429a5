"""Timeline of one forward inside a rocprofv3 kernel trace of bench.py: every forward
kernel of the last complete forward with its start / end relative to the forward's first
launch, the gap to the previous kernel's end and how many other forward kernels it
overlaps; then the idle time (no forward kernel running) and the critical tail.
Usage: python tools/forward_timeline.py run_kernel_trace.csv [forward_index_from_end]"""
import csv
import sys

FWD = ("stem_", "conv_", "head_pred", "spp_maxpool", "focus_pack", "dwconv")
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
back = int(sys.argv[2]) if len(sys.argv) > 2 else 2
fw = [r for r in rows if any(k in r["Kernel_Name"] for k in FWD)]
starts = [i for i, r in enumerate(fw) if "stem_" in r["Kernel_Name"]]
i0 = starts[-back]
i1 = starts[-back + 1] if back > 1 else len(fw)
win = fw[i0:i1]
t0 = int(win[0]["Start_Timestamp"])
ivs = [(int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0, r["Kernel_Name"]) for r in win]
end_prev = 0
print(f"{'#':>3} {'start':>8} {'end':>8} {'dur':>7} {'gap':>6} {'ovl':>3}  kernel")
for k, (s, e, n) in enumerate(ivs):
    ovl = sum(1 for j, (s2, e2, _) in enumerate(ivs) if j != k and s2 < e and s < e2)
    short = n.split("(")[0].replace("void ", "")[:70]
    print(f"{k:>3} {s / 1e3:8.1f} {e / 1e3:8.1f} {(e - s) / 1e3:7.1f} {(s - end_prev) / 1e3:6.1f} {ovl:>3}  {short}")
    end_prev = max(end_prev, e)
# idle: union of intervals vs span
span = max(e for _, e, _ in ivs)
cov, cur_s, cur_e = 0, None, None
for s, e, _ in sorted(ivs):
    if cur_e is None or s > cur_e:
        if cur_e is not None:
            cov += cur_e - cur_s
        cur_s, cur_e = s, e
    else:
        cur_e = max(cur_e, e)
cov += cur_e - cur_s
print(f"span {span / 1e3:.1f} us, covered {cov / 1e3:.1f} us, idle {(span - cov) / 1e3:.1f} us, "
      f"kernel sum {sum(e - s for s, e, _ in ivs) / 1e3:.1f} us over {len(ivs)} launches")
