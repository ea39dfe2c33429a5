#!/usr/bin/env python3
"""Aggregate rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes (tools/gpu_profile.sh)
into HBM bytes per TIMED forward of the bench workload -> profiles/traffic_<tag>.json.

Units and the gfx950 correction follow /opt/skills/guides/MI355X_MICROARCH.md (HBM):
FETCH_SIZE / WRITE_SIZE are KiB; FETCH_SIZE counts half of the bytes of a wide
coalesced read on gfx950, so hbm_read = 2 * FETCH_SIZE * 1024.

Which dispatches count (round 6): the capture also holds the bench's pre-capture work (the
eager planning forward, autotune candidates, calibration), whose kernels are forward-family
too.  The dispatches are cut into segments at each forward's first kernel (the stem launch);
the timed forwards are the trailing segments whose forward-family launch lists are identical
(graph replays of one plan), and only the last ``--replays`` of them (the bench's --steps) are
summed.  Per kernel name, the dispatch count must equal replays x its count in one forward's
launch list, and -- given ``--timeline`` (tools/forward_timeline.py output of the kernel-trace
pass) -- that launch list must be the timeline's, name for name.

Usage: python tools/traffic.py PREFIX OUT.json [--replays K] [--timeline T.txt] [model batch size dtype]
       (PREFIX_FETCH_SIZE/ and PREFIX_WRITE_SIZE/ hold run_counter_collection.csv)
"""
import argparse
import csv
import json
from collections import Counter, defaultdict

FWD_KEYS = ("conv_igemm", "conv_glds", "conv_rows", "conv_pw", "conv_r3", "conv_ws", "head_pred", "stem_conv", "stem_rows",
            "stem_s2", "spp_maxpool", "focus_pack", "dwconv")
STEM_KEYS = ("stem_conv", "stem_rows", "stem_s2", "focus_pack")


def is_fwd(name: str) -> bool:
    return any(k in name for k in FWD_KEYS)


def segments(path):
    """[(dispatch rows of one forward-family segment)] in dispatch order, cut at stem launches."""
    rows = [r for r in csv.DictReader(open(path))]
    rows.sort(key=lambda r: int(r["Dispatch_Id"]))
    segs, cur = [], None
    for r in rows:
        name = r["Kernel_Name"]
        if any(k in name for k in STEM_KEYS):
            cur = []
            segs.append(cur)
        if cur is not None and is_fwd(name):
            cur.append((name, float(r["Counter_Value"])))
    return segs


def timed(segs, replays):
    sig = Counter(n for n, _ in segs[-1])
    n_same = 0
    for s in reversed(segs):
        if Counter(n for n, _ in s) != sig:
            break
        n_same += 1
    k = replays or n_same
    if k > n_same:
        raise SystemExit(f"only {n_same} trailing replays share one launch list, {k} asked")
    use = segs[-k:]
    per = defaultdict(float)
    cnt = Counter()
    for s in use:
        for n, v in s:
            per[n] += v
            cnt[n] += 1
    for n, c in sig.items():
        assert cnt[n] == k * c, (n, cnt[n], k, c)
    return use, sig, per, k, n_same, len(segs) - n_same


def timeline_names(path):
    """Kernel names of one forward from tools/forward_timeline.py output ('#  start end dur gap ovl kernel')."""
    names = []
    for line in open(path):
        parts = line.split()
        if len(parts) >= 7 and parts[0].isdigit():
            names.append(" ".join(parts[6:]))
    return names


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("prefix")
    ap.add_argument("out")
    ap.add_argument("rest", nargs="*")
    ap.add_argument("--replays", type=int, default=0, help="timed forwards to sum (the bench's --steps)")
    ap.add_argument("--timeline", default=None)
    a = ap.parse_args()
    model, batch, size, dtype = (a.rest + ["yolox_s", "32", "640", "bf16"][len(a.rest):])[:4]
    fs = segments(f"{a.prefix}_FETCH_SIZE/run_counter_collection.csv")
    ws = segments(f"{a.prefix}_WRITE_SIZE/run_counter_collection.csv")
    _, sig_f, fetch, kf, nsf, pre_f = timed(fs, a.replays)
    _, sig_w, write, kw, nsw, pre_w = timed(ws, a.replays)
    if sig_f != sig_w or kf != kw:
        raise SystemExit("the FETCH_SIZE and WRITE_SIZE passes replayed different launch lists")
    launches = sum(sig_f.values())
    check = None
    if a.timeline:
        tl = timeline_names(a.timeline)
        # the timeline truncates long names: map each launch-list name to its longest timeline prefix
        keys = sorted(set(tl), key=len, reverse=True)
        want = Counter()
        for n, c in sig_f.items():
            d = n[5:] if n.startswith("void ") else n  # demangled names: the timeline drops "void " and the args
            d = d.split("(")[0] if "::" in d else d
            t = next((t for t in keys if d.startswith(t)), "?" + n)
            want[t] += c
        got = Counter(tl)
        if got != want:
            raise SystemExit(f"launch list differs from the timeline's: {sorted((got - want).items())[:4]} / "
                             f"{sorted((want - got).items())[:4]}")
        check = f"{len(tl)} launches per forward, name for name as {a.timeline}"
    rd = 2 * sum(fetch.values()) * 1024 / kf
    wr = sum(write.values()) * 1024 / kw
    top = sorted(((2 * fetch[k] * 1024 + write.get(k, 0) * 1024) / kf, k) for k in fetch)[::-1][:14]
    res = {
        "model": model, "batch": int(batch), "size": int(size), "dtype": dtype,
        "forwards": kf,
        "launches_per_forward": launches,
        "segments_before_the_timed_replays": {"fetch_pass": pre_f + (nsf - kf), "write_pass": pre_w + (nsw - kw)},
        "dispatch_counts_per_kernel": {n: [c, c * kf] for n, c in sorted(sig_f.items())},
        "timeline_check": check,
        "hbm_read_bytes_per_forward": rd,
        "hbm_write_bytes_per_forward": wr,
        "hbm_bytes_per_forward": rd + wr,
        "source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes), FETCH_SIZE x2 (gfx950), KiB->B; "
                  "only the last `forwards` graph replays (identical launch lists, dispatch counts reconciled per "
                  "kernel: [per forward, in the sum]); Infinity-Cache hits are counted (guide)",
        "top_kernels_bytes_per_forward": [[k, b] for b, k in top],
    }
    json.dump(res, open(a.out, "w"), indent=1)
    print(f"{kf} timed forwards of {launches} launches ({pre_f} earlier segments dropped): read {rd / 1e6:.1f} MB, "
          f"write {wr / 1e6:.1f} MB per forward")


if __name__ == "__main__":
    main()
