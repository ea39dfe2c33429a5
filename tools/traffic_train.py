#!/usr/bin/env python3
"""HBM bytes per TRAINING step from rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of
``bench.py --workload train`` (tools/gpu_train_traffic.sh) -> profiles/traffic_<tag>.json.

A step is delimited by the fused optimizer launch (sgd_ema_step, once per step): the bytes of
every kernel dispatched after the first optimizer launch up to and including the last one are
summed (whole steps only: warm-up / first-step repacks excluded) and divided by the number of
optimizer launches in that window.  Units and the gfx950 correction as tools/traffic.py
(MI355X_MICROARCH.md HBM section): KiB, FETCH_SIZE x 2.

Usage: python tools/traffic_train.py gpurun_out/pmc_t2 profiles/traffic_r04_train_yolox_s_bs8_fp32.json \
           yolox_s 8 640 fp32
"""
import csv
import json
import sys
from collections import defaultdict

STEP_KERNEL = "sgd_ema_step"


def load(path):
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Dispatch_Id"]), r["Kernel_Name"], float(r["Counter_Value"])))
    rows.sort()
    marks = [d for d, n, _ in rows if STEP_KERNEL in n]
    if len(marks) < 2:
        raise SystemExit(f"{path}: fewer than two optimizer launches")
    lo, hi = marks[0], marks[-1]
    per_kernel = defaultdict(float)
    for d, n, v in rows:
        if lo < d <= hi:
            per_kernel[n] += v
    return per_kernel, len(marks) - 1


def main():
    prefix, out = sys.argv[1], sys.argv[2]
    model, batch, size, dtype = sys.argv[3:7]
    fetch, nf = load(f"{prefix}_FETCH_SIZE/run_counter_collection.csv")
    write, nw = load(f"{prefix}_WRITE_SIZE/run_counter_collection.csv")
    if nf != nw:
        raise SystemExit(f"step counts differ: {nf} vs {nw}")
    rd = 2 * sum(fetch.values()) * 1024 / nf
    wr = sum(write.values()) * 1024 / nw
    top = sorted(((2 * fetch[k] * 1024 + write.get(k, 0) * 1024) / nf, k) for k in fetch)[::-1][:12]
    res = {
        "workload": "train", "model": model, "batch": int(batch), "size": int(size), "dtype": dtype, "steps": nf,
        "hbm_read_bytes_per_step": rd, "hbm_write_bytes_per_step": wr, "hbm_bytes_per_step": rd + wr,
        "source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes), FETCH_SIZE x2 (gfx950), KiB->B; "
                  "every kernel of whole training steps (between optimizer launches); Infinity-Cache hits are "
                  "counted (guide)",
        "top_kernels_bytes_per_step": [[k, b] for b, k in top],
    }
    json.dump(res, open(out, "w"), indent=1)
    print(f"{nf} steps: read {rd / 1e9:.2f} GB, write {wr / 1e9:.2f} GB per step")


if __name__ == "__main__":
    main()
