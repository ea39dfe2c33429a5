#!/usr/bin/env python3
"""Aggregate rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes (tools/gpu_profile.sh)
into HBM bytes per forward of the bench workload -> profiles/traffic_<tag>.json.

Units and the gfx950 correction follow /opt/skills/guides/MI355X_MICROARCH.md (HBM):
FETCH_SIZE / WRITE_SIZE are KiB; FETCH_SIZE counts half of the bytes of a wide
coalesced read on gfx950, so hbm_read = 2 * FETCH_SIZE * 1024.

Usage: python tools/traffic.py gpurun_out/pmc_v4 profiles/traffic_r01.json [model batch size dtype]
"""
import csv
import json
import sys
from collections import defaultdict

FWD_KEYS = ("conv_igemm", "conv_glds", "conv_rows", "conv_pw", "conv_r3", "conv_ws", "head_pred", "stem_conv", "stem_rows",
            "stem_s2", "spp_maxpool", "focus_pack", "dwconv")


def load(path):
    per_kernel = defaultdict(float)
    n_stem = 0
    with open(path) as f:
        for row in csv.DictReader(f):
            name = row["Kernel_Name"]
            if not any(k in name for k in FWD_KEYS):
                continue
            if "stem_conv" in name or "stem_rows" in name or "stem_s2" in name or "focus_pack" in name:
                n_stem += 1
            per_kernel[name] += float(row["Counter_Value"])
    return per_kernel, n_stem


def main():
    prefix, out = sys.argv[1], sys.argv[2]
    model, batch, size, dtype = (sys.argv[3:7] + ["yolox_s", "32", "640", "bf16"][len(sys.argv[3:7]):])
    fetch, nf = load(f"{prefix}_FETCH_SIZE/run_counter_collection.csv")
    write, nw = load(f"{prefix}_WRITE_SIZE/run_counter_collection.csv")
    if not nf or nf != nw:
        raise SystemExit(f"forward counts differ or zero: {nf} vs {nw}")
    rd = 2 * sum(fetch.values()) * 1024 / nf
    wr = sum(write.values()) * 1024 / nw
    top = sorted(((2 * fetch[k] * 1024 + write.get(k, 0) * 1024) / nf, k) for k in fetch)[::-1][:12]
    res = {
        "model": model, "batch": int(batch), "size": int(size), "dtype": dtype,
        "forwards": nf,
        "hbm_read_bytes_per_forward": rd,
        "hbm_write_bytes_per_forward": wr,
        "hbm_bytes_per_forward": rd + wr,
        "source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes), FETCH_SIZE x2 (gfx950), KiB->B; "
                  "forward kernels only (conv/stem/spp/focus); Infinity-Cache hits are counted (guide)",
        "top_kernels_bytes_per_forward": [[k, b] for b, k in top],
    }
    json.dump(res, open(out, "w"), indent=1)
    print(f"{nf} forwards: read {rd / 1e6:.1f} MB, write {wr / 1e6:.1f} MB per forward")


if __name__ == "__main__":
    main()
