#!/usr/bin/env python3
"""How much box mAP a FAITHFUL bf16 implementation of configs[1] may lose, by summation order alone.

tests/test_gpu_configs.py scores the device's detections of the 32 configs[1] images against the
fp32 oracle's (ground truth) and compares the loss with the oracle run with bf16 storage
(oracle.stored_as: BN-folded weights and every stored map rounded, fp32 sums).  That emulation is
ONE faithful bf16 implementation; this tool runs others that differ from it only in the order of
the fp32 sums -- exactly the freedom a GPU kernel has -- and scores each the same way:

  emu            F.conv2d's own fp32 summation (the test's emulation)
  emu_f64        the convolution summed in float64, then rounded to fp32 (the correctly rounded sum)
  emu_ksplit2/4  the input channels split in 2 / 4 groups, each group summed, the partials added
  emu_ksplit2r   the same in the reversed group order

Run on the CPU (no GPU, no reference): python tools/map_noise.py [n_images] [out.json]
"""
import json
import os
import sys
import time

import numpy as np
import torch
import torch.nn.functional as F

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "pixeltable-yolox_amd"))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))

from oracle import reference_cpu as O  # noqa: E402  (test infrastructure: this is a diagnostic tool)

_conv2d = F.conv2d


def conv_f64(x, w, b=None, stride=1, padding=0, dilation=1, groups=1):
    y = _conv2d(x.double(), w.double(), None if b is None else b.double(), stride, padding, dilation, groups)
    return y.float()


def conv_ksplit(parts, reverse=False):
    def conv(x, w, b=None, stride=1, padding=0, dilation=1, groups=1):
        cin = w.shape[1]
        if groups != 1 or cin % parts:
            return _conv2d(x, w, b, stride, padding, dilation, groups)
        step = cin // parts
        order = list(range(parts))[::-1] if reverse else list(range(parts))
        y = None
        for g in order:
            t = _conv2d(x[:, g * step:(g + 1) * step], w[:, g * step:(g + 1) * step], None, stride, padding, dilation, 1)
            y = t if y is None else y + t
        return y if b is None else y + b.view(1, -1, 1, 1)
    return conv


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 32
    out_path = sys.argv[2] if len(sys.argv) > 2 else None
    torch.set_num_threads(os.cpu_count() or 8)
    from test_gpu_configs import box_map_vs_oracle  # the test's own scoring
    from yolox_amd.config import named_config
    from yolox_amd.weights import synthetic_images, synthetic_state_dict
    sd = synthetic_state_dict(named_config("yolox_s").get_model().state_dict(), seed=0, bn_stats="yolox_s")
    imgs = synthetic_images(32, 640, 640, seed=1000)[:n]  # bench_plan's images
    x = torch.from_numpy(O.letterbox_identity(imgs))
    arch = O.ARCHS["yolox_s"]

    def run(conv, stored):
        F.conv2d = conv
        try:
            with torch.no_grad(), O.stored_as(stored):
                return O.forward_eval(sd, arch, x).numpy()
        finally:
            F.conv2d = _conv2d

    t0 = time.time()
    ref = run(_conv2d, None)
    ref_dets = O.postprocess(ref.copy(), 80, 0.5, 0.65)
    runs = {"emu": _conv2d, "emu_f64": conv_f64, "emu_ksplit2": conv_ksplit(2), "emu_ksplit2r": conv_ksplit(2, True),
            "emu_ksplit4": conv_ksplit(4)}
    res = {"images": n, "ndet_ref": int(sum(len(np.asarray(d).reshape(-1, 7)) for d in ref_dets))}
    outs = {}
    for name, conv in runs.items():
        o = run(conv, torch.bfloat16)
        outs[name] = o
        dets = O.postprocess(o.copy(), 80, 0.5, 0.65)
        ap = box_map_vs_oracle(dets, ref_dets, 640)
        dp = np.abs(o[..., 4:] - ref[..., 4:])
        res[name] = {"ap50_95": ap[0], "ap50": ap[1], "prob_max": float(dp.max()), "prob_p99": float(np.quantile(dp, 0.99)),
                     "ndet": int(sum(len(np.asarray(d).reshape(-1, 7)) for d in dets))}
        print(name, res[name], f"{time.time() - t0:.0f}s", flush=True)
    # the faithful implementations against each other (emu's detections as the ground truth)
    emu_dets = O.postprocess(outs["emu"].copy(), 80, 0.5, 0.65)
    for name in runs:
        if name != "emu":
            ap = box_map_vs_oracle(O.postprocess(outs[name].copy(), 80, 0.5, 0.65), emu_dets, 640)
            res[f"{name}_vs_emu"] = {"ap50_95": ap[0], "ap50": ap[1]}
    print(json.dumps(res, indent=1))
    if out_path:
        json.dump(res, open(out_path, "w"), indent=1)


if __name__ == "__main__":
    main()
