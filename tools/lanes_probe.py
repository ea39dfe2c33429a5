"""Probe: one batch of 32 yolox_s 640 bf16 images as L concurrent half/quarter batches,
each its own Plan (arena + hipGraph) replayed on its own HIP stream, + device NMS.
Run on the GPU box: python tools/lanes_probe.py"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "pixeltable-yolox_amd"))
from yolox_amd import _native as N  # noqa: E402
from yolox_amd.engine import Plan  # noqa: E402
from yolox_amd.models import YoloxModule  # noqa: E402
from yolox_amd.utils.boxes import postprocess_device  # noqa: E402
from yolox_amd.weights import synthetic_images  # noqa: E402

dev = torch.device("cuda:0")
torch.cuda.set_device(dev)
dt = torch.bfloat16
model = YoloxModule.synthetic("yolox_s", seed=0, device=dev, dtype=dt)
B, S = 32, 640
imgs = torch.from_numpy(synthetic_images(B, S, S, seed=1000)).to(dev).to(dt)
main = torch.cuda.current_stream(dev)
for L in (1, 2, 4, 3):
    bs = [B // L + (1 if i < B % L else 0) for i in range(L)]
    lanes = []
    off = 0
    for i, b in enumerate(bs):
        s = torch.cuda.Stream(dev)
        with torch.cuda.stream(s):
            p = Plan(model, b, S, S, dt, dev, N.NHWC, dt)
            p.static_input().copy_(imgs[off:off + b])
            p.autotune()
            p.capture()
            det = torch.empty(b, p.anchors, 7, dtype=torch.float32, device=dev)
            cnt = torch.empty(b, dtype=torch.int32, device=dev)
        torch.cuda.synchronize()
        lanes.append((s, p, det, cnt))
        off += b

    def step():
        for s, p, det, cnt in lanes:
            s.wait_stream(main)
        for s, p, det, cnt in lanes:
            with torch.cuda.stream(s):
                out = p.replay()
                postprocess_device(out, 80, 0.5, 0.65, det=det, counts=cnt)
        for s, *_ in lanes:
            main.wait_stream(s)

    for _ in range(5):
        step()
    torch.cuda.synchronize()
    K = 30
    t0 = time.perf_counter()
    for _ in range(K):
        step()
    torch.cuda.synchronize()
    dtm = (time.perf_counter() - t0) / K
    dets = sum(int(c.sum()) for *_, c in lanes)
    print(f"lanes {L} {bs}: {dtm * 1e3:.3f} ms/step  {B / dtm:.0f} img/s  dets {dets}", flush=True)
