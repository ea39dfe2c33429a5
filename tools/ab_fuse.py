"""A/B (GPU box): yolox_s bs32 bf16 forward with Bottleneck fusion on vs off, both plans
autotuned and graph-captured in ONE process, replays alternated in rounds so clock and
box state are shared.  Usage: python tools/ab_fuse.py [rounds]"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "pixeltable-yolox_amd"))
from yolox_amd import _native as N  # noqa: E402
from yolox_amd.engine import Plan  # noqa: E402
from yolox_amd.models import YoloxModule  # noqa: E402
from yolox_amd.weights import synthetic_images  # noqa: E402

dev = torch.device("cuda:0")
B, S = 32, 640
model = YoloxModule.synthetic("yolox_s", seed=0, device=dev, dtype=torch.bfloat16)
imgs = torch.from_numpy(synthetic_images(B, S, S, seed=1000)).to(dev)
plans = {}
for fuse in (True, False):
    p = Plan(model, B, S, S, torch.bfloat16, dev, N.NHWC, torch.bfloat16, fuse_bottleneck=fuse)
    p.static_input().copy_(imgs.to(torch.bfloat16))
    p.autotune()
    p.capture()
    plans[fuse] = p
outs = {k: p.replay().clone() for k, p in plans.items()}
torch.cuda.synchronize()
d = (outs[True][..., 4:] - outs[False][..., 4:]).abs()
print(f"obj/cls max diff {d.max().item():.4f}, p99 {d.flatten()[::97].quantile(0.99).item():.4f}")
rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 6
res = {True: [], False: []}
s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
for r in range(rounds):
    for fuse in (True, False) if r % 2 == 0 else (False, True):
        p = plans[fuse]
        for _ in range(3):
            p.replay()
        s.record()
        for _ in range(20):
            p.replay()
        e.record()
        e.synchronize()
        res[fuse].append(s.elapsed_time(e) / 20)
for fuse in (True, False):
    v = sorted(res[fuse])
    print(f"fuse={fuse}: forward median {v[len(v) // 2]:.4f} ms, min {v[0]:.4f} ms over {len(v)} rounds "
          f"({sum(1 for o in plans[fuse].ctx.ops if o.args.get('pre_spec') is not None)} fused Bottlenecks, "
          f"{len(plans[fuse].ctx.ops)} ops)")
