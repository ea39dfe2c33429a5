"""GPU box: CapturedTrainStep vs eager losses over 3 optimizer steps (diagnostic).
Env: YOLOX_AMD_WGRAD_STREAM / YOLOX_AMD_WGRAD_GROUP as in train.py; CAP_SYNC=1 synchronises
after every replayed segment (no main/side concurrency)."""
import os
import sys

import numpy as np
import torch

R = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(R, "pixeltable-yolox_amd"))
os.environ.setdefault("YOLOX_AMD_TRAIN_TUNE", "0")
import yolox_amd.train as T  # noqa: E402
from yolox_amd.config import named_config  # noqa: E402
from yolox_amd.weights import synthetic_state_dict  # noqa: E402

d = np.load(os.path.join(R, "tests", "golden", "train_yolox_s_128.npz"))
x = torch.from_numpy(d["input_u8"]).permute(0, 3, 1, 2).float().cuda()
ls = torch.from_numpy(d["labels"]).cuda()
mods = []
for _ in range(2):
    m = named_config("yolox_s").get_model()
    m.load_state_dict(synthetic_state_dict(m.state_dict(), seed=0, bn_stats="yolox_s"))
    m = m.cuda().train()
    opt = torch.optim.SGD(m.parameters(), lr=0.01, momentum=0.9, nesterov=True)
    m(x, ls)["total_loss"].backward()
    opt.step()
    mods.append((m, opt))
(m1, o1), (m2, o2) = mods
cap = T.CapturedTrainStep(m2, x, ls)
print("plan", [k for k, _ in cap.plan].count("side"), "side segments", flush=True)
if os.environ.get("CAP_SYNC") == "1":
    orig = torch.cuda.CUDAGraph.replay

    def replay(self):
        orig(self)
        torch.cuda.synchronize()
    torch.cuda.CUDAGraph.replay = replay
for it in range(3):
    o1.zero_grad(set_to_none=True)
    ref = m1(x, ls)
    ref["total_loss"].backward()
    got = cap(x, ls)
    torch.cuda.synchronize()
    bad = [n for (n, p1), (_, p2) in zip(m1.named_parameters(), m2.named_parameters()) if not torch.equal(p1.grad, p2.grad)]
    print(it, float(ref["total_loss"]), float(got["total_loss"]), "grad mismatches", len(bad), bad[:4], flush=True)
    o1.step()
    o2.step()
