"""GPU box diagnostic: SPP max-pool input of the yolox_s train forward (fp32, 640, bs 8):
GPU vs oracle values and how many pooling windows pick a different argmax."""
import os
import sys

import torch
import torch.nn.functional as F

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "pixeltable-yolox_amd"), REPO]

from oracle import reference_cpu as O  # noqa: E402
import yolox_amd.train as T  # noqa: E402
from yolox_amd.models import YoloxModule  # noqa: E402
from yolox_amd.weights import synthetic_images, synthetic_labels  # noqa: E402

torch.set_num_threads(16)
m = YoloxModule.synthetic("yolox_s", seed=0, device="cuda").train()
sd = {k: v.detach().cpu().clone() for k, v in m.state_dict().items()}
target = m.backbone.backbone.dark5[1].conv1
got = {}
orig_bc = T.TrainGraph.base_conv


def bc(self, mod, inputs, out=None, residual=None, cin_store=None):
    r = orig_bc(self, mod, inputs, out, residual, cin_store)
    if mod is target:
        got["x"] = r
    return r


T.TrainGraph.base_conv = bc
x = torch.from_numpy(synthetic_images(8, 640, 640, seed=1000)).permute(0, 3, 1, 2).float()
labels = torch.from_numpy(synthetic_labels(8, 640, 640, seed=2000))
out = m(x.cuda(), labels.cuda())
torch.cuda.synchronize()
a = got["x"]
g = a.t[..., a.coff:a.coff + a.ch].permute(0, 3, 1, 2).cpu().float()
cap = {}
orig = F.max_pool2d


def mp(t, k, stride=None, padding=0, *args, **kw):
    cap.setdefault("x", t.detach().clone())
    return orig(t, k, stride=stride, padding=padding, *args, **kw)


F.max_pool2d = mp
with torch.no_grad():
    O.backbone(sd, O.ARCHS["yolox_s"], x, bn_train=True)
r = cap["x"]
print("max abs diff", float((g - r).abs().max()), "max |x|", float(r.abs().max()))
for k in (5, 9, 13):
    _, ig = orig(g, k, 1, k // 2, return_indices=True)
    _, ir = orig(r, k, 1, k // 2, return_indices=True)
    print(k, "argmax differs in", int((ig != ir).sum()), "of", ig.numel(), "windows")
