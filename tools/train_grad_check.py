"""GPU box diagnostic: yolox_s train step (fp32) gradients vs the oracle's autograd,
every parameter's max-abs error relative to its gradient's max, worst first.
Usage: python tools/train_grad_check.py [size] [batch]"""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "pixeltable-yolox_amd"), REPO]

from oracle import reference_cpu as O  # noqa: E402
from yolox_amd.models import YoloxModule  # noqa: E402
from yolox_amd.weights import synthetic_images, synthetic_labels  # noqa: E402

S = int(sys.argv[1]) if len(sys.argv) > 1 else 640
B = int(sys.argv[2]) if len(sys.argv) > 2 else 8
torch.set_num_threads(16)
m = YoloxModule.synthetic("yolox_s", seed=0, device="cuda").train()
sd = {k: v.detach().cpu().clone() for k, v in m.state_dict().items()}
x = torch.from_numpy(synthetic_images(B, S, S, seed=1000)).permute(0, 3, 1, 2).float()
labels = torch.from_numpy(synthetic_labels(B, S, S, seed=2000))
out = m(x.cuda(), labels.cuda())
out["total_loss"].backward()
torch.cuda.synchronize()
sdo = {k: v.float().requires_grad_(v.is_floating_point() and "running" not in k and "num_batches" not in k)
       for k, v in sd.items()}
ref = O.forward_train(sdo, O.ARCHS["yolox_s"], x, labels)
ref["total_loss"].backward()
print({k: (float(out[k]), float(ref[k])) for k in ("total_loss", "num_fg")})
errs = []
for name, p in m.named_parameters():
    g, gr = p.grad.cpu(), sdo[name].grad
    errs.append((float((g - gr).abs().max() / (gr.abs().max() + 1e-12)), name, float(gr.abs().max())))
errs.sort(reverse=True)
for e in errs[:25]:
    print(f"{e[0]:.3e} {e[1]} (max |g| {e[2]:.3e})")
