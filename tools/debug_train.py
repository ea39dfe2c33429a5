"""Debug: run one fp32 train step of yolox_s@128 and report the first tape entry whose
outputs (parameter gradients / activation gradients) turn non-finite."""
import os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "pixeltable-yolox_amd"), REPO, os.path.join(REPO, "tests")]
import numpy as np, torch
from test_gpu_train import _model_and_batch
from yolox_amd import train as T

m, sd, x, labels, d = _model_and_batch()
m = m.cuda().train()
out = m(x.cuda(), labels.cuda())
print({k: float(v) for k, v in out.items()})
g = m._train_graph
names = {id(p): n for n, p in m.named_parameters()}
tape = list(g.tape)
g.grads.begin()
for i, fn in enumerate(reversed(tape)):
    fn()
    torch.cuda.synchronize()
    flat = g.grads.flat
    if not torch.isfinite(flat).all():
        bad = [names[id(p)] for p in g.grads.params if not torch.isfinite(g.grads.of(p)).all()]
        print("step", i, "non-finite param grads:", bad[:8])
        cl = fn.__closure__ or ()
        for c in cl:
            try:
                v = c.cell_contents
            except ValueError:
                continue
            if isinstance(v, T.Act):
                print("  act", v.ch, v.h, v.w, "grad finite:", None if v.grad is None else bool(torch.isfinite(v.grad).all()))
        break
else:
    print("all finite")
