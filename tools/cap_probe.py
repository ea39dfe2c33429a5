"""GPU box (diagnostic): one torch.cuda.graph capture of TrainGraph.forward + backward on a
yolox_s 128x128 fixture batch, replayed; which intervening work breaks a later replay?
Usage: python tools/cap_probe.py {interleave|optstep}
  interleave: replay 3x with another model's eager step between replays, no optimizer steps
  optstep:    optimizer step between replays, no other model's work in between"""
import os
import sys

import numpy as np
import torch

R = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(R, "pixeltable-yolox_amd"))
os.environ.setdefault("YOLOX_AMD_TRAIN_TUNE", "0")
from yolox_amd.config import named_config  # noqa: E402
from yolox_amd.weights import synthetic_state_dict  # noqa: E402

mode = sys.argv[1]
d = np.load(os.path.join(R, "tests", "golden", "train_yolox_s_128.npz"))
x = torch.from_numpy(d["input_u8"]).permute(0, 3, 1, 2).float().cuda().contiguous()
ls = torch.from_numpy(d["labels"]).cuda().float().contiguous()


def make():
    m = named_config("yolox_s").get_model()
    m.load_state_dict(synthetic_state_dict(m.state_dict(), seed=0, bn_stats="yolox_s"))
    m = m.cuda().train()
    m(x, ls)["total_loss"].backward()  # eager warm-up
    return m, torch.optim.SGD(m.parameters(), lr=0.01, momentum=0.9, nesterov=True)


m1, o1 = make()
m2, o2 = make()
g = m2._train_graph
for p in m2.parameters():
    p.grad = None
g.grad_total.fill_(1.0)
graph = torch.cuda.CUDAGraph()
with torch.cuda.graph(graph):
    out = g.forward(x, ls)
    g.backward(None)
torch.cuda.synchronize()
print("captured", flush=True)
losses = []
for it in range(3):
    graph.replay()
    g.grads.publish(None)
    torch.cuda.synchronize()
    losses.append(float(out["total_loss"]))
    print(it, "replay", losses[-1], flush=True)
    if mode == "interleave":
        m1.zero_grad(set_to_none=True)
        r = m1(x, ls)
        r["total_loss"].backward()
        torch.cuda.synchronize()
        print(it, "eager other model", float(r["total_loss"].detach()), flush=True)
    else:
        o2.step()
        torch.cuda.synchronize()
        print(it, "optimizer step done", flush=True)
