"""GPU box (diagnostic): one torch.cuda.graph capture of TrainGraph.forward + backward on a
yolox_s 128x128 fixture batch, replayed three times, against an eager model's sequence of the
same steps computed BEFORE the capture (so no other model's work runs between replays).

Usage: python tools/cap_probe.py {seq|noopt|snap}
  seq:   SGD step between replays (eager reference steps too)
  noopt: no optimizer steps (every replay must reproduce step 0 exactly)
  snap:  ONE replay, then check that every eager-allocated tensor the graph reads is unchanged
         and that an eager step of the same model still matches (never replays twice)
Per replay it prints the loss vs the eager one, how many parameter gradients differ, whether
the parameters are finite, and whether the forward-layout weight copies the graph repacked
equal a fresh eager pack of the current master weights."""
import ctypes as C
import os
import sys

import numpy as np
import torch

R = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(R, "pixeltable-yolox_amd"))
os.environ.setdefault("YOLOX_AMD_TRAIN_TUNE", "0")
from yolox_amd import _native as N  # noqa: E402
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
    m(x, ls)["total_loss"].backward()  # eager warm-up (repack table recorded)
    for p in m.parameters():
        p.grad = None
    return m, torch.optim.SGD(m.parameters(), lr=0.01, momentum=0.9, nesterov=True)


names = [n for n, _ in named_config("yolox_s").get_model().named_parameters()]

# eager reference sequence first
m3, o3 = make()
ref = []
for it in range(3):
    for p in m3.parameters():
        p.grad = None
    r = m3(x, ls)
    r["total_loss"].backward()
    torch.cuda.synchronize()
    ref.append((float(r["total_loss"].detach()), [p.grad.detach().clone() for p in m3.parameters()],
                [p.detach().clone() for p in m3.parameters()]))
    if mode == "seq":
        o3.step()
torch.cuda.synchronize()
print("eager losses", [v[0] for v in ref], flush=True)

m2, o2 = make()
g = m2._train_graph
g.grad_total.fill_(1.0)
graph = torch.cuda.CUDAGraph()
with torch.cuda.graph(graph):
    out = g.forward(x, ls)
    g.backward(None)
torch.cuda.synchronize()
print("captured; pack table", g._pack_table is not None, "batched", g._batched, flush=True)
lib = N.lib()
convs = [mod for mod in m2.modules() if isinstance(mod, torch.nn.Conv2d) and id(mod) in g._fwd_w]


def pack_mismatches():
    bad = 0
    for conv in convs:
        w0, w1 = g._fwd_w[id(conv)]
        kh, kw = conv.kernel_size
        cin_pad = w0.numel() // (conv.out_channels * kh * kw)
        t0, t1 = torch.empty_like(w0), torch.empty_like(w1)
        b = conv.bias.detach() if conv.bias is not None else None
        N.check(lib.yxh_fold_bn_pack(conv.weight.detach().data_ptr(), b.data_ptr() if b is not None else None, None,
                                     None, None, None, 0.0, conv.out_channels, conv.in_channels // conv.groups, kh, kw,
                                     cin_pad, g.dcode, t0.data_ptr(), t1.data_ptr(), N.stream_ptr()), "pack")
        torch.cuda.synchronize()
        bad += int(not (torch.equal(t0, w0) and torch.equal(t1, w1)))
    return bad


if mode == "snap":
    ro = {"x": x, "labels": ls, "zero_bias": g.zero_bias, "grad_total": g.grad_total, "pack_table": g._pack_table[0]}
    ro.update({"param." + n: p for n, p in zip(names, m2.parameters())})
    snap = {k: v.detach().clone() for k, v in ro.items()}
    graph.replay()
    torch.cuda.synchronize()
    print("replay loss", float(out["total_loss"]), "eager", ref[0][0], flush=True)
    changed = [k for k, v in ro.items() if not torch.equal(v, snap[k])]
    print("read-only tensors changed by the replay:", changed[:10], len(changed), flush=True)
    for p in m2.parameters():
        p.grad = None
    r = m2(x, ls)
    r["total_loss"].backward()
    torch.cuda.synchronize()
    gbad = [names[i] for i, p in enumerate(m2.parameters()) if not torch.equal(p.grad, ref[1][1][i])]
    print("eager step after the replay: loss", float(r["total_loss"].detach()), "eager", ref[1][0],
          "grads differing", len(gbad), gbad[:3], flush=True)
    sys.exit(0)

for it in range(3):
    before = [p.detach().clone() for p in m2.parameters()]
    pdiff = sum(int(not torch.equal(a, b)) for a, b in zip(before, ref[it][2]))
    graph.replay()
    g.grads.publish(None)
    torch.cuda.synchronize()
    loss = float(out["total_loss"])
    gbad = [names[i] for i, p in enumerate(m2.parameters()) if not torch.equal(p.grad, ref[it][1][i])]
    print(f"{it} replay loss {loss} eager {ref[it][0]} | params differing before replay {pdiff} | grads differing "
          f"{len(gbad)} {gbad[:3]} | packs stale {pack_mismatches()} of {len(convs)} | params finite "
          f"{all(bool(torch.isfinite(p).all()) for p in m2.parameters())}", flush=True)
    if mode == "seq":
        o2.step()
        torch.cuda.synchronize()
