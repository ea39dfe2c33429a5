"""Graph-branch planning (engine.op_dependencies + head lanes), CPU only: no kernels run."""
import torch

from yolox_amd import _native as N
from yolox_amd.config import named_config
from yolox_amd.engine import Buffer, OpRec, OutBuffer, PlanCtx, op_dependencies


def test_dependency_kinds():
    """Read-after-write, write-after-write and write-after-read edges."""
    a, b, c = (Buffer(4, 4, 8, 2) for _ in range(3))

    def conv(src, out):
        return OpRec(N.OP_CONV, dict(srcs=[src.full()], out=out.full(), residual=None))

    ops = [conv(a, b),   # 0
           conv(b, c),   # 1: reads b (RAW on 0)
           conv(a, b),   # 2: rewrites b (WAW on 0, WAR on 1)
           conv(c, a)]   # 3: reads c (RAW on 1), overwrites a (WAR on 0 and 2)
    assert op_dependencies(ops) == [[], [0], [0, 1], [0, 1, 2]]


def test_head_levels_plan_on_their_own_lanes():
    """Each head level (yolo_head.py:140-211) is its own lane; every cross-lane edge goes
    from the backbone/neck lane into a head lane (the levels wait only for their feature
    map), and the dependency lists only point backwards."""
    m = named_config("yolox_s").get_model()
    ctx = PlanCtx(2, torch.bfloat16, torch.device("cpu"))
    feats = m.backbone.plan(ctx, ctx.image(128, 128))
    m.head.plan(ctx, feats, OutBuffer(sum(f.lh * f.lw for f in feats), 85))
    lanes = [o.lane for o in ctx.ops]
    assert sorted(set(lanes)) == [0, 1, 2, 3]
    deps = op_dependencies(ctx.ops)
    assert all(j < i for i, d in enumerate(deps) for j in d)
    assert all(deps[i] for i in range(1, len(deps)))  # one connected chain from the stem
    cross = [(j, i) for i, d in enumerate(deps) for j in d if lanes[j] != lanes[i]]
    assert cross and all(lanes[j] == 0 and lanes[i] > 0 for j, i in cross)
    for k in (1, 2, 3):  # a level's first op waits only for the neck op producing its input
        first = lanes.index(k)
        assert [lanes[j] for j in deps[first]] == [0]
