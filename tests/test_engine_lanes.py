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


def test_hoisted_lanes_follow_their_inputs():
    """engine.hoist_lanes: every head-lane op moves up to just after the last op it depends on
    (level 0 starts right after the 80x80 PAN output, not after the whole neck), lane 0 and each
    lane keep their order, and the result is a topological order of the same dataflow DAG."""
    from yolox_amd.engine import hoist_lanes
    m = named_config("yolox_s").get_model()
    ctx = PlanCtx(2, torch.bfloat16, torch.device("cpu"))
    feats = m.backbone.plan(ctx, ctx.image(128, 128))
    m.head.plan(ctx, feats, OutBuffer(sum(f.lh * f.lw for f in feats), 85))
    ops = hoist_lanes(ctx.ops)
    assert sorted(map(id, ops)) == sorted(map(id, ctx.ops))
    for k in range(4):
        assert [o for o in ops if o.lane == k] == [o for o in ctx.ops if o.lane == k]
    deps = op_dependencies(ops)
    assert all(j < i for i, d in enumerate(deps) for j in d)
    lanes = [o.lane for o in ops]
    for i, o in enumerate(ops):
        if o.lane and (i == 0 or lanes[i - 1] != o.lane):  # a lane segment starts right after its input
            assert deps[i] and max(deps[i]) == i - 1 or lanes[i - 1] != 0
    first = {k: lanes.index(k) for k in (1, 2, 3)}
    assert first[1] < first[2] < first[3]
    # level 0 starts before the neck's bottom-up path (its stride-2 convs) has run
    assert any(l == 0 for l in lanes[first[1]:])
    assert sum(1 for l in lanes[first[1]:] if l == 0) > 4


def test_dag_dependencies_per_chunk_arena():
    """The DAG of a chunked plan: with a shared arena chunk 1's writers wait for chunk 0's
    readers of the same buffers; with arenas of their own the chunks are not ordered."""
    from yolox_amd.engine import dependencies_rw, op_buffers
    m = named_config("yolox_s").get_model()
    ctx = PlanCtx(2, torch.bfloat16, torch.device("cpu"))
    feats = m.backbone.plan(ctx, ctx.image(128, 128))
    m.head.plan(ctx, feats, OutBuffer(sum(f.lh * f.lw for f in feats), 85))
    n = len(ctx.ops)
    for shared in (True, False):
        rw = []
        for c in range(2):
            key = 0 if shared else c
            for r in ctx.ops:
                reads, writes = op_buffers(r)
                rw.append(([(key, id(b)) for b in reads], [(key, id(b)) for b in writes]))
        deps = dependencies_rw(rw)
        cross = [(j, i) for i in range(n, 2 * n) for j in deps[i] if j < n]
        assert bool(cross) == shared
        assert deps[n:] == [[j + n for j in d] for d in deps[:n]] or shared


def test_lane_and_dag_capture_argument_checks():
    """yxh_graph_create_lanes refuses more than 8 capture streams (the most a GPU test replays;
    round 2's 7-stream crash is unexplained); both graph builders reject
    forward/self dependencies -- all before any HIP call, so this runs without a device."""
    import ctypes as C
    lib = N.lib()
    ops = (N.Op * 2)()
    g = C.c_void_p()
    i32 = lambda v: (C.c_int32 * len(v))(*v)  # noqa: E731
    assert lib.yxh_graph_create_lanes(ops, 2, i32([0, 8]), i32([0, 0, 1]), i32([0]), 9, None, C.byref(g)) == N.EINVAL
    assert b"nlanes" in lib.yxh_last_error()
    assert lib.yxh_graph_create_dag(ops, 2, i32([0, 1, 1]), i32([0]), None, C.byref(g)) == N.EINVAL
    assert b"dependency" in lib.yxh_last_error()
    assert lib.yxh_graph_create_dag(ops, 2, i32([1, 1, 1]), i32([0]), None, C.byref(g)) == N.EINVAL
