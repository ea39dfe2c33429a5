"""One rank of tests/test_gpu_dp.py: the HIP train graph under yolox_amd.dp.DistributedDataParallel
(gloo, both ranks on GPU 0), against the mean of the two ranks' single-process gradients."""
import argparse
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "pixeltable-yolox_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rank", type=int)
    ap.add_argument("--world", type=int, default=2)
    ap.add_argument("--port", type=int)
    ap.add_argument("--out")
    ap.add_argument("--captured", action="store_true",
                    help="the captured DP step (CapturedTrainStep under DistributedDataParallel) vs the eager DP step")
    a = ap.parse_args()
    if a.captured:
        return captured(a)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(a.port), RANK=str(a.rank), WORLD_SIZE=str(a.world))
    import torch
    import torch.distributed as dist

    from yolox_amd.dp import DistributedDataParallel
    from yolox_amd.models import YoloxModule
    from yolox_amd.weights import synthetic_images, synthetic_labels
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=a.rank, world_size=a.world)
    m = YoloxModule.synthetic("yolox_s", seed=0, device="cuda").train()
    x = torch.from_numpy(synthetic_images(2, 128, 128, seed=50 + a.rank)).cuda().permute(0, 3, 1, 2).float()
    lab = torch.from_numpy(synthetic_labels(2, 128, 128, max_gt=8, seed=60 + a.rank)).cuda()
    names = [n for n, _ in m.named_parameters()]
    # single-process gradients of this rank's batch
    out = m(x, lab)
    out["total_loss"].backward()
    torch.cuda.synchronize()
    single = torch.cat([p.grad.detach().flatten().cpu() for p in m.parameters()])
    allg = [None] * a.world
    dist.all_gather_object(allg, single)
    mean = (allg[0] + allg[1]) * 0.5
    for p in m.parameters():
        p.grad = None
    # the same step data parallel
    ddp = DistributedDataParallel(m, device_ids=[0], broadcast_buffers=False)
    out = ddp(x, lab)
    g = m._train_graph
    red = ddp._reducer
    fired = {}
    inner = g.on_param_ready

    def counting(p):
        fired[id(p)] = fired.get(id(p), 0) + 1
        inner(p)

    g.on_param_ready = counting
    out["total_loss"].backward()
    torch.cuda.synchronize()
    got = torch.cat([p.grad.detach().flatten().cpu() for p in m.parameters()])
    err = []
    off = 0
    for n, p in zip(names, m.parameters()):
        k = p.numel()
        d = (got[off:off + k] - mean[off:off + k]).abs().max().item()
        ref = mean[off:off + k].abs().max().item()
        err.append((d / (ref + 1e-12), n))
        off += k
    res = {"rank": a.rank, "worst": max(err), "fired": sorted(set(fired.values())),
           "nfired": len(fired), "nparams": len(names), "order": red.launch_order, "nbuckets": len(red.buckets),
           "loss": float(out["total_loss"]), "single_differs": bool((allg[0] - allg[1]).abs().max() > 0)}
    with open(a.out, "w") as f:
        json.dump(res, f)
    dist.destroy_process_group()


def captured(a):
    """Two copies of the model, each under DistributedDataParallel (gloo, both ranks on GPU 0, a batch of
    its own per rank): copy 1 takes eager DP steps, copy 2 the captured DP step (the reducer's bucket
    all-reduces issued between the replayed segments), fused SGD between steps; losses, every
    parameter gradient (the mean over the ranks) and BN buffer must agree bit for bit over three
    steps, and the averaged gradients must differ from this rank's single-batch ones."""
    os.environ["YOLOX_AMD_TRAIN_TUNE"] = "0"  # by-shape tiles: the same launches in both copies
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(a.port), RANK=str(a.rank), WORLD_SIZE=str(a.world))
    import torch
    import torch.distributed as dist

    import yolox_amd.train as T
    from yolox_amd.dp import DistributedDataParallel
    from yolox_amd.models import YoloxModule
    from yolox_amd.optim import FusedStep
    from yolox_amd.weights import synthetic_images, synthetic_labels
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=a.rank, world_size=a.world)
    x = torch.from_numpy(synthetic_images(2, 128, 128, seed=50 + a.rank)).cuda().permute(0, 3, 1, 2).float()
    lab = torch.from_numpy(synthetic_labels(2, 128, 128, max_gt=8, seed=60 + a.rank)).cuda()
    runs = []
    for _ in range(2):
        m = YoloxModule.synthetic("yolox_s", seed=0, device="cuda").train()
        ddp = DistributedDataParallel(m, device_ids=[0], broadcast_buffers=False)
        opt = torch.optim.SGD(m.parameters(), lr=0.01, momentum=0.9, nesterov=True)
        step = FusedStep(m, opt, None).step
        ddp(x, lab)["total_loss"].backward()  # eager DP warm-up: tiles, repack table, reducer hooks
        step()
        runs.append((m, ddp, opt, step))
    (m1, d1, o1, s1), (m2, d2, o2, s2) = runs
    o2.zero_grad(set_to_none=True)
    cap = T.CapturedTrainStep(m2, x, lab)
    assert cap.on_ready is not None and cap.on_end is not None
    res = {"rank": a.rank, "steps": 0, "segments": len(cap.plan),
           "reported": sum(len(r) for _, _, r in cap.plan), "nparams": len(list(m2.parameters()))}
    differs = False
    for it in range(3):
        o1.zero_grad(set_to_none=True)
        ref = d1(x, lab)
        ref["total_loss"].backward()
        got = cap(x, lab)
        torch.cuda.synchronize()
        for k in ("total_loss", "iou_loss", "conf_loss", "cls_loss", "num_fg"):
            assert float(got[k]) == float(ref[k]), (it, k, float(got[k]), float(ref[k]))
        p1, p2 = dict(m1.named_parameters()), dict(m2.named_parameters())
        for name in p1:
            assert torch.equal(p1[name].grad, p2[name].grad), (it, name)
        b1, b2 = dict(m1.named_buffers()), dict(m2.named_buffers())
        for name in b1:
            assert torch.equal(b1[name], b2[name]), (it, name)
        if it == 0:  # the gradients really are the mean over the ranks, not this rank's own
            flat = torch.cat([p.grad.flatten() for p in m2.parameters()]).cpu()
            other = [None] * a.world
            dist.all_gather_object(other, flat)
            differs = bool((other[0] - other[1]).abs().max() == 0)  # identical on both ranks after averaging
        s1()
        s2()
        res["steps"] = it + 1
    res["grads_equal_across_ranks"] = differs
    with open(a.out, "w") as f:
        json.dump(res, f)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
