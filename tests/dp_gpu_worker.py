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
    a = ap.parse_args()
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


if __name__ == "__main__":
    main()
