#!/usr/bin/env python3
"""Benchmark: YOLOX-s 640x640 bf16 forward + NMS images/sec (BASELINE.json metric,
configs[1]: batch 32 per GPU, synthetic uniform [0,255] images, seeded weights).

One step = one batch through the hot path: the captured hipGraph of the whole
forward (Focus -> CSPDarknet -> PAFPN -> decoupled head with fused decode, 53
kernels) followed by device post-processing (filter, sort, bitmask NMS) at the
processor defaults (conf 0.5, nms 0.65); the NMS filter pass (the one reader of the forward's
output) runs in stream order behind its forward and the rest of that batch's NMS on a side stream
beside the next batch's forward (yxh_postprocess_split; --nms-event: the whole NMS on the side
stream, the next forward waiting on the filter's event) -- --serial-nms runs them back to back on
one stream.  The filter reads the per-anchor score records the head launches write beside the rows
(32 bytes per anchor instead of 340; yxh_postprocess_scored, identical detections; --no-scores: the
rows' class columns).  Inputs are resident in HBM (uint8 NHWC, as the
processor's letterbox hands them to the forward) before the timed region.  With --gpus N (torchrun, one process per GPU) each rank
runs an independent replica -- inference has no exchange step, so there is no
collective in the data path -- and value = all images / max
rank time.

roofline: the forward's conv stack (conv_ws / conv_ws1 / conv_pwf / conv_r3h /
stem_rows / head_pred; every launch of one forward); one "launch" = one forward's conv stack, timed with HIP events on the plan's stream
around every replay inside the timed region; achieved = algorithmic conv FLOPs per
forward / mean forward duration, against the dense bf16 MFMA peak (2.5 PF).
traffic: HBM bytes per forward from a rocprofv3 --pmc pass (profiles/traffic_*.json,
FETCH_SIZE x2 + WRITE_SIZE per the MI355X guide), else null.
cpu_baseline: the oracle (PyTorch-CPU fp32 restatement + C NMS) on a bounded
sample, rank 0 only.
"""
from __future__ import annotations

import argparse
import glob
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "pixeltable-yolox_amd"))
sys.path.insert(0, REPO)

import numpy as np  # noqa: E402
import torch  # noqa: E402

METRIC = "images/sec (fwd+NMS) YOLOX-s 640×640 bf16 @1/2/4/8 MI355X; box mAP parity"  # BASELINE.json
PEAK_BF16_TFLOPS = 2500.0  # dense MFMA bf16/fp16, MI355X_MICROARCH.md
PEAK_F32_TFLOPS = 157.3    # dense MFMA fp32 (v_mfma_f32_16x16x4_f32)
PEAK_HBM_GBS = 8000.0

# BASELINE.json configs this bench reproduces: index -> (workload, model, size, dtype, batch per GPU)
CONFIGS = {
    1: ("infer", "yolox_s", 640, "bf16", 32),
    2: ("train", "yolox_s", 640, "fp32", 8),   # -d 8 -b 64, no --fp16 (cli/train.py:56-58)
    3: ("infer", "yolox_l", 640, "fp16", 16),
    4: ("train", "yolox_x", 1280, "fp16", 8),  # -d 8 --fp16, default batch 64 -> 8 per GPU
}


def config_index(args):
    for i, c in CONFIGS.items():
        if c == (args.workload, args.model, args.size, args.dtype, args.batch):
            return i
    return None


def metric_name(args) -> str:
    idx = config_index(args)
    if idx == 1:
        return METRIC
    what = "fwd+NMS" if args.workload == "infer" else "train step"
    tag = f" (BASELINE configs[{idx}])" if idx is not None else " (not a BASELINE config)"
    return f"images/sec ({what}) {args.model} {args.size}x{args.size} {args.dtype} batch {args.batch}/GPU MI355X{tag}"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # 100 timed steps (~0.17 s of the default workload): the 20-step window read 0.8-1.6 % low on one
    # box (clock ramp; profiles/r05/bench_r5p_*.json)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--model", default="yolox_s")
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--chunk", type=int, default=0, help="images per pass of the op list (0 = whole batch)")
    ap.add_argument("--par-chunks", action="store_true",
                    help="with --chunk: chunks on arenas of their own, side by side in the captured graph")
    ap.add_argument("--size", type=int, default=640)
    ap.add_argument("--dtype", default=None, choices=["bf16", "fp16", "fp32"],
                    help="compute dtype (default: bf16 for infer = configs[1]; fp32 for train = configs[2], "
                         "the reference's precision without --fp16)")
    ap.add_argument("--conf", type=float, default=0.5)
    ap.add_argument("--nms", type=float, default=0.65)
    ap.add_argument("--cpu-seconds", type=float, default=15.0, help="budget of the CPU baseline sample")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--fwd-priority", action="store_true",
                    help="run the forward on a high-priority stream (the NMS side stream stays normal)")
    ap.add_argument("--two-slot", action="store_true",
                    help="two output slots (two captured graphs): a forward never waits for the previous batch's "
                         "NMS filter; measured slower (the NMS then overlaps the next forward's first layers)")
    ap.add_argument("--serial-nms", action="store_true",
                    help="NMS behind each forward on one stream (default: beside the next batch's forward)")
    ap.add_argument("--nms-event", action="store_true",
                    help="the whole NMS on the side stream, the next forward waiting on its filter event across "
                         "streams (round 4-5 form; default: the filter in order behind the forward on its stream, "
                         "the rest of the NMS on the side stream, yxh_postprocess_split)")
    ap.add_argument("--no-scores", action="store_true",
                    help="the NMS filter reads the rows' class columns (default: the per-anchor score records the head "
                         "launches write beside the rows, Plan.enable_scores / yxh_postprocess_scored)")
    ap.add_argument("--dry-run", action="store_true",
                    help="exercise only the process topology (spawn, rendezvous, barrier, max over ranks) "
                         "with gloo on the CPU; prints one JSON line from rank 0")
    ap.add_argument("--refine-tiles", action="store_true",
                    help="after the per-op autotune, re-time close runner-up tiles inside the captured forward")
    ap.add_argument("--layers", action="store_true", help="print a per-op time/roofline table to stderr")
    ap.add_argument("--tune-file", default="", help="JSON tile choices: loaded if present (skips tuning), else written")
    ap.add_argument("--workload", default="infer", choices=["infer", "train"],
                    help="infer: BASELINE configs[1] (default); train: configs[2] train step (8 images / GPU)")
    args = ap.parse_args()
    if args.workload == "train" and args.batch == 32:
        args.batch = 8  # -b 64 over -d 8 (config.py:249-250)
    if args.dtype is None:
        args.dtype = "fp32" if args.workload == "train" else "bf16"
    return args


def spawn_ranks(args) -> int:
    """`bench.py --gpus N` without a launcher: start N fresh processes, one per GPU, under
    torch.distributed.run (the reference's launch.py:57-94 creates its own process
    topology the same way: mp.start_processes, one worker per GPU).  Nothing here has
    touched the GPU (device_count does not initialise it on this image), and the ranks
    are children -- this process only waits and forwards their exit status."""
    import socket
    import subprocess
    if _BACKEND != "gloo" and torch.cuda.device_count() < args.gpus:
        sys.exit(f"--gpus {args.gpus}: only {torch.cuda.device_count()} GPU(s) visible")
    with socket.socket() as sk:  # launch.py:22-34 _find_free_port
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


# "nccl" (RCCL over xGMI, one rank per GPU) for real runs; "gloo" only to rehearse the
# multi-rank code path with several ranks sharing one GPU (numbers then meaningless)
_BACKEND = os.environ.get("YOLOX_AMD_BENCH_BACKEND", "nccl")


def dist_setup(args):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.dry_run:
        if world > 1:
            import torch.distributed as dist
            dist.init_process_group("gloo")
        return world, rank, local
    if world > 1:
        import torch.distributed as dist
        if _BACKEND == "gloo":  # rehearsal of the N>1 path on a box with fewer GPUs than ranks
            local = local % torch.cuda.device_count()
            torch.cuda.set_device(local)
            dist.init_process_group("gloo")
        else:
            torch.cuda.set_device(local)
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(0)
    return world, rank, local


def barrier(world):
    if world > 1:
        import torch.distributed as dist
        dist.barrier()


def max_over_ranks(x: float, world: int) -> float:
    if world == 1:
        return x
    import torch.distributed as dist
    t = torch.tensor([x], dtype=torch.float64, device="cpu" if _BACKEND == "gloo" else "cuda")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def load_traffic(model, batch, size, dtype, workload="infer"):
    """The latest committed PMC traffic record (profiles/traffic_*.json, by file name) of this
    workload: tools/traffic.py (forward) or tools/traffic_train.py (training step)."""
    best = None
    for path in sorted(glob.glob(os.path.join(REPO, "profiles", "traffic_*.json"))):
        try:
            d = json.load(open(path))
        except Exception:
            continue
        if (d.get("workload", "infer"), d.get("model"), d.get("batch"), d.get("size"), d.get("dtype")) == \
                (workload, model, batch, size, dtype):
            best = d
    return best


def layer_table(plan, iters=5):
    """Per-op HIP-event timing of the eager op list (diagnostic; stderr)."""
    from yolox_amd import _native as N
    lib = N.lib()
    st = torch.cuda.current_stream()
    n = plan._nops
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(n + 1)]
    tot = np.zeros(n)
    for _ in range(iters):
        ev[0].record(st)
        for i in range(n):
            N.check(lib.yxh_run_ops(C_op(plan, i), 1, st.cuda_stream))
            ev[i + 1].record(st)
        torch.cuda.synchronize()
        tot += [ev[i].elapsed_time(ev[i + 1]) for i in range(n)]
    tot /= iters
    rows = []
    for i, rec in enumerate(plan.ctx.ops):
        a = rec.args
        if rec.kind == N.OP_CONV:
            flop = 2.0 * plan.chunk * a["out_h"] * a["out_w"] * a["cout"] * a["k"] * a["k"] * (
                a["cin"] // a["groups"] if a["groups"] > 1 else a["cin"])
            if a["groups"] > 1:
                flop = 2.0 * plan.chunk * a["out_h"] * a["out_w"] * a["cout"] * a["k"] * a["k"]
            es = plan.ctx.esize
            byt = plan.chunk * (a["in_h"] * a["in_w"] * a["cin"] // (1 if not a["srcs"][0].up else 4)
                                + a["out_h"] * a["out_w"] * a["cout"] * (4 if a["dst_f32"] else 1)) * es
            rows.append((i, f"conv k{a['k']}s{a['stride']} {a['cin']}->{a['cout']} @{a['out_h']}x{a['out_w']}",
                         tot[i], flop / tot[i] / 1e9, byt / tot[i] / 1e6))
        else:
            rows.append((i, {N.OP_FOCUS: "focus", N.OP_SPP: "spp", N.OP_STEM: "stem (focus+conv)",
                             N.OP_STEM2: "stem + dark2.0 (fused, stem_s2)",
                             N.OP_HEAD: f"head preds+decode @{a.get('h')}x{a.get('w')}"}[rec.kind], tot[i],
                         0.0, 0.0))
    print(f"{'op':>3} {'layer':<40} {'ms':>8} {'TFLOP/s':>9} {'GB/s':>8}", file=sys.stderr)
    for r in rows:
        print(f"{r[0]:>3} {r[1]:<40} {r[2]:8.4f} {r[3]:9.1f} {r[4]:8.0f}", file=sys.stderr)
    print(f"total {tot.sum():.3f} ms", file=sys.stderr)


def C_op(plan, i):
    import ctypes
    from yolox_amd import _native as N
    return ctypes.cast(ctypes.addressof(plan._ops) + i * ctypes.sizeof(N.Op), ctypes.POINTER(N.Op))


def cpu_baseline(args, budget_s):
    """Oracle forward (fp32, torch CPU) + oracle NMS on 640x640 images."""
    import subprocess
    from oracle import reference_cpu as O
    from yolox_amd.weights import synthetic_images, synthetic_state_dict
    from yolox_amd.config import named_config

    lib = os.path.join(REPO, "oracle", "_build", "liboracle.so")
    if not os.path.exists(lib):
        subprocess.run(["make", "-C", os.path.join(REPO, "oracle")], check=True, stdout=subprocess.DEVNULL)
    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or min(16, os.cpu_count() or 1)
    torch.set_num_threads(threads)
    cfg = named_config(args.model)
    sd = synthetic_state_dict(cfg.get_model().state_dict(), seed=0, bn_stats=cfg.name)
    arch = O.ARCHS[args.model]
    bs = 2
    x = torch.from_numpy(O.letterbox_identity(synthetic_images(bs, args.size, args.size, seed=0)))
    out = O.forward_eval(sd, arch, x)  # warm-up
    n_img, t0 = 0, time.perf_counter()
    while True:
        out = O.forward_eval(sd, arch, x)
        O.postprocess(out.numpy().copy(), 80, args.conf, args.nms)
        n_img += bs
        if time.perf_counter() - t0 > budget_s:
            break
    dt = time.perf_counter() - t0
    return {"value": round(n_img / dt, 3), "unit": "images/s", "cores": threads, "kind": "port",
            "sample": f"{n_img} images ({args.model} {args.size}x{args.size}, batch {bs}, fp32 PyTorch-CPU "
                      f"oracle forward + C oracle NMS conf {args.conf}) in {dt:.1f}s"}


def cpu_baseline_train(args, budget_s):
    """Oracle training step (fp32 PyTorch-CPU forward + SimOTA + losses + autograd)."""
    from oracle import reference_cpu as O
    from yolox_amd.config import named_config
    from yolox_amd.weights import synthetic_images, synthetic_labels, synthetic_state_dict

    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or min(16, os.cpu_count() or 1)
    torch.set_num_threads(threads)
    cfg = named_config(args.model)
    sd = synthetic_state_dict(cfg.get_model().state_dict(), seed=0, bn_stats=cfg.name)
    sd = {k: v.float().requires_grad_(v.is_floating_point() and "running" not in k and "num_batches" not in k)
          for k, v in sd.items()}
    arch = O.ARCHS[args.model]
    bs = 2
    x = torch.from_numpy(O.letterbox_identity(synthetic_images(bs, args.size, args.size, seed=0)))
    lab = torch.from_numpy(synthetic_labels(bs, args.size, args.size, seed=0))
    n_img, t0 = 0, time.perf_counter()
    while True:
        O.forward_train(sd, arch, x, lab)["total_loss"].backward()
        n_img += bs
        if time.perf_counter() - t0 > budget_s:
            break
    dt = time.perf_counter() - t0
    return {"value": round(n_img / dt, 3), "unit": "images/s", "cores": threads, "kind": "port",
            "sample": f"{n_img} images ({args.model} {args.size}x{args.size}, batch {bs}, fp32 PyTorch-CPU oracle "
                      f"train forward + SimOTA + losses + autograd backward) in {dt:.1f}s"}


def main_train(args, world, rank):
    """BASELINE configs[2]: yolox_s 640 train step, per-GPU batch 8, synthetic COCO-shaped
    targets, data parallel over RCCL (bucketed all-reduce overlapped with the HIP reverse
    pass), SGD nesterov + EMA like Trainer.train_one_iter."""
    from yolox_amd.dp import DistributedDataParallel
    from yolox_amd.models import YoloxModule
    from yolox_amd.trainer import ModelEMA, get_optimizer, train_one_iter
    from yolox_amd.weights import synthetic_images, synthetic_labels

    dev = torch.device("cuda", torch.cuda.current_device())
    amp = {"bf16": torch.bfloat16, "fp16": torch.float16, "fp32": None}[args.dtype]
    model = YoloxModule.synthetic(args.model, seed=0, device=dev)
    model.train()
    B, S = args.batch, args.size
    net = DistributedDataParallel(model) if world > 1 else model
    opt = get_optimizer(model, lr=0.01 / 64 * B * world)
    scaler = torch.amp.GradScaler("cuda") if args.dtype == "fp16" else None
    ema = ModelEMA(model, 0.9998)
    imgs = torch.from_numpy(synthetic_images(B, S, S, seed=1000 + rank)).to(dev).permute(0, 3, 1, 2).float()
    if amp is not None:
        imgs = imgs.to(amp)  # trainer.py:100 (inps.to(data_type) under --fp16)
    labels = torch.from_numpy(synthetic_labels(B, S, S, seed=2000 + rank)).to(dev)

    from yolox_amd.optim import FusedStep
    fused = FusedStep(model, opt, ema)  # SGD + EMA (+ GradScaler under fp16) on the device

    cap = None

    def step():
        return train_one_iter(net, opt, imgs, labels, amp_dtype=amp, scaler=scaler, ema=ema, fused=fused,
                              captured=cap)

    for _ in range(args.warmup):
        out = step()
    # the forward + reverse pass replays as hipGraph segments (under DDP the reducer's bucket all-reduces
    # are issued between the replayed segments, CapturedTrainStep); YOLOX_AMD_TRAIN_GRAPH=0: the eager
    # step.  Default since round 6: on the GPU boxes of that round the eager step's host issue (16.5-17 ms
    # per configs[2] step) outran the GPU, captured 534 vs eager 467-475 img/s (configs[4]: 105.6 vs 98.2)
    if args.warmup >= 1 and os.environ.get("YOLOX_AMD_TRAIN_GRAPH", "1") == "1":
        from yolox_amd.train import CapturedTrainStep
        opt.zero_grad(set_to_none=True)
        cap = CapturedTrainStep(model, imgs, labels, dtype=amp or torch.float32,
                                grad_scale=scaler._scale if scaler is not None else None)
        out = step()
    torch.cuda.synchronize()
    stream = torch.cuda.current_stream(dev)
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    barrier(world)
    torch.cuda.synchronize()
    # diagnostic (BENCH_HOST_PROFILE=<file>): cProfile of the host side of the timed steps, for the eager
    # step's issue path (configs[2] is host-issue-bound); the timed numbers of such a run are not reported
    prof = None
    if os.environ.get("BENCH_HOST_PROFILE") and rank == 0:
        import cProfile
        prof = cProfile.Profile()
        prof.enable()
    t0 = time.perf_counter()
    host_s = 0.0  # time the host spends issuing a step (ctypes launches + tensor bookkeeping)
    for k in range(args.steps):
        evs[k][0].record(stream)
        h0 = time.perf_counter()
        out = step()
        host_s += time.perf_counter() - h0
        evs[k][1].record(stream)
    if prof is not None:
        prof.disable()
        prof.dump_stats(os.environ["BENCH_HOST_PROFILE"])
    torch.cuda.synchronize()
    barrier(world)
    dt = time.perf_counter() - t0
    dt_max = max_over_ranks(dt, world)
    gpu_ms = float(np.mean([a.elapsed_time(b) for a, b in evs]))
    loss = float(out["total_loss"].detach())
    from yolox_amd import train as _T
    if _T._LAUNCH_LOG is not None and rank == 0:  # diagnostic: conv / wgrad launches of every step
        with open(os.environ["YOLOX_AMD_TRAIN_LOG"], "w") as f:
            json.dump({"steps": args.warmup + args.steps, "launches": _T._LAUNCH_LOG}, f)
    if rank != 0:
        if world > 1:
            import torch.distributed as dist
            dist.destroy_process_group()
        return
    flops_fwd = _fwd_flops(model, B, S)
    flops = 3.0 * flops_fwd  # forward + data gradient + weight gradient of every conv
    achieved = flops / (gpu_ms * 1e-3) / 1e12
    peak = PEAK_BF16_TFLOPS if amp is not None else PEAK_F32_TFLOPS
    idx = config_index(args)
    ttr = load_traffic(args.model, B, S, args.dtype, workload="train")
    result = {
        "metric": metric_name(args),
        "value": round(world * B * args.steps / dt_max, 2),
        "unit": "images/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(dt_max / args.steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": args.dtype,
        "data": "synthetic uniform [0,255] images + COCO-shaped random targets (G ~ U{1..50}), seeded weights",
        "config": {"workload": f"{args.model} {S}x{S} {args.dtype} train step (fwd + SimOTA/losses + bwd + "
                               f"DP all-reduce + SGD + EMA), batch {B}/GPU"
                               + (f" (BASELINE configs[{idx}])" if idx is not None else " (not a BASELINE config)"),
                   "baseline_config_index": idx,
                   "batch_per_gpu": B, "global_batch": B * world, "image_size": S,
                   "parallelism": f"dp{world} (bucketed RCCL all-reduce overlapped with the reverse pass)",
                   "issue": "hipGraph replay" if cap is not None else "eager"},
        "roofline": {"kernel": "whole step (conv fwd/dgrad/wgrad dominate; HIP events around each step)",
                     "bound": "mfma", "achieved": round(achieved, 2), "peak": peak, "unit": "TFLOP/s",
                     "frac": round(achieved / peak, 4),
                     "traffic": None if ttr is None else ttr["hbm_bytes_per_step"],
                     "algorithmic_flops_per_launch": flops, "step_gpu_ms": round(gpu_ms, 3)},
        "last_loss": round(loss, 4),
        **({"traffic_source": ttr.get("source")} if ttr is not None else {}),
        "host_issue_ms_per_step": round(host_s / args.steps * 1e3, 3),
    }
    if not args.no_cpu_baseline and world == 1:
        result["cpu_baseline"] = cpu_baseline_train(args, args.cpu_seconds)
    else:
        result["cpu_baseline"] = None
    print(json.dumps(result))
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


def _fwd_flops(model, B, S) -> float:
    """Algorithmic conv FLOPs of one forward (the planner's count, no device work)."""
    from yolox_amd.engine import PlanCtx
    ctx = PlanCtx(B, torch.float32, torch.device("cpu"))
    feats = model.backbone.plan(ctx, ctx.image(S, S))
    from yolox_amd.engine import OutBuffer
    model.head.plan(ctx, feats, OutBuffer(sum(f.lh * f.lw for f in feats), 5 + model.head.num_classes))
    return ctx.flops


def main_dry_run(args, world, rank, local):
    """The launch/timing skeleton of main() without device work (CPU test of --gpus N)."""
    ranks = [(rank, local, os.getpid())]
    if world > 1:
        import torch.distributed as dist
        ranks = [None] * world
        dist.all_gather_object(ranks, (rank, local, os.getpid()))
    t0 = time.perf_counter()
    barrier(world)
    dt_max = max_over_ranks(time.perf_counter() - t0 + 0.001 * rank, world)
    if rank == 0:
        print(json.dumps({"metric": metric_name(args), "n_gpus": world, "dry_run": True, "ranks": ranks,
                          "max_rank_seconds": dt_max}))
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(args))
    world, rank, local = dist_setup(args)
    if world != args.gpus and rank == 0:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE={world}; reporting n_gpus={world}", file=sys.stderr)
    if args.dry_run:
        return main_dry_run(args, world, rank, local)
    if args.workload == "train":
        return main_train(args, world, rank)
    from yolox_amd import _native as N
    from yolox_amd.models import YoloxModule
    from yolox_amd.utils.boxes import postprocess_device
    from yolox_amd.weights import synthetic_images

    dtype = {"bf16": torch.bfloat16, "fp16": torch.float16, "fp32": torch.float32}[args.dtype]
    dev = torch.device("cuda", torch.cuda.current_device())
    model = YoloxModule.synthetic(args.model, seed=0, device=dev, dtype=dtype)
    B, S = args.batch, args.size
    # input: letterboxed uint8 NHWC images resident in HBM -- the form YoloxProcessor's
    # letterbox_batch hands Yolox.__call__'s forward (forward_nhwc)
    plan = model.plan_for(B, S, S, N.NHWC, torch.uint8, chunk=args.chunk or None, parallel_chunks=args.par_chunks)
    imgs = torch.from_numpy(synthetic_images(B, S, S, seed=1000 + rank)).to(dev)
    plan.static_input().copy_(imgs)
    from yolox_amd import engine
    if args.tune_file and os.path.exists(args.tune_file):
        engine.load_tune_cache(args.tune_file)
    t_tune = time.perf_counter()
    plan.autotune(verbose=args.layers and rank == 0)
    if args.refine_tiles:  # second pass: runner-up tiles timed inside the captured forward
        changed = plan.refine_in_graph(verbose=args.layers and rank == 0)
        if rank == 0:
            for (old, new, ma, mb) in changed.values():
                print(f"refine: tile {old >> 1}/{(old & 1) + 1} -> {new >> 1}/{(new & 1) + 1}: forward "
                      f"{ma * 1e3:.1f} -> {mb * 1e3:.1f} us", file=sys.stderr)
    t_tune = time.perf_counter() - t_tune
    if args.tune_file and rank == 0 and not os.path.exists(args.tune_file):
        engine.save_tune_cache(args.tune_file)
    # Serving pipeline: the NMS of batch k runs on a side stream beside the forward of batch
    # k+1, which waits only for batch k's filter pass (the one reader of the forward's output rows,
    # event recorded by yxh_postprocess_ev); detections are double-buffered.  --two-slot also
    # double-buffers the output rows (Plan.capture(slots=2)) so no forward waits at all: on MI355X
    # that measured slower (18 147-18 302 vs 18 508-18 577 img/s, profiles/r05/output_slots_ab.txt) --
    # the NMS kernels then run beside the next forward's stem and stretch it more than the wait
    # costs.  --serial-nms puts the NMS back behind each forward on one stream.
    slots = 2 if args.two_slot and not args.serial_nms else 1
    # the head launches also write 16-byte score records per anchor, which the NMS filter reads
    # instead of the 85 fp32 columns of every row (identical detections; tests/test_gpu_postprocess.py)
    scores = None if args.no_scores or slots == 2 else plan.enable_scores()
    plan.capture(slots)
    A = plan.anchors
    # --fwd-priority: the forward on a high-priority stream, so the NMS kernels of the previous batch
    # (side stream, normal priority) fill gaps instead of taking CUs from the forward
    stream = torch.cuda.Stream(dev, priority=-1) if args.fwd_priority else torch.cuda.current_stream(dev)
    side = torch.cuda.Stream(dev) if not args.serial_nms else stream
    dets = [torch.empty(B, A, 7, dtype=torch.float32, device=dev) for _ in range(2)]
    cnts = [torch.empty(B, dtype=torch.int32, device=dev) for _ in range(2)]
    filt = [torch.cuda.Event() for _ in range(2)]
    fwd_done = torch.cuda.Event()
    state = {"k": 0}
    det, counts = dets[0], cnts[0]

    def step(ev0=None, ev1=None):
        nonlocal det, counts
        k = state["k"]
        if not args.serial_nms and k >= slots:
            stream.wait_event(filt[(k - slots) % 2])  # the filter of the last batch in this output slot
        if ev0 is not None:
            ev0.record(stream)
        with torch.cuda.stream(stream):
            out = plan.replay(k % slots)
        if ev1 is not None:
            ev1.record(stream)
        det, counts = dets[k % 2], cnts[k % 2]
        if args.serial_nms:
            with torch.cuda.stream(stream):
                postprocess_device(out, model.head.num_classes, args.conf, args.nms, det=det, counts=counts,
                                   scores=scores)
        elif args.nms_event:
            fwd_done.record(stream)
            side.wait_event(fwd_done)
            with torch.cuda.stream(side):
                postprocess_device(out, model.head.num_classes, args.conf, args.nms, det=det, counts=counts,
                                   filter_done=filt[k % 2], scores=scores)
        else:  # filter in stream order behind the forward, sort / mask / reduce beside the next forward
            with torch.cuda.stream(stream):
                postprocess_device(out, model.head.num_classes, args.conf, args.nms, det=det, counts=counts,
                                   filter_done=filt[k % 2], rest_stream=side, scores=scores)
        state["k"] = k + 1

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if args.layers and rank == 0:
        layer_table(plan)
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    barrier(world)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(args.steps):
        step(*evs[k])
    torch.cuda.synchronize()
    barrier(world)
    dt = time.perf_counter() - t0
    dt_max = max_over_ranks(dt, world)
    fwd_ms = float(np.mean([a.elapsed_time(b) for a, b in evs]))
    n_det = counts.cpu().tolist()

    if rank != 0:
        if world > 1:
            import torch.distributed as dist
            dist.destroy_process_group()
        return
    imgs_total = world * B * args.steps
    value = imgs_total / dt_max
    flops = plan.flops  # algorithmic conv FLOPs of one forward (all images of the batch)
    achieved = flops / (fwd_ms * 1e-3) / 1e12
    traffic = load_traffic(args.model, B, S, args.dtype)
    idx = config_index(args)
    result = {
        "metric": metric_name(args),
        "value": round(value, 2),
        "unit": "images/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(dt_max / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": args.dtype,
        "data": "synthetic uniform [0,255] images, seeded weights with calibrated BN (no checkpoints offline)",
        "config": {
            "workload": f"{args.model} {S}x{S} {args.dtype} batch={B}/GPU inference: forward (hipGraph) + "
                        f"device NMS conf={args.conf} nms={args.nms}"
                        + (f" (BASELINE configs[{idx}])" if idx is not None else " (not a BASELINE config)"),
            "baseline_config_index": idx,
            "batch_per_gpu": B, "global_batch": B * world, "image_size": S,
            "parallelism": f"replicas x{world} (no data-path collective)",
            "input": "uint8 NHWC letterboxed images resident in HBM",
            "chunk": plan.chunk,
            "parallel_chunks": plan.parallel_chunks,
            "graph": plan.graph_mode,
            "output_slots": slots,
            "nms_streams": "serial" if args.serial_nms else ("event" if args.nms_event else "split"),
            "nms_filter": "score records" if scores is not None else "rows",
        },
        "roofline": {
            "kernel": "the forward conv stack (conv_ws / conv_ws1 / conv_r3h / conv_pwf / stem_rows / head_pred: every launch of one forward; HIP events on the plan stream around each graph replay)",
            "bound": "mfma",
            "achieved": round(achieved, 2),
            "peak": PEAK_BF16_TFLOPS if args.dtype != "fp32" else PEAK_F32_TFLOPS,
            "unit": "TFLOP/s",
            "frac": round(achieved / (PEAK_BF16_TFLOPS if args.dtype != "fp32" else PEAK_F32_TFLOPS), 4),
            "traffic": None if traffic is None else traffic["hbm_bytes_per_forward"],
            "algorithmic_flops_per_launch": flops,
            "forward_ms": round(fwd_ms, 4),
        },
        "detections_per_image_last_step": n_det[:4],
        "autotune_s": round(t_tune, 2),
    }
    if traffic is not None:
        result["roofline"]["traffic_source"] = traffic.get("source")
    if not args.no_cpu_baseline and world == 1:
        result["cpu_baseline"] = cpu_baseline(args, args.cpu_seconds)
    else:
        result["cpu_baseline"] = None
    print(json.dumps(result))
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
