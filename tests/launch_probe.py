"""Rank body for tests/test_launch.py: the launch-path pieces a training rank runs before its
first GPU call (multiscale size broadcast, per-rank batch, rank-strided sampling)."""
import json
import os
import random


def probe(out_dir: str, batch_size: int, dataset_size: int) -> None:
    import torch

    from yolox_amd.config import named_config
    from yolox_amd.launch import get_local_rank, get_rank, get_world_size
    rank, world = get_rank(), get_world_size()
    random.seed(1000 + rank)  # different on every rank: only the broadcast makes sizes agree
    cfg = named_config("yolox_s")
    sizes = [cfg.random_resize(None, 0, rank, world > 1) for _ in range(3)]
    loader = cfg.get_data_loader(batch_size=batch_size, is_distributed=world > 1, dataset_size=dataset_size,
                                 device="cpu", distinct_images=4)
    batches = [loader.next_indices() for _ in range(2)]
    t = torch.tensor([[[1.0, 32.0, 16.0, 8.0, 4.0]]])
    cfg.input_size = (64, 64)
    # preprocess's label half (its image half is a HIP launch: tests/test_gpu_augment.py)
    t2 = cfg.scale_targets(t.clone(), (96, 128))
    with open(os.path.join(out_dir, f"rank{rank}.json"), "w") as f:
        json.dump({"rank": rank, "world": world, "local_rank": get_local_rank(), "sizes": sizes,
                   "batch": loader.batch_size, "len": len(loader), "batches": batches,
                   "pre_t": t2[0, 0].tolist()}, f)
