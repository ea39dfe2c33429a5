"""Process topology of ``yolox train -d N``: one process per GPU (reference
yolox/core/launch.py:37-145).

``launch`` spawns ``num_gpus_per_machine`` workers with ``mp.start_processes`` (start method
"spawn": the parent never touches the GPU, each child initialises its own device) and
calls ``main_func(*args)`` in each after ``init_process_group`` -- backend "nccl" is RCCL
over xGMI on ROCm; "gloo" runs the same topology on CPU (tests) or beside a GPU.  With one
process in the world ``main_func`` runs in place, as in the reference.
"""
from __future__ import annotations

import socket
from datetime import timedelta

import torch
import torch.distributed as dist
import torch.multiprocessing as mp

__all__ = ["launch", "get_rank", "get_world_size", "get_local_rank", "synchronize"]

DEFAULT_TIMEOUT = timedelta(minutes=30)
_LOCAL_RANK = 0


def _find_free_port() -> int:
    """launch.py:22-34 (bound on 127.0.0.1: the container hostname may not resolve)."""
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as sock:
        sock.bind(("127.0.0.1", 0))
        return sock.getsockname()[1]


def launch(main_func, num_gpus_per_machine: int, num_machines: int = 1, machine_rank: int = 0,
           backend: str = "nccl", dist_url=None, args=(), timeout=DEFAULT_TIMEOUT) -> None:
    """launch.py:37-96: ``main_func(*args)`` once per process of the world."""
    world_size = num_machines * num_gpus_per_machine
    if world_size > 1:
        if dist_url is None or dist_url == "auto":
            assert num_machines == 1, "dist_url=auto cannot work with distributed training."
            dist_url = f"tcp://127.0.0.1:{_find_free_port()}"
        mp.start_processes(_distributed_worker, nprocs=num_gpus_per_machine,
                           args=(main_func, world_size, num_gpus_per_machine, machine_rank, backend, dist_url, args,
                                 timeout),
                           daemon=False, start_method="spawn")
    else:
        main_func(*args)


def _distributed_worker(local_rank: int, main_func, world_size: int, num_gpus_per_machine: int, machine_rank: int,
                        backend: str, dist_url: str, args, timeout=DEFAULT_TIMEOUT) -> None:
    """launch.py:99-145: rank = machine_rank * gpus + local_rank; device = local_rank."""
    global _LOCAL_RANK
    if backend == "nccl":
        assert torch.cuda.is_available(), "cuda is not available. Please check your installation."
        assert num_gpus_per_machine <= torch.cuda.device_count()
    global_rank = machine_rank * num_gpus_per_machine + local_rank
    _LOCAL_RANK = local_rank
    if backend == "nccl":
        torch.cuda.set_device(local_rank)
        dist.init_process_group(backend=backend, init_method=dist_url, world_size=world_size, rank=global_rank,
                                timeout=timeout, device_id=torch.device("cuda", local_rank))
    else:
        dist.init_process_group(backend=backend, init_method=dist_url, world_size=world_size, rank=global_rank,
                                timeout=timeout)
    synchronize()
    try:
        main_func(*args)
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


def get_world_size() -> int:
    return dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1


def get_rank() -> int:
    return dist.get_rank() if dist.is_available() and dist.is_initialized() else 0


def get_local_rank() -> int:
    return _LOCAL_RANK if get_world_size() > 1 else 0


def synchronize() -> None:
    """utils/dist.py:73-84: barrier among all processes."""
    if get_world_size() > 1:
        dist.barrier()
