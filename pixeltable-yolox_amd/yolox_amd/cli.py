"""``yolox train`` (reference yolox/cli/train.py:19-143 + cli/utils.py) on the HIP path.

    python -m yolox_amd train -c yolox-s -d 8 -b 64 --fp16 [-o] [-D key=value ...]

Same flags and meaning as the reference: ``-c`` a named config (or ``module:Class``),
``-d`` processes = GPUs of this machine (one process per GPU, yolox_amd.launch), ``-b`` the
GLOBAL batch (each rank trains on b / d images), ``--fp16`` mixed precision through
autocast + GradScaler, ``-D`` config overrides.  Added: ``--max-iter`` (stop after that
many iterations) and ``--dataset-size`` (length of the synthetic COCO-shaped dataset that
stands in for COCO offline).  Loggers, checkpoint resume and evaluation are out of scope.
"""
from __future__ import annotations

import argparse
import importlib
import random
import sys
from typing import Optional

import torch

from .config import YoloxConfig
from .launch import launch


def resolve_config(config_str: str) -> YoloxConfig:
    """cli/utils.py:7-29."""
    config = YoloxConfig.get_named_config(config_str)
    if config is not None:
        return config
    config_class: Optional[type] = None
    classpath = config_str.split(":")
    if len(classpath) == 2:
        try:
            config_class = getattr(importlib.import_module(classpath[0]), classpath[1], None)
        except ImportError:
            pass
    if config_class is None:
        raise ValueError(f"Unknown config class: {config_str}")
    if not issubclass(config_class, YoloxConfig):
        raise ValueError(f"Invalid config class (does not extend `YoloxConfig`): {config_str}")
    return config_class()


def parse_model_config_opts(kv_opts) -> dict:
    """cli/utils.py:32-42."""
    kv = {}
    for item in kv_opts or []:
        if "=" not in item:
            raise ValueError(f"Invalid model configuration option (must be of the form OPT=VALUE): {item}")
        k, v = item.split("=", 1)
        kv[k] = v
    return kv


def make_parser() -> argparse.ArgumentParser:
    p = argparse.ArgumentParser("yolox train")
    p.add_argument("-c", "--config", type=str, help="a builtin config such as yolox_s, or module:Class")
    p.add_argument("-n", "--name", type=str, default=None)
    p.add_argument("--dist-backend", default="nccl", type=str, help="distributed backend (nccl = RCCL)")
    p.add_argument("--dist-url", default=None, type=str)
    p.add_argument("-b", "--batch-size", type=int, default=64, help="global batch size")
    p.add_argument("-d", "--devices", default=None, type=int, help="GPUs (processes) for training")
    p.add_argument("--resume", default=False, action="store_true")
    p.add_argument("--ckpt", default=None, type=str)
    p.add_argument("-e", "--start_epoch", default=None, type=int)
    p.add_argument("--num_machines", default=1, type=int)
    p.add_argument("--machine_rank", default=0, type=int)
    p.add_argument("--fp16", dest="fp16", default=False, action="store_true")
    p.add_argument("--cache", type=str, nargs="?", const="ram")
    p.add_argument("-o", "--occupy", dest="occupy", default=False, action="store_true")
    p.add_argument("-l", "--logger", type=str, default="tensorboard")
    p.add_argument("-D", type=str, metavar="OPT=VALUE", action="append")
    p.add_argument("--max-iter", dest="max_iter", type=int, default=None, help="stop after this many iterations")
    p.add_argument("--dataset-size", dest="dataset_size", type=int, default=118287)
    return p


def train(config: YoloxConfig, args) -> None:
    """cli/train.py:95-113."""
    if config.seed is not None:
        random.seed(config.seed)
        torch.manual_seed(config.seed)
    trainer = config.get_trainer(args)
    trainer.train()


def main(argv: list) -> None:
    """cli/train.py:116-143: resolve and validate the config, then one process per GPU."""
    args = make_parser().parse_args(argv)
    if args.config is None:
        raise AttributeError("Please specify a model configuration.")
    if args.resume or args.ckpt or args.cache:
        raise NotImplementedError("--resume / --ckpt / --cache: checkpoint files and dataset caches are out of scope")
    config = resolve_config(args.config)
    config.update(parse_model_config_opts(args.D))
    config.validate()
    if not args.name:
        args.name = config.name
    ngpu = torch.cuda.device_count()  # does not initialise the device on this image
    num_gpu = ngpu if args.devices is None else args.devices
    if args.dist_backend == "nccl":
        assert 0 < num_gpu <= ngpu, f"-d {num_gpu}: {ngpu} GPU(s) visible"
    launch(train, num_gpu, args.num_machines, args.machine_rank, backend=args.dist_backend,
           dist_url="auto" if args.dist_url is None else args.dist_url, args=(config, args))


def cli(argv=None) -> None:
    argv = sys.argv[1:] if argv is None else argv
    if not argv or argv[0] != "train":
        sys.exit("usage: python -m yolox_amd train -c <config> [-d N] [-b B] [--fp16] [-D k=v ...]")
    main(argv[1:])
