"""`yolox train -d N` process topology on CPU (gloo, world 2): yolox_amd.launch spawns the
ranks (reference core/launch.py:37-145), rank 0's multiscale draw is broadcast
(config.py:275-294), each rank trains on batch / world images from its rank-strided slice
of one shuffled stream (config.py:249-250, samplers.py:28-82), config.preprocess resizes
(config.py:296-305); the CLI parses the reference's flags; yoloxwarmcos matches the
reference formula at its breakpoints."""
import json
import math
import os

import pytest
import torch

from launch_probe import probe


def test_launch_world2_broadcast_and_rank_batches(tmp_path):
    from yolox_amd.launch import launch
    launch(probe, 2, backend="gloo", dist_url="auto", args=(str(tmp_path), 16, 50))
    r = [json.load(open(tmp_path / f"rank{i}.json")) for i in range(2)]
    assert [x["rank"] for x in r] == [0, 1] and all(x["world"] == 2 for x in r)
    assert [x["local_rank"] for x in r] == [0, 1]
    assert r[0]["sizes"] == r[1]["sizes"]
    for h, w in r[0]["sizes"]:
        assert h == w and h % 32 == 0 and 640 - 5 * 32 <= h <= 640 + 5 * 32
    assert r[0]["batch"] == r[1]["batch"] == 8  # -b 16 over 2 ranks
    assert r[0]["len"] == math.ceil((50 // 2) / 8)
    g = torch.Generator()
    g.manual_seed(0)
    stream = torch.randperm(50, generator=g).tolist()
    for k in range(2):
        assert r[0]["batches"][k] == stream[0::2][8 * k:8 * k + 8]
        assert r[1]["batches"][k] == stream[1::2][8 * k:8 * k + 8]
    assert not set(sum(r[0]["batches"], [])) & set(sum(r[1]["batches"], []))
    assert r[0]["pre_t"] == [1.0, 64.0, 24.0, 16.0, 6.0]  # x cols * 2, y cols * 1.5


def test_launch_single_process_runs_in_place(tmp_path):
    from yolox_amd.launch import launch
    launch(probe, 1, backend="gloo", args=(str(tmp_path), 8, 20))
    r = json.load(open(tmp_path / "rank0.json"))
    assert r["world"] == 1 and r["batch"] == 8 and len(r["sizes"]) == 3


def test_cli_parses_reference_flags():
    from yolox_amd.cli import make_parser, parse_model_config_opts, resolve_config
    a = make_parser().parse_args(["-c", "yolox-s", "-d", "8", "-b", "64", "--fp16", "-o", "-D", "max_epoch=3",
                                  "-D", "input_size=(320,320)"])
    assert (a.config, a.devices, a.batch_size, a.fp16, a.occupy) == ("yolox-s", 8, 64, True, True)
    cfg = resolve_config(a.config)
    cfg.update(parse_model_config_opts(a.D))
    assert cfg.name == "yolox_s" and cfg.max_epoch == 3 and tuple(cfg.input_size) == (320, 320)
    with pytest.raises(ValueError):
        resolve_config("nope")
    with pytest.raises(ValueError):
        parse_model_config_opts(["novalue"])


def test_yoloxwarmcos_breakpoints():
    from yolox_amd.config import named_config
    cfg = named_config("yolox_s")
    s = cfg.get_lr_scheduler(0.01, 100)  # 300 epochs x 100 iters, warm-up 5 epochs, no-aug 15
    assert s.update_lr(0) == 0.0
    assert s.update_lr(250) == pytest.approx(0.01 * 0.25)  # quadratic warm-up
    assert s.update_lr(500) == pytest.approx(0.01)
    assert s.update_lr(30000 - 1500) == pytest.approx(0.01 * 0.05)
    mid = 500 + (30000 - 500 - 1500) // 2
    assert s.update_lr(mid) == pytest.approx(0.0005 + 0.5 * 0.0095 * (1 + math.cos(math.pi * 0.5)), rel=1e-6)
