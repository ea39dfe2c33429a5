"""bench.py --gpus N creates its own N ranks (reference yolox/core/launch.py:57-94) when
no launcher did, and labels each line with the BASELINE config it measures.  Runs the
topology-only dry run on the CPU with gloo at world size 2."""
import json
import os
import subprocess
import sys

from conftest import REPO


def run_bench(*args, env_extra=None):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["YOLOX_AMD_BENCH_BACKEND"] = "gloo"
    env.update(env_extra or {})
    p = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), *args], capture_output=True, text=True,
                       env=env, timeout=300)
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout
    return json.loads(lines[0])


def test_gpus_2_spawns_two_ranks():
    out = run_bench("--gpus", "2", "--dry-run")
    assert out["n_gpus"] == 2
    ranks = sorted(r[0] for r in out["ranks"])
    assert ranks == [0, 1]
    assert len({r[2] for r in out["ranks"]}) == 2  # two processes
    assert sorted(r[1] for r in out["ranks"]) == [0, 1]  # one local rank (GPU) each
    assert out["max_rank_seconds"] >= 0.001  # max over ranks, not rank 0's own time


def test_single_gpu_default_is_configs_1():
    out = run_bench("--dry-run")
    assert out["n_gpus"] == 1
    with open(os.path.join(REPO, "BASELINE.json")) as f:
        assert out["metric"] == json.load(f)["metric"]


def test_metric_labels_name_the_config():
    assert "configs[3]" in run_bench("--dry-run", "--model", "yolox_l", "--dtype", "fp16", "--batch", "16")["metric"]
    m = run_bench("--dry-run", "--workload", "train")["metric"]
    assert "configs[2]" in m and "fp32" in m and "yolox_s" in m  # reference precision by default
    m = run_bench("--dry-run", "--workload", "train", "--dtype", "bf16")["metric"]
    assert "not a BASELINE config" in m
    m = run_bench("--dry-run", "--workload", "train", "--model", "yolox_x", "--size", "1280", "--dtype", "fp16")["metric"]
    assert "configs[4]" in m
