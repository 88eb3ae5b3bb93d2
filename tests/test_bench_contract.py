"""The driver's bench.py contract (one JSON line with the documented fields) on the CPU plumbing path,
single rank and a 2-rank gloo run under torch.distributed.run."""
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KEYS = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
        "vs_baseline", "dtype", "data", "config"}


def _json_lines(out: str):
    return [json.loads(l) for l in out.splitlines() if l.startswith("{")]


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.timeout(300)
def test_bench_single_rank_json_line():
    env = dict(os.environ, PYTHONPATH=ROOT)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK"):
        env.pop(k, None)
    p = subprocess.run([sys.executable, "bench.py", "--model", "mlp_mnist", "--batch-per-gpu", "64", "--steps", "3",
                        "--warmup", "1"], cwd=ROOT, env=env, capture_output=True, text=True, timeout=280)
    assert p.returncode == 0, p.stderr[-2000:]
    lines = _json_lines(p.stdout)
    assert len(lines) == 1
    d = lines[0]
    assert KEYS <= set(d)
    assert d["n_gpus"] == 1 and d["steps"] == 3 and d["warmup"] == 1 and d["higher_is_better"] is True
    assert d["value"] > 0 and d["scaling"] == "weak"
    assert {"model", "global_batch", "per_gpu_batch", "parallelism"} <= set(d["config"])


@pytest.mark.timeout(300)
def test_bench_two_rank_gloo_json_line():
    env = dict(os.environ, PYTHONPATH=ROOT)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK"):
        env.pop(k, None)
    p = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", str(_port()), "bench.py", "--gpus", "2",
                        "--model", "mlp_mnist", "--batch-per-gpu", "64", "--steps", "3", "--warmup", "1"],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=280)
    assert p.returncode == 0, p.stderr[-2000:]
    lines = _json_lines(p.stdout)
    assert len(lines) == 1  # rank 0 only
    d = lines[0]
    assert d["n_gpus"] == 2 and d["config"]["global_batch"] == 128 and d["config"]["parallelism"] == "dp2"


@pytest.mark.timeout(300)
def test_bench_self_spawns_ranks_without_torchrun():
    """``bench.py --gpus N`` with WORLD_SIZE unset launches N ranks itself."""
    env = dict(os.environ, PYTHONPATH=ROOT)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT"):
        env.pop(k, None)
    p = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--model", "mlp_mnist", "--batch-per-gpu", "64",
                        "--steps", "3", "--warmup", "1"], cwd=ROOT, env=env, capture_output=True, text=True,
                       timeout=280)
    assert p.returncode == 0, p.stderr[-2000:]
    lines = _json_lines(p.stdout)
    assert len(lines) == 1
    d = lines[0]
    assert d["n_gpus"] == 2 and d["world"] == 2 and d["backend"] == "gloo"
    assert d["config"]["global_batch"] == 128


@pytest.mark.timeout(120)
def test_bench_refuses_world_mismatch():
    """A process group whose size differs from --gpus is an error, never a mislabelled number."""
    env = dict(os.environ, PYTHONPATH=ROOT, RANK="0", WORLD_SIZE="1", LOCAL_RANK="0")
    p = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--model", "mlp_mnist", "--batch-per-gpu", "64",
                        "--steps", "1", "--warmup", "0"], cwd=ROOT, env=env, capture_output=True, text=True,
                       timeout=110)
    assert p.returncode != 0
    assert not _json_lines(p.stdout)
