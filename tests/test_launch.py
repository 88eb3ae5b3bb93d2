"""The ``python -m distriflow_amd.launch`` CLI: every mode end to end on CPU, plus the
fault drill of SURVEY §5.3 — a rank killed mid-run, the job restarted from its checkpoint."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, timeout=600):
    env = dict(os.environ, PYTHONPATH=ROOT)
    env.pop("WORLD_SIZE", None)
    p = subprocess.run([sys.executable, "-m", "distriflow_amd.launch"] + args, cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=timeout)
    return p


def _last_json(out: str) -> dict:
    lines = [l for l in out.splitlines() if l.startswith("{")]
    assert lines, out
    return json.loads(lines[-1])


@pytest.mark.timeout(600)
def test_ps_modes_single_process():
    from distriflow_amd.launch import main

    # in-process: server + worker threads over the local transport
    for argv in (["async", "--model", "mlp_mnist", "--num-examples", "1024", "--batch", "64", "--workers", "2",
                  "--max-staleness", "1", "--device", "cpu"],
                 ["fedavg", "--model", "mlp_mnist", "--num-examples", "2048", "--batch", "64", "--workers", "3",
                  "--rounds", "2", "--local-steps", "5", "--device", "cpu"],
                 ["fedsgd", "--model", "mlp_mnist", "--num-examples", "1024", "--batch", "32", "--workers", "2",
                  "--updates-per-worker", "4", "--device", "cpu"]):
        assert main(argv) == 0


@pytest.mark.timeout(900)
def test_sync_fault_kill_and_resume(tmp_path):
    d = str(tmp_path / "ckpt")
    p = _run(["--nproc", "2", "--max-restarts", "1", "sync", "--model", "mlp_mnist", "--num-examples", "2048",
              "--batch", "64", "--epochs", "3", "--device", "cpu", "--save-dir", d,
              "--fault-kill-rank", "1", "--fault-kill-step", "20"])
    assert p.returncode == 0, p.stderr[-3000:]
    assert "[fault] rank 1 killed" in p.stderr
    assert "exited with 17" in p.stderr
    res = _last_json(p.stdout)
    assert res["mode"] == "sync" and res["world"] == 2
    rec = json.load(open(os.path.join(d, "resume.json")))
    assert rec["epoch"] == 2
    assert os.path.exists(os.path.join(d, "current", "model.json"))


@pytest.mark.timeout(900)
def test_async_parameter_server_three_ranks():
    p = _run(["--nproc", "3", "async", "--model", "mlp_mnist", "--num-examples", "1024", "--batch", "64",
              "--max-staleness", "2", "--device", "cpu"])
    assert p.returncode == 0, p.stderr[-3000:]
    res = _last_json(p.stdout)
    assert res["world"] == 3 and res["updates"] >= 16


@pytest.mark.timeout(300)
def test_fedavg_device_engine_two_ranks_cpu():
    """FedAvgTrainer (parallel/fedavg.py): every rank a client on a non-IID shard, collective averaging."""
    import socket

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    env = dict(os.environ, PYTHONPATH=ROOT)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK"):
        env.pop(k, None)
    p = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", str(port), "-m", "distriflow_amd.launch",
                        "fedavg", "--engine", "device", "--device", "cpu", "--model", "mlp_mnist",
                        "--num-examples", "4096", "--batch", "64", "--rounds", "4", "--local-steps", "10",
                        "--lr", "0.1"], cwd=ROOT, env=env, capture_output=True, text=True, timeout=280)
    assert p.returncode == 0, p.stderr[-3000:]
    out = _last_json(p.stdout)
    assert out["engine"] == "device" and out["clients"] == 2 and out["rounds"] == 4
    assert out["test_accuracy"] > 0.3


@pytest.mark.timeout(900)
def test_resumed_job_matches_uninterrupted_job(tmp_path):
    """a job killed mid-epoch and resumed from its last checkpoint trains on exactly the batches
    of an uninterrupted job (the schedule is rebuilt from the original seed and the resumed job skips the
    steps already taken), so both end with bit-identical weights."""
    common = ["sync", "--model", "mlp_mnist", "--num-examples", "2048", "--batch", "64", "--epochs", "3",
              "--device", "cpu"]
    a, b = str(tmp_path / "a"), str(tmp_path / "b")
    p = _run(["--nproc", "2"] + common + ["--save-dir", a])
    assert p.returncode == 0, p.stderr[-3000:]
    p = _run(["--nproc", "2", "--max-restarts", "1"] + common +
             ["--save-dir", b, "--fault-kill-rank", "0", "--fault-kill-step", "25"])
    assert p.returncode == 0, p.stderr[-3000:]
    assert "[fault] rank 0 killed" in p.stderr and "exited with 17" in p.stderr
    wa = open(os.path.join(a, "current", "weights.bin"), "rb").read()
    wb = open(os.path.join(b, "current", "weights.bin"), "rb").read()
    assert len(wa) > 0 and wa == wb


@pytest.mark.timeout(600)
def test_sync_metrics_jsonl_has_per_step_upload_records(tmp_path):
    """The device engine's callbacks (DataParallelTrainer.on_upload) write one JSONL record per replay:
    versions advance by the replay's steps and every record carries loss / accuracy."""
    m = str(tmp_path / "m.jsonl")
    p = _run(["--nproc", "2", "sync", "--model", "mlp_mnist", "--num-examples", "1024", "--batch", "64",
              "--epochs", "1", "--device", "cpu", "--metrics", m])
    assert p.returncode == 0, p.stderr[-3000:]
    recs = [json.loads(l) for l in open(m)]
    ups = [r for r in recs if r.get("event") == "upload" and r.get("rank") == 0]
    assert [u["version"] for u in ups] == list(range(1, 9))  # 1024 / 64 / 2 ranks = 8 steps, one per replay
    assert all(u["updates"] == 1 and u["world"] == 2 and 0.0 <= u["accuracy"] <= 1.0 for u in ups)
