"""bench.py --gpus N is authoritative (CPU, no GPU work): without torchrun it starts N ranks itself,
under torchrun WORLD_SIZE must equal N, and the nccl backend needs N visible GPUs. The launch is
checked with --launch-probe (process group + all_gather of the ranks over gloo, nothing on a GPU)."""

import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _run(args, env=None):
    e = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        e.pop(k, None)
    e.update(env or {})
    return subprocess.run([sys.executable, BENCH, *args], capture_output=True, text=True, timeout=180, cwd=ROOT, env=e)


def test_self_launch_two_ranks_gloo():
    out = _run(["--gpus", "2", "--dist-backend", "gloo", "--launch-probe"])
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout
    res = json.loads(lines[0])
    assert res["n_gpus"] == 2 and res["ranks_seen"] == 2 and res["ranks"] == [0, 1]


def test_self_launch_three_ranks_gloo():
    out = _run(["--gpus", "3", "--dist-backend", "gloo", "--launch-probe"])
    assert out.returncode == 0, out.stderr[-2000:]
    res = json.loads([ln for ln in out.stdout.splitlines() if ln.startswith("{")][0])
    assert res["ranks_seen"] == 3 and res["ranks"] == [0, 1, 2]


def test_world_size_mismatch_exits():
    out = _run(["--gpus", "1"], env={"WORLD_SIZE": "2"})
    assert out.returncode == 2 and "WORLD_SIZE=2" in out.stderr
    out = _run(["--gpus", "4", "--launch-probe"], env={"WORLD_SIZE": "2"})
    assert out.returncode == 2


def test_nccl_needs_a_gpu_per_rank():
    import torch

    n = max(2, torch.cuda.device_count() + 1)
    out = _run(["--gpus", str(n)])
    assert out.returncode == 2 and "device(s) are visible" in out.stderr


def test_bad_gpu_count_exits():
    assert _run(["--gpus", "0"]).returncode == 2


def test_parent_makes_no_device_query(monkeypatch):
    """The self-launching parent decides the world size without asking HIP for devices (ADVICE r05:
    torch's device count may initialise HIP when amdsmi is absent); the ranks check the devices."""
    import argparse

    import torch

    sys.path.insert(0, ROOT)
    import bench

    def boom(*a, **k):
        raise AssertionError("the parent queried the devices")

    monkeypatch.setattr(torch.cuda, "device_count", boom)
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    args = argparse.Namespace(gpus=4, dist_backend="nccl", launch_probe=False)
    assert bench.check_world(args) == (4, True)
    with __import__("pytest").raises(AssertionError):
        bench.check_devices(args)
