"""Multi-rank sharding of the HIP engine on the GPU box (gloo rehearsal, ranks sharing one GPU).

RCCL needs one GPU per rank, so on the one-GPU test box two processes share cuda:0 and exchange
over gloo; the data path has no collective either way. Checks:
  * two ranks, each a HipEngine over its half of the global envs (env_offset = rank * n), give
    bit-identical per-env states to one process over all envs (RNG keyed by global env id);
  * bench.py under torch.distributed.run with 2 ranks prints one JSON line with the whole-job value,
    and so does `bench.py --gpus 2` launched without torchrun (it starts its ranks itself);
  * RCCL itself at world size 1 (one GPU, one rank): the statistics reduction's all_gather and the
    barriers through the `nccl` backend, in a spawned rank and in bench.py --init-dist.
"""

import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
N_GLOBAL = 96
STEPS = 4
SEED = 21


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run_rank(rank, world, port, outdir):
    import torch
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import oracle as O
    from zbot_amd import compile_model, default_config
    from zbot_amd.dist import shard
    from zbot_amd.engine import HipEngine

    cm = compile_model()
    cfg = default_config(solver="newton", push=True, randomize=True)
    off, n = shard(N_GLOBAL, world, rank)
    eng = HipEngine(cm, cfg, n, env_offset=off, seed=SEED)
    eng.reset()
    for t in range(STEPS):
        eng.step(torch.from_numpy(O.synthetic_actions(cm.cmodel, SEED, n, off, t)).cuda())
    st = eng.get_state().cpu()
    parts = [torch.zeros_like(st) for _ in range(world)]
    dist.all_gather(parts, st)
    if rank == 0:
        np.save(os.path.join(outdir, "state.npy"), torch.cat(parts).numpy())
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_shards_equal_one_process(tmp_path, cmodel, oracle_mod):
    import torch
    import torch.multiprocessing as mp

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from zbot_amd import default_config
    from zbot_amd.engine import HipEngine

    mp.start_processes(_run_rank, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True, start_method="spawn")
    sharded = np.load(tmp_path / "state.npy")
    eng = HipEngine(cmodel, default_config(solver="newton", push=True, randomize=True), N_GLOBAL, seed=SEED)
    eng.reset()
    for t in range(STEPS):
        eng.step(torch.from_numpy(oracle_mod.synthetic_actions(cmodel.cmodel, SEED, N_GLOBAL, 0, t)).cuda())
    single = eng.get_state().cpu().numpy()
    assert np.array_equal(sharded.view(np.uint32), single.view(np.uint32))


def test_bench_two_ranks_gloo_rehearsal():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(ROOT, "bench.py"),
           "--gpus", "2", "--dist-backend", "gloo", "--steps", "3", "--warmup", "1", "--envs", "1024",
           "--no-cpu-baseline"]
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout[-2000:]
    res = json.loads(lines[0])
    assert res["n_gpus"] == 2 and res["config"]["global_envs"] == 2048 and res["scaling"] == "weak"
    assert res["value"] > 0 and np.isfinite(res["value"])
    assert res["rollout_pipeline"]["env_steps_per_s"] > 0 and res["ppo_inputs"]["gae_kernel_ms"] > 0
    assert res["ranks_seen"] == 2


def test_bench_self_launch_two_ranks():
    # `bench.py --gpus 2` without torchrun starts its two ranks itself (spawn, from a parent that
    # made no GPU call); gloo rehearsal: both ranks share cuda:0 on the one-GPU box
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dist-backend", "gloo", "--steps", "3",
           "--warmup", "1", "--envs", "1024", "--no-cpu-baseline", "--no-extra-legs", "--no-policy", "--no-pipeline"]
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout[-2000:]
    res = json.loads(lines[0])
    assert res["n_gpus"] == 2 and res["ranks_seen"] == 2 and res["process_group"] == "gloo"
    assert res["config"]["global_envs"] == 2048 and res["value"] > 0


def _run_rccl_rank(rank, world, port, outdir):
    # one rank over RCCL (the `nccl` backend) on cuda:0: the communicator set-up, the all_gather of
    # reduce_fixed_order and the barrier that bench.py runs at N > 1, here at world size 1
    import torch
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)
    import oracle as O
    from zbot_amd import compile_model, default_config
    from zbot_amd.dist import reduce_episode_stats
    from zbot_amd.engine import HipEngine

    cm = compile_model()
    cfg = default_config(solver="newton", push=True, randomize=True)
    eng = HipEngine(cm, cfg, 64, seed=SEED)
    eng.reset()
    for t in range(STEPS):
        eng.step(torch.from_numpy(O.synthetic_actions(cm.cmodel, SEED, 64, 0, t)).cuda())
    st = eng.get_stats(clear=False)
    tot = reduce_episode_stats(st)
    dist.barrier()
    assert dist.get_backend() == "nccl" and tot.device.type == "cuda"
    np.save(os.path.join(outdir, "rccl.npy"), np.stack([tot.cpu().numpy(), st.double().sum(0).cpu().numpy()]))
    dist.destroy_process_group()


def test_rccl_one_rank_reduction(tmp_path):
    import torch
    import torch.multiprocessing as mp

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    mp.start_processes(_run_rccl_rank, args=(1, _free_port(), str(tmp_path)), nprocs=1, join=True,
                       start_method="spawn")
    tot, local = np.load(tmp_path / "rccl.npy")
    assert np.array_equal(tot, local)


def test_bench_one_rank_rccl():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(ROOT, "bench.py"),
           "--gpus", "1", "--init-dist", "--dist-backend", "nccl", "--steps", "3", "--warmup", "1", "--envs", "1024",
           "--no-cpu-baseline", "--no-extra-legs"]
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout[-2000:]
    res = json.loads(lines[0])
    assert res["process_group"] == "nccl" and res["n_gpus"] == 1
    assert res["value"] > 0 and res["ppo_inputs"]["gae_kernel_ms"] > 0
