"""World-size-2 sharding over the env axis with the gloo backend (CPU).

The GPU path shards identically (one process per GPU, RCCL); here the CPU
oracle stands in for the per-rank engine so the sharding/RNG-keying and the
statistics reduction are exercised without a GPU.
"""

import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

N_GLOBAL = 16
STEPS = 4
SEED = 11


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run_rank(rank, world, port, outdir):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    os.environ["OMP_NUM_THREADS"] = "1"
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import oracle as O
    from zbot_amd import compile_model, default_config
    from zbot_amd.dist import reduce_episode_stats, shard

    cm = compile_model()
    cfg = default_config(solver="newton")
    off, n = shard(N_GLOBAL, world, rank)
    env = O.OracleEnv(cm.cmodel, cfg, n, env_offset=off, seed=SEED)
    env.reset()
    for t in range(STEPS):
        env.step(O.synthetic_actions(cm.cmodel, SEED, n, off, t))
    env.stats[:, 2] += 1.0  # make the statistics non-trivial
    total = reduce_episode_stats(torch.from_numpy(env.stats))
    states = [torch.zeros(n, env.state.shape[1]) for _ in range(world)]
    dist.all_gather(states, torch.from_numpy(env.state))
    if rank == 0:
        np.save(os.path.join(outdir, "state.npy"), torch.cat(states).numpy())
        np.save(os.path.join(outdir, "stats.npy"), total.numpy())
    dist.barrier()
    dist.destroy_process_group()


def test_sharded_equals_single_process(tmp_path, cmodel, oracle_mod):
    world = 2
    mp.start_processes(_run_rank, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True,
                       start_method="spawn")
    sharded = np.load(tmp_path / "state.npy")
    stats = np.load(tmp_path / "stats.npy")
    from zbot_amd import default_config

    env = oracle_mod.OracleEnv(cmodel.cmodel, default_config(solver="newton"), N_GLOBAL, seed=SEED)
    env.reset()
    for t in range(STEPS):
        env.step(oracle_mod.synthetic_actions(cmodel.cmodel, SEED, N_GLOBAL, 0, t))
    env.stats[:, 2] += 1.0
    # RNG keyed by global env id -> bit-identical per-env state for any world size
    assert np.array_equal(sharded, env.state)
    ref = env.stats.astype(np.float64).sum(0)
    # rank partials summed in fixed order; equals the single-process sum to fp64 rounding
    np.testing.assert_allclose(stats, ref, rtol=1e-12)
    assert stats[2] == pytest.approx(N_GLOBAL)


def test_shard_rejects_uneven():
    from zbot_amd.dist import shard

    assert shard(65536, 8, 3) == (3 * 8192, 8192)
    with pytest.raises(ValueError):
        shard(10, 3, 0)
