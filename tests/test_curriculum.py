"""EpisodeLengthCurriculum (train.py:1595-1602; zbot_amd.curriculum): the level law as a transition
table, the rollout episode-length measure, and the same level on every rank (gloo, world 2)."""

import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from zbot_amd import cstructs as cs
from zbot_amd.curriculum import CurriculumState, EpisodeLengthCurriculum, rollout_episode_length


def test_train_py_defaults():
    c = EpisodeLengthCurriculum()
    assert (c.num_levels, c.increase_threshold, c.decrease_threshold, c.min_level_steps, c.min_level) == (
        30, 30.0, 10.0, 10, 0.5)
    assert c.initial_state() == CurriculumState(level=0.5, steps=0)


def test_transition_table():
    c = EpisodeLengthCurriculum()
    s = c.initial_state()
    # min_level_steps = 10: ten updates at the level before any move
    for k in range(10):
        s = c.update(s, 40.0)
        assert s == CurriculumState(0.5, k + 1)
    s = c.update(s, 40.0)  # above 30 s: up one level (1 / 30), counter restarts
    assert s.level == pytest.approx(0.5 + 1 / 30) and s.steps == 0
    # between the thresholds: hold, count
    for k in range(12):
        s = c.update(s, 20.0)
    assert s.level == pytest.approx(0.5 + 1 / 30) and s.steps == 12
    s = c.update(s, 5.0)  # below 10 s: down
    assert s == CurriculumState(0.5, 0) or (s.level == pytest.approx(0.5) and s.steps == 0)
    # clipped at min_level: a further "down" holds the level and counts
    s = CurriculumState(0.5, 10)
    assert c.update(s, 1.0) == CurriculumState(0.5, 11)
    # clipped at 1
    s = CurriculumState(1.0, 50)
    assert c.update(s, 79.0) == CurriculumState(1.0, 51)
    # exactly at a threshold: no move (strict comparisons)
    s = CurriculumState(0.7, 10)
    assert c.update(s, 30.0).level == 0.7 and c.update(s, 10.0).level == 0.7


def test_climb_to_one_takes_15_moves():
    c = EpisodeLengthCurriculum()
    s, moves = c.initial_state(), 0
    for _ in range(1000):
        nxt = c.update(s, 60.0)
        moves += nxt.level != s.level
        s = nxt
    # (1 - 0.5) * 30 = 15 levels; float steps of 1/30 can leave a last sliver that one more move clips
    assert s.level == 1.0 and moves in (15, 16)


def _stats_state(n, seed):
    rng = np.random.default_rng(seed)
    stats = np.zeros((n, cs.NUM_STATS), np.float32)
    ndone = rng.integers(0, 3, n)
    stats[:, cs.ST_DONE] = ndone
    stats[:, cs.ST_LENGTH] = ndone * rng.integers(5, 400, n)
    state = np.zeros((n, cs.STATE_STRIDE), np.float32)
    state[:, cs.S_EP_STEPS] = rng.integers(0, 4000, n).astype(np.uint32).view(np.float32)
    done_last = (rng.random(n) < 0.2).astype(np.uint8)
    return torch.from_numpy(stats), torch.from_numpy(state), torch.from_numpy(done_last)


def _expected_length(stats, state, done_last, ctrl_dt):
    s = stats.numpy().astype(np.float64)
    run = state.numpy()[:, cs.S_EP_STEPS].view(np.uint32).astype(np.float64)
    open_end = (done_last.numpy() == 0).astype(np.float64)
    per = (s[:, cs.ST_LENGTH] + open_end * run) / np.maximum(s[:, cs.ST_DONE] + open_end, 1.0) * ctrl_dt
    return per.mean()


def test_rollout_episode_length():
    stats, state, done_last = _stats_state(64, 0)
    got = rollout_episode_length(stats, state, done_last, 0.02)
    assert got == pytest.approx(_expected_length(stats, state, done_last, 0.02), rel=1e-12)
    # one env, hand case: two episodes ended (10 and 30 steps) and one still runs (20 steps)
    st = torch.zeros(1, cs.NUM_STATS)
    st[0, cs.ST_DONE], st[0, cs.ST_LENGTH] = 2, 40
    row = torch.zeros(1, cs.STATE_STRIDE)
    row[0, cs.S_EP_STEPS] = torch.tensor([20], dtype=torch.int32).view(torch.float32)[0]
    assert rollout_episode_length(st, row, torch.zeros(1, dtype=torch.uint8), 0.02) == pytest.approx(20 * 0.02)
    # the last step ended the episode: its length is in the stats already, nothing running counts
    assert rollout_episode_length(st, row, torch.ones(1, dtype=torch.uint8), 0.02) == pytest.approx(20 * 0.02)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run_rank(rank, world, port, outdir):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    cur = EpisodeLengthCurriculum(min_level_steps=2)
    s = cur.initial_state()
    levels, lengths = [], []
    for it in range(8):
        # every rank has different local statistics (its own shard of envs)
        stats, state, done_last = _stats_state(32, 100 * it + rank)
        if it >= 4:
            stats[:, cs.ST_LENGTH] = 0.0  # short episodes: the level must come back down
            state[:, cs.S_EP_STEPS] = torch.zeros(32, dtype=torch.int32).view(torch.float32)
        else:
            stats[:, cs.ST_LENGTH] *= 20
        ln = rollout_episode_length(stats, state, done_last, 0.02)
        s = cur.update(s, ln)
        levels.append(s.level)
        lengths.append(ln)
    np.save(os.path.join(outdir, f"r{rank}.npy"), np.array([levels, lengths]))
    dist.barrier()
    dist.destroy_process_group()


def test_every_rank_computes_the_same_level(tmp_path):
    world = 2
    mp.start_processes(_run_rank, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True,
                       start_method="spawn")
    r0, r1 = (np.load(os.path.join(tmp_path, f"r{r}.npy")) for r in range(world))
    assert np.array_equal(r0, r1)  # bit-identical lengths and levels on both ranks
    # the global length is the mean over both shards' envs
    for it in range(8):
        parts = [_stats_state(32, 100 * it + r) for r in range(world)]
        if it < 4:
            for p in parts:
                p[0][:, cs.ST_LENGTH] *= 20
            exp = np.mean([_expected_length(*p, 0.02) for p in parts])
            assert r0[1, it] == pytest.approx(exp, rel=1e-12)
    levels = r0[0]
    assert levels.max() > 0.5 and levels[-1] < levels.max()
