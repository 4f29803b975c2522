"""Post-rollout PPO inputs: oracle known answers, the
moment tree's shard invariance, and the world-size-2 rank combine (gloo).

The oracle (oracle/zb_oracle_ppo.c) restates ksim 0.1.99 compute_ppo_inputs
[U]; ksim is not importable here and the reference holds no fixtures, so the
restatement is pinned by the closed forms below (parity vs ksim: unpinned).
"""

import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

G, LAM = 0.99, 0.95


def np_gae(r, v, d, gamma, lam, succ=None, boot=None):
    """Independent numpy fp32 restatement (same operation order; the recurrence as one fma)."""
    r, v = r.astype(np.float32), v.astype(np.float32)
    T, n = r.shape
    g32, gl = np.float32(gamma), np.float32(gamma) * np.float32(lam)
    out = np.zeros((T, n), np.float32)
    a = np.zeros(n, np.float32)
    for t in range(T - 1, -1, -1):
        vs = v[t + 1] if t + 1 < T else (v[t] if boot is None else boot.astype(np.float32))
        mask = np.where(d[t] != 0, np.float32(0), np.float32(1))
        nxt = vs * mask
        if succ is not None:
            nxt = np.where(succ[t] != 0, v[t], nxt)
        delta = (r[t] + g32 * nxt) - v[t]
        # fma(c, a, delta) with one rounding: the fp32 product is exact in fp64 and the fp64
        # sum rounds once more to fp32 (double rounding can differ by 1 ulp in rare ties)
        a = ((gl * mask).astype(np.float64) * a.astype(np.float64) + delta.astype(np.float64)).astype(np.float32)
        out[t] = a
    return out


def _rollout(T, n, seed, p_done=0.05, p_succ=0.0):
    rng = np.random.default_rng(seed)
    r = rng.normal(0.5, 1.0, (T, n)).astype(np.float32)
    v = rng.normal(2.0, 3.0, (T, n)).astype(np.float32)
    d = (rng.random((T, n)) < p_done).astype(np.uint8)
    s = ((rng.random((T, n)) < p_succ) & (d != 0)).astype(np.uint8) if p_succ else None
    return r, v, d, s


def test_single_step_known_answer(oracle_mod):
    r = np.array([[1.5]], np.float32)
    v = np.array([[2.0]], np.float32)
    d = np.zeros((1, 1), np.uint8)
    g, vt, mom = oracle_mod.gae(r, v, d, G, LAM)
    # last row bootstraps from its own value (ksim convention [U])
    assert g[0, 0] == np.float32((np.float32(1.5) + np.float32(G) * np.float32(2.0)) - np.float32(2.0))
    assert vt[0, 0] == np.float32(g[0, 0] + np.float32(2.0))
    assert mom[0, 0] == float(g[0, 0]) and mom[0, 1] == float(g[0, 0]) ** 2
    g, _, _ = oracle_mod.gae(r, v, d, G, LAM, bootstrap=np.array([0.0], np.float32))
    assert g[0, 0] == np.float32(1.5 - 2.0)
    g, _, _ = oracle_mod.gae(r, v, np.ones((1, 1), np.uint8), G, LAM)
    assert g[0, 0] == np.float32(1.5 - 2.0)  # terminal: no bootstrap


def test_constant_reward_geometric_series(oracle_mod):
    T, n = 40, 3
    r = np.ones((T, n), np.float32)
    v = np.zeros((T, n), np.float32)
    d = np.zeros((T, n), np.uint8)
    g, _, _ = oracle_mod.gae(r, v, d, G, LAM)
    k = np.arange(T)[::-1]  # steps remaining after t
    want = (1 - (G * LAM) ** (k + 1)) / (1 - G * LAM)
    np.testing.assert_allclose(g[:, 0], want, rtol=1e-5)


def test_done_cuts_the_trace(oracle_mod):
    T = 10
    r = np.ones((T, 1), np.float32)
    v = np.zeros((T, 1), np.float32)
    d = np.zeros((T, 1), np.uint8)
    d[4] = 1
    g, _, _ = oracle_mod.gae(r, v, d, G, LAM)
    assert g[4, 0] == 1.0  # episode ends at t=4: delta only
    np.testing.assert_allclose(g[3, 0], 1 + G * LAM, rtol=1e-6)
    g_tail, _, _ = oracle_mod.gae(r[5:], v[5:], d[5:], G, LAM)
    np.testing.assert_array_equal(g[5:], g_tail)  # later episode independent of the earlier one


def test_success_bootstraps_own_value(oracle_mod):
    r = np.zeros((2, 1), np.float32)
    v = np.array([[3.0], [5.0]], np.float32)
    d = np.array([[1], [0]], np.uint8)
    s = np.array([[1], [0]], np.uint8)
    g, _, _ = oracle_mod.gae(r, v, d, G, LAM, success=s)
    assert g[0, 0] == np.float32(np.float32(G) * np.float32(3.0) - np.float32(3.0))


@pytest.mark.parametrize("T,n,succ", [(1, 5, 0.0), (17, 33, 0.3), (300, 40, 0.5)])
def test_oracle_matches_numpy(oracle_mod, T, n, succ):
    r, v, d, s = _rollout(T, n, 7 + T, p_succ=succ)
    boot = np.random.default_rng(1).normal(size=n).astype(np.float32)
    for b in (None, boot):
        g, vt, _ = oracle_mod.gae(r, v, d, G, LAM, success=s, bootstrap=b)
        ref = np_gae(r, v, d, G, LAM, s, b)
        np.testing.assert_allclose(g, ref, rtol=1e-6, atol=1e-6)
        np.testing.assert_allclose(vt, ref + v, rtol=1e-6, atol=1e-6)


def test_moment_tree_is_shard_invariant(oracle_mod):
    """Rank subtrees combined in rank order == the one-GPU tree (power-of-two shards)."""
    r, v, d, _ = _rollout(64, 256, 3)
    _, _, mom = oracle_mod.gae(r, v, d, G, LAM)
    full = oracle_mod.moments_tree(mom)
    for world in (2, 4, 8):
        per = 256 // world
        ranks = np.stack([oracle_mod.moments_tree(mom[k * per:(k + 1) * per]) for k in range(world)])
        assert np.array_equal(oracle_mod.moments_tree(ranks), full)
    np.testing.assert_allclose(full, mom.sum(0), rtol=1e-12)


def test_normalize_unit_moments(oracle_mod):
    r, v, d, _ = _rollout(50, 64, 5)
    g, _, mom = oracle_mod.gae(r, v, d, G, LAM)
    tot = oracle_mod.moments_tree(mom)
    adv = oracle_mod.adv_normalize(g, tot, g.size)
    assert abs(float(adv.astype(np.float64).mean())) < 1e-5
    assert abs(float(adv.astype(np.float64).std()) - 1.0) < 1e-4


def test_host_rank_tree_matches_oracle_tree(oracle_mod):
    from zbot_amd.ppo import pairwise_tree_host

    rng = np.random.default_rng(0)
    for k in (1, 2, 3, 5, 8):
        pairs = rng.normal(size=(k, 2))
        assert np.array_equal(pairwise_tree_host(torch.from_numpy(pairs)).numpy(), oracle_mod.moments_tree(pairs))


# ---- world size 2 over gloo: the rank combine of compute_ppo_inputs ----

def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank(rank, world, port, outdir):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    os.environ["OMP_NUM_THREADS"] = "1"
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import oracle as O
    from zbot_amd.dist import shard
    from zbot_amd.ppo import combine_moments, global_count

    r, v, d, _ = _rollout(32, 64, 9)
    off, n = shard(64, world, rank)
    g, _, mom = O.gae(r[:, off:off + n], v[:, off:off + n], d[:, off:off + n], G, LAM)
    local = torch.from_numpy(O.moments_tree(mom))
    tot = combine_moments(local)
    cnt = global_count(g.size)
    gathered = [torch.zeros(2, dtype=torch.float64) for _ in range(world)]
    dist.all_gather(gathered, tot)
    if rank == 0:
        np.save(os.path.join(outdir, "tot.npy"), torch.stack(gathered).numpy())
        np.save(os.path.join(outdir, "cnt.npy"), np.array([cnt]))
    dist.barrier()
    dist.destroy_process_group()


def test_rank_combine_world2_equals_single_process(tmp_path, oracle_mod):
    world = 2
    mp.start_processes(_rank, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True,
                       start_method="spawn")
    tot = np.load(tmp_path / "tot.npy")
    r, v, d, _ = _rollout(32, 64, 9)
    _, _, mom = oracle_mod.gae(r, v, d, G, LAM)
    want = oracle_mod.moments_tree(mom)
    assert np.array_equal(tot[0], want) and np.array_equal(tot[1], want)  # every rank, same bits
    assert int(np.load(tmp_path / "cnt.npy")[0]) == 32 * 64
