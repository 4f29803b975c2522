"""GPU parity of the post-rollout PPO inputs, through
the C ABI (include/zbot_ppo.h) via zbot_amd.ppo.

Bar: bit-exact against the CPU oracle (oracle/zb_oracle_ppo.c) — the kernel
runs the same fp32 reverse scan without contraction, the same fp64 moment
tree and the same IEEE normalization.
"""

import numpy as np
import pytest
import torch

from test_ppo import G, LAM, _rollout

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ppo():
    from zbot_amd import ppo as P

    assert torch.cuda.is_available()
    return P


def _cuda(*xs):
    return [None if x is None else torch.from_numpy(x).cuda() for x in xs]


@pytest.mark.parametrize("T,n,succ,boot", [
    (1, 1, 0.0, False), (7, 33, 0.0, True), (256, 64, 0.3, False), (300, 100, 0.5, True),
    (513, 31, 0.2, False), (256, 8192, 0.0, False),
])
def test_gae_bit_exact(ppo, oracle_mod, T, n, succ, boot):
    r, v, d, s = _rollout(T, n, T * 31 + n, p_succ=succ)
    b = np.random.default_rng(n).normal(size=n).astype(np.float32) if boot else None
    rg, vg, dg, sg, bg = _cuda(r, v, d, s, b)
    g, vt, mom = ppo.gae(rg, vg, dg, G, LAM, successes_t=sg, bootstrap=bg)
    go, vto, mo = oracle_mod.gae(r, v, d, G, LAM, success=s, bootstrap=b)
    np.testing.assert_array_equal(g.cpu().numpy(), go)
    np.testing.assert_array_equal(vt.cpu().numpy(), vto)
    assert np.array_equal(mom.cpu().numpy(), oracle_mod.moments_tree(mo))


def test_normalize_bit_exact_and_rank_combine(ppo, oracle_mod):
    T, n = 64, 256
    r, v, d, _ = _rollout(T, n, 5)
    rg, vg, dg = _cuda(r, v, d)
    out = ppo.compute_ppo_inputs(vg, rg, dg)
    go, _, mo = oracle_mod.gae(r, v, d, G, LAM)
    tot = oracle_mod.moments_tree(mo)
    np.testing.assert_array_equal(out.advantages_t.cpu().numpy(), oracle_mod.adv_normalize(go, tot, go.size))
    np.testing.assert_array_equal(out.gae_t.cpu().numpy(), go)
    # world-size invariance: shards' moments combined on the GPU == the one-GPU moments
    for world in (2, 4, 8):
        per = n // world
        parts = [ppo.gae(rg[:, k * per:(k + 1) * per].contiguous(), vg[:, k * per:(k + 1) * per].contiguous(),
                         dg[:, k * per:(k + 1) * per].contiguous(), G, LAM)[2] for k in range(world)]
        stacked = torch.stack(parts).contiguous()
        comb = torch.empty(2, dtype=torch.float64, device="cuda")
        L = ppo.load_library()
        assert L.zb_moments_combine(stacked.data_ptr(), world, comb.data_ptr(), None) == 0
        assert np.array_equal(comb.cpu().numpy(), tot)


def test_empty_and_errors(ppo):
    L = ppo.load_library()
    z = torch.zeros(2, dtype=torch.float64, device="cuda")
    assert L.zb_gae(None, None, None, None, None, 0, 5, 0.99, 0.95, None, None, None, None, None) == 0
    assert L.zb_gae(None, None, None, None, None, 4, 5, 0.99, 0.95, None, None, None, None, None) == -1
    assert b"null" in L.zb_last_error()
    assert L.zb_gae(None, None, None, None, None, 4, 5, 0.99, 0.95, None, None, None, z.data_ptr(), None) == -1
    assert L.zb_adv_normalize(None, None, 0, None, 1.0, 1e-6, None) == 0
    with pytest.raises(ppo.ZbError):
        ppo.gae(torch.zeros(3, 4), torch.zeros(3, 4), torch.zeros(3, 4, dtype=torch.uint8))


def test_unaligned_normalize(ppo, oracle_mod):
    g = np.random.default_rng(2).normal(size=1001).astype(np.float32)
    mom = np.array([g.astype(np.float64).sum(), (g.astype(np.float64) ** 2).sum()])
    gg = torch.from_numpy(g).cuda()
    src = gg[1:]  # 4-byte offset: scalar path
    out = ppo.normalize(src, torch.from_numpy(mom).cuda(), 1000)
    np.testing.assert_array_equal(out.cpu().numpy(), oracle_mod.adv_normalize(g[1:], mom, 1000))


def test_rollout_buffers_from_zb_step(ppo, oracle_mod, cmodel):
    """zb_step writes reward/done straight into rows of [T, n] buffers; GAE consumes them in place."""
    from zbot_amd import default_config
    from zbot_amd.engine import HipEngine

    T, n = 12, 64
    eng = HipEngine(cmodel, default_config(solver="newton"), n, seed=4)
    eng.reset()
    rew = torch.zeros(T, n, device="cuda")
    done = torch.zeros(T, n, dtype=torch.uint8, device="cuda")
    import oracle as O

    L = eng.L
    for t in range(T):
        a = torch.from_numpy(O.synthetic_actions(cmodel.cmodel, 4, n, 0, t)).cuda()
        assert L.zb_step(eng.h, a.data_ptr(), eng.obs_actor.data_ptr(), eng.obs_critic.data_ptr(), None, None,
                         rew[t].data_ptr(), done[t].data_ptr(), None, 1.0, eng._stream()) == 0
    vals = torch.linspace(-1, 1, T * n, device="cuda").reshape(T, n)
    out = ppo.compute_ppo_inputs(vals, rew, done)
    go, _, _ = oracle_mod.gae(rew.cpu().numpy(), vals.cpu().numpy(), done.cpu().numpy(), G, LAM)
    np.testing.assert_array_equal(out.gae_t.cpu().numpy(), go)
    assert torch.isfinite(out.advantages_t).all()
