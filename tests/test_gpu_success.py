"""zb_step / zb_rollout `success` output (time-limit ends) vs the oracle, and its use in GAE.

Flags are integer outputs: exact. GAE through the C ABI is bit-exact against the oracle
(tests/test_gpu_ppo.py), here fed the engine's own done / success rows.
"""

import numpy as np
import pytest

from zbot_amd import default_config

pytestmark = pytest.mark.gpu
MAX_SEC = 0.09  # 5 control steps (tests/test_success.py)
G, LAM = 0.99, 0.95


@pytest.fixture(scope="module")
def torch_gpu():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch


def _bias(cm, n):
    return np.tile(np.array([cm.cmodel.joint_bias[a] for a in range(20)], np.float32), (n, 1))


def test_success_flags_match_oracle(torch_gpu, cmodel, oracle_mod):
    torch = torch_gpu
    from zbot_amd.engine import HipEngine

    cfg = default_config(solver="newton", max_episode_sec=MAX_SEC)
    n = 40
    ref = oracle_mod.OracleEnv(cmodel.cmodel, cfg, n, seed=5)
    ref.reset()
    eng = HipEngine(cmodel, cfg, n, seed=5)
    eng.reset()
    eng.set_state(torch.from_numpy(ref.state.copy()))
    seen_success = seen_fail = 0
    for t in range(12):
        if t == 4:  # lift a third of the envs above BadZ on the time-limit step: failures, not successes
            st = ref.state.copy()
            st[::3, 2] = 0.7
            ref.state[:] = st
            eng.set_state(torch.from_numpy(st))
        a = oracle_mod.synthetic_actions(cmodel.cmodel, 5, n, 0, t)
        r = ref.step(a)
        o = eng.step(torch.from_numpy(a).cuda())
        torch.cuda.synchronize()
        np.testing.assert_array_equal(o["done"].cpu().numpy(), r["done"])
        np.testing.assert_array_equal(o["success"].cpu().numpy(), r["success"])
        seen_success += int(r["success"].sum())
        seen_fail += int((r["done"] & ~r["success"].astype(bool)).sum())
        ref.state[:] = eng.get_state().cpu().numpy()  # keep the chaotic trajectories together
    assert seen_success > 0 and seen_fail > 0


def test_rollout_success_is_last_step(torch_gpu, cmodel):
    torch = torch_gpu
    from zbot_amd.engine import HipEngine

    cfg = default_config(solver="newton", max_episode_sec=MAX_SEC)
    n = 16
    a = torch.from_numpy(np.tile(_bias(cmodel, n), (5, 1, 1))).cuda()
    e1 = HipEngine(cmodel, cfg, n, seed=2)
    e2 = HipEngine(cmodel, cfg, n, seed=2)
    e1.reset()
    e2.reset()
    for t in range(5):
        o1 = e1.step(a[t])
    o2 = e2.rollout(a)
    torch.cuda.synchronize()
    assert o1["success"].cpu().numpy().all()
    np.testing.assert_array_equal(o2["success"].cpu().numpy(), o1["success"].cpu().numpy())
    np.testing.assert_array_equal(o2["done"].cpu().numpy(), o1["done"].cpu().numpy())


def test_policy_rollout_successes_feed_gae(torch_gpu, cmodel, oracle_mod):
    """PolicyRollout records successes_t; compute_ppo_inputs bootstraps those steps with V(s_t)."""
    torch = torch_gpu
    from zbot_amd import policy as P
    from zbot_amd import ppo
    from zbot_amd.engine import HipEngine

    cfg = default_config(solver="newton", max_episode_sec=MAX_SEC)
    n, T = 64, 12
    eng = HipEngine(cmodel, cfg, n, seed=9)
    ro = P.PolicyRollout(eng, P.GruPolicy(P.ACTOR, P.init_params(P.ACTOR, seed=0)), seed=1)
    ro.reset()
    traj = ro.run(T)
    done = traj["done"].cpu().numpy()
    succ = traj["success"].cpu().numpy()
    assert succ[4].sum() > 0 and (succ <= done).all()
    assert not succ[:4].any()
    vals = torch.linspace(-2, 2, T * n, device="cuda").reshape(T, n)
    out = ppo.compute_ppo_inputs(vals, traj["reward"], traj["done"], traj["success"], normalize_advantages=False)
    rew = traj["reward"].cpu().numpy()
    v = vals.cpu().numpy()
    go, vto, _ = oracle_mod.gae(rew, v, done, G, LAM, success=succ)
    np.testing.assert_array_equal(out.gae_t.cpu().numpy(), go)
    np.testing.assert_array_equal(out.value_targets_t.cpu().numpy(), vto)
    g = out.gae_t.cpu().numpy()
    for e in np.flatnonzero(succ[4]):  # delta at the time-limit step bootstraps with V(s_t), no trace
        assert g[4, e] == np.float32((rew[4, e] + np.float32(G) * v[4, e]) - v[4, e])


def test_bad_buffers_raise_before_the_kernel(torch_gpu, cmodel):
    """Buffers the kernels dereference through raw pointers are checked on the host first."""
    torch = torch_gpu
    from zbot_amd import ppo
    from zbot_amd.cstructs import RAND_STRIDE
    from zbot_amd.engine import HipEngine, ZbError

    eng = HipEngine(cmodel, default_config(solver="newton"), 8)
    eng.reset()
    with pytest.raises(ZbError):
        eng.set_rand(torch.zeros(4, RAND_STRIDE))  # short: would read past its end
    with pytest.raises(ZbError):
        eng.rollout(torch.zeros(2, 8, 20, device="cuda"), reward_sum=torch.zeros(4, device="cuda"))
    with pytest.raises(ZbError):
        eng.rollout(torch.zeros(2, 8, 20, device="cuda"), reward_sum=torch.zeros(8, dtype=torch.float64, device="cuda"))
    g = torch.randn(3, 8, device="cuda")
    with pytest.raises(ZbError):
        ppo.normalize(g, torch.tensor([1.0, 2.0], dtype=torch.float64), 24.0)  # host moments
    with pytest.raises(ZbError):
        ppo.normalize(g, torch.tensor([1.0, 2.0], device="cuda"), 24.0)  # float32 moments
    ok = ppo.normalize(g, torch.tensor([0.0, 24.0], dtype=torch.float64, device="cuda"), 24.0)
    torch.cuda.synchronize()
    np.testing.assert_allclose(ok.cpu().numpy(), g.cpu().numpy() / (1.0 + 1e-6), rtol=1e-6)
