"""Time-limit (successful) terminations of the oracle (CPU).

ksim marks an episode that reaches EpisodeLengthTermination (train.py:1592, 80 s) without a
failure (BadZ / NotUpright, train.py:1589-1591) as a *success*: compute_ppo_inputs then
bootstraps the step with V(s_t) instead of zero [U]. The engine exports the flag as zb_step's
`success` output; here the oracle's flag is pinned on hand-built cases.
"""

import numpy as np

from zbot_amd import default_config

MAX_SEC = 0.09  # 5 control steps of 0.02 s: 4 * 0.02 < 0.09 <= 5 * 0.02, clear of fp32 rounding


def _bias(cm, n):
    return np.tile(np.array([cm.cmodel.joint_bias[a] for a in range(20)], np.float32), (n, 1))


def test_time_limit_sets_success_unless_failed(oracle_mod, cmodel):
    cfg = default_config(solver="newton", obs_noise=False, max_episode_sec=MAX_SEC)
    n = 6
    env = oracle_mod.OracleEnv(cmodel.cmodel, cfg, n, seed=0)
    env.reset()
    a = _bias(cmodel, n)
    for _ in range(4):
        out = env.step(a)
        assert not out["done"].any() and not out["success"].any()
    env.state[3:, 2] = 0.7  # above BadZ's 0.5: these envs fail on the time-limit step
    out = env.step(a)
    assert out["done"].tolist() == [1] * n
    assert out["success"].tolist() == [1, 1, 1, 0, 0, 0]
    # the auto-reset restarts the episode clock
    out = env.step(a)
    assert not out["done"].any() and not out["success"].any()


def test_failure_alone_is_not_success(oracle_mod, cmodel):
    cfg = default_config(solver="newton", obs_noise=False)
    env = oracle_mod.OracleEnv(cmodel.cmodel, cfg, 2, seed=0)
    env.reset()
    env.state[1, 2] = 0.7
    out = env.step(_bias(cmodel, 2))
    assert out["done"].tolist() == [0, 1] and out["success"].tolist() == [0, 0]


def test_success_step_bootstraps_own_value(oracle_mod):
    """GAE at a time-limit step uses V(s_t): delta = r + gamma V(s_t) - V(s_t), no trace carried."""
    T, n, G, LAM = 6, 3, 0.99, 0.95
    rng = np.random.default_rng(3)
    r = rng.normal(size=(T, n)).astype(np.float32)
    v = rng.normal(size=(T, n)).astype(np.float32)
    d = np.zeros((T, n), np.uint8)
    s = np.zeros((T, n), np.uint8)
    d[4, :] = 1
    s[4, 0] = 1  # env 0 truncated at t = 4, env 1 failed there, env 2 too
    g, _, _ = oracle_mod.gae(r, v, d, G, LAM, success=s)
    assert g[4, 0] == np.float32((r[4, 0] + np.float32(G) * v[4, 0]) - v[4, 0])
    assert g[4, 1] == np.float32(r[4, 1] - v[4, 1])
