"""GRU actor / critic + mixture head, on the CPU.

The oracle (oracle/zb_oracle_policy.c) is checked against an independent
float64 numpy restatement of train.py's Actor / Critic (:885-1023) and the
mixture head (:952-965), the shared fp32 math (include/zbot_fmath.h) against
numpy, threefry against Random123's known answers, and the sampler against the
mixture's moments. Parity vs the reference (jax / equinox / distrax / ksim) is
unpinned: none of them is importable here.
"""

import numpy as np
import pytest

from zbot_amd.policy import ACTOR, CRITIC, EVAL, MODE, SAMPLE, init_params, param_count

H, D, NJ, NM = 128, 5, 20, 5


def _split(P, I, O, actor):
    P = P.astype(np.float64)
    i = 0

    def take(*shape):
        nonlocal i
        k = int(np.prod(shape))
        a = P[i:i + k].reshape(shape)
        i += k
        return a

    win, bin_ = take(H, I), take(H)
    layers = [(take(3 * H, H), take(3 * H, H), take(3 * H), take(H)) for _ in range(D)]
    wout, bout = take(O, H), take(O)
    mb = take(NJ) if actor else None
    assert i == P.size
    return win, bin_, layers, wout, bout, mb


def _sig(x):
    return 1.0 / (1.0 + np.exp(-x))


def np_forward(P, I, O, actor, obs, carry):
    """float64 restatement of Actor/Critic.forward (train.py:943-950, 1011-1017) with equinox GRUCell [U]."""
    win, bin_, layers, wout, bout, _ = _split(P, I, O, actor)
    x = obs.astype(np.float64) @ win.T + bin_
    newc = np.zeros(carry.shape, np.float64)
    for l, (wih, whh, b, bn) in enumerate(layers):
        h = carry[:, l].astype(np.float64)
        ig, hg = x @ wih.T + b, h @ whh.T
        r = _sig(ig[:, :H] + hg[:, :H])
        z = _sig(ig[:, H:2 * H] + hg[:, H:2 * H])
        nn = np.tanh(ig[:, 2 * H:] + r * (hg[:, 2 * H:] + bn))
        x = nn + z * (h - nn)
        newc[:, l] = x
    return x @ wout.T + bout, newc


def np_head(out, mb):
    mu = out[:, :100].reshape(-1, NJ, NM) + mb[None, :, None]
    sd = np.minimum(np.logaddexp(out[:, 100:200], 0.0).reshape(-1, NJ, NM) + 0.01, 1.0)
    lg = out[:, 200:300].reshape(-1, NJ, NM)
    return mu, sd, lg


def _lse(x, axis=-1):
    m = x.max(axis=axis, keepdims=True)
    return (m + np.log(np.exp(x - m).sum(axis=axis, keepdims=True))).squeeze(axis)


def np_mix_log_prob(mu, sd, lg, a):
    logw = lg - _lse(lg)[..., None]
    z = (a[..., None] - mu) / sd
    return _lse(logw - 0.5 * z * z - np.log(sd) - 0.5 * np.log(2 * np.pi))


def test_param_counts(oracle_mod):
    for kind in (ACTOR, CRITIC):
        assert oracle_mod.policy_param_count(kind) == param_count(kind) == init_params(kind).size
    assert param_count(ACTOR) == 128 * 50 + 128 + 5 * (6 * 128 * 128 + 4 * 128) + 300 * 128 + 300 + 20


def test_shared_math_against_numpy(oracle_mod):
    x = np.linspace(-80, 80, 4001).astype(np.float32)
    ref = np.exp(x.astype(np.float64))
    assert np.max(np.abs(oracle_mod.fm("exp", x) - ref) / ref) < 4e-7
    x = np.exp(np.linspace(-60, 60, 4001)).astype(np.float32)
    ref = np.log(x.astype(np.float64))
    assert np.all(np.abs(oracle_mod.fm("log", x) - ref) <= 3e-7 * np.abs(ref) + 3e-7)
    x = np.linspace(-12, 12, 4001).astype(np.float32)
    xd = x.astype(np.float64)
    assert np.max(np.abs(oracle_mod.fm("tanh", x) - np.tanh(xd))) < 3e-7
    assert np.max(np.abs(oracle_mod.fm("sigmoid", x) - _sig(xd))) < 3e-7
    sp = oracle_mod.fm("softplus", x)
    ref = np.logaddexp(xd, 0.0)
    assert np.max(np.abs(sp - ref) / ref) < 2e-6
    t = (np.arange(4096) / 4096).astype(np.float32)
    s, c = oracle_mod.fm_sincos(t)
    ang = 2 * np.pi * t.astype(np.float64)
    assert np.max(np.abs(s - np.sin(ang))) < 5e-7 and np.max(np.abs(c - np.cos(ang))) < 5e-7


def test_threefry_known_answers(oracle_mod):
    """Random123 threefry2x32-20 KATs, for the shared header and the engine oracle."""
    kats = [((0, 0), (0, 0), (0x6B200159, 0x99BA4EFE)),
            ((0xFFFFFFFF, 0xFFFFFFFF), (0xFFFFFFFF, 0xFFFFFFFF), (0x1CB996FC, 0xBB002BE7)),
            ((0x13198A2E, 0x03707344), (0x243F6A88, 0x85A308D3), (0xC4923A9C, 0x483DF7A0))]
    for (k0, k1), (c0, c1), want in kats:
        assert oracle_mod.fm_threefry(k0, k1, c0, c1) == want
        assert oracle_mod.threefry2x32(k0, k1, c0, c1) == want


def test_normal_draws(oracle_mod):
    z = oracle_mod.fm_normals(3, 5, 200000).astype(np.float64)
    assert abs(z.mean()) < 0.01 and abs(z.std() - 1.0) < 0.01
    assert abs(((z - z.mean()) ** 4).mean() / z.var() ** 2 - 3.0) < 0.1


@pytest.mark.parametrize("kind", [ACTOR, CRITIC])
def test_oracle_matches_float64_restatement(oracle_mod, kind):
    I, O = (50, 300) if kind == ACTOR else (484, 1)
    P = init_params(kind, seed=5)
    rng = np.random.default_rng(11)
    T, n = 3, 4
    obs = rng.normal(size=(T, n, I)).astype(np.float32)
    carry0 = (0.5 * rng.normal(size=(n, D, H))).astype(np.float32)
    reset = np.zeros((T, n), np.uint8)
    reset[1, 2] = 1
    acts = (0.3 * rng.normal(size=(T, n, NJ))).astype(np.float32)
    if kind == ACTOR:
        _, lp, cend = oracle_mod.policy_actor(P, obs, carry0, reset, mode=EVAL, actions=acts, log_prob=True)
    else:
        val, cend = oracle_mod.policy_critic(P, obs, carry0, reset)
    c = carry0.astype(np.float64)
    for t in range(T):
        c[reset[t] != 0] = 0.0
        out, c = np_forward(P, I, O, kind == ACTOR, obs[t], c)
        if kind == ACTOR:
            mu, sd, lg = np_head(out, _split(P, I, O, True)[5])
            np.testing.assert_allclose(lp[t], np_mix_log_prob(mu, sd, lg, acts[t].astype(np.float64)),
                                       rtol=1e-4, atol=2e-4)
        else:
            np.testing.assert_allclose(val[t], out[:, 0], rtol=1e-5, atol=2e-5)
    np.testing.assert_allclose(cend, c, rtol=1e-5, atol=2e-5)


def test_reset_restarts_the_carry(oracle_mod):
    P = init_params(ACTOR, seed=2)
    rng = np.random.default_rng(0)
    obs = rng.normal(size=(2, 3, 50)).astype(np.float32)
    carry = rng.normal(size=(3, D, H)).astype(np.float32)
    reset = np.array([[0, 0, 0], [1, 0, 0]], np.uint8)
    a, _, _ = oracle_mod.policy_actor(P, obs, carry, reset, mode=MODE)
    fresh, _, _ = oracle_mod.policy_actor(P, obs[1:2, :1], np.zeros((1, D, H), np.float32), None, mode=MODE)
    np.testing.assert_array_equal(a[1, 0], fresh[0, 0])


def test_mixture_sampler_and_mode(oracle_mod):
    mu = np.array([-0.4, 0.1, 0.5, 0.9, -1.2], np.float32)
    sd = np.array([0.05, 0.2, 0.1, 0.3, 0.02], np.float32)
    lg = np.array([0.3, -0.5, 1.2, 0.0, -2.0], np.float32)
    n = 60000
    x = oracle_mod.mix_sample_batch(mu, sd, lg, seed=7, n=n).astype(np.float64)
    w = np.exp(lg - lg.max())
    w /= w.sum()
    mean = (w * mu).sum()
    var = (w * (sd.astype(np.float64) ** 2 + mu.astype(np.float64) ** 2)).sum() - mean ** 2
    assert abs(x.mean() - mean) < 5 * np.sqrt(var / n)
    assert abs(x.var() - var) < 0.05 * var
    # the whole distribution: Kolmogorov-Smirnov distance to the mixture CDF
    from scipy.stats import norm

    xs = np.sort(x)
    cdf = (w[None, :] * norm.cdf((xs[:, None] - mu[None, :]) / sd[None, :])).sum(1)
    ks = np.max(np.abs(np.arange(1, n + 1) / n - cdf))
    assert ks < 1.63 / np.sqrt(n)  # 1 % critical value
    assert oracle_mod.mix_sample_batch(mu, sd, lg, seed=7, n=3, argmax=True)[0] == mu[2]
    for a in (-1.2, 0.0, 0.45, 2.0):
        want = np_mix_log_prob(mu.astype(np.float64), sd.astype(np.float64), lg.astype(np.float64), np.float64(a))
        assert abs(oracle_mod.mix_log_prob(mu, sd, lg, a) - want) < 2e-5 * max(1.0, abs(want))


def test_sampling_is_keyed_by_global_env_and_step(oracle_mod):
    P = init_params(ACTOR, seed=1)
    obs = np.tile(np.random.default_rng(4).normal(size=(1, 1, 50)).astype(np.float32), (1, 6, 1))
    c0 = np.zeros((6, D, H), np.float32)
    a, _, _ = oracle_mod.policy_actor(P, obs, c0, mode=SAMPLE, seed=9, env_offset=0, step0=5)
    b, _, _ = oracle_mod.policy_actor(P, obs[:, 3:], c0[3:], mode=SAMPLE, seed=9, env_offset=3, step0=5)
    np.testing.assert_array_equal(a[:, 3:], b)
    assert not np.array_equal(a[0, 0], a[0, 1])  # same observation, different env stream
