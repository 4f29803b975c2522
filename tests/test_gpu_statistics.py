"""Ensemble statistics of the HIP engine against the oracle over a long horizon (GPU).

A legged robot in contact is chaotic: two fp32 implementations that agree to rounding at every
substep (tests/test_gpu_parity.py) separate after tens of control steps. What must still agree
is the distribution they sample. Over 512 envs and 150 control steps with pushes and action
noise (and per-env randomization in the second configuration), from the same reset states and
with the same actions, the time-averaged ensemble means
of the reward, its terms, the base height, the joint speed and the episode ends match the
oracle's within their statistical spread (tolerances below, several standard errors wide).
"""

import numpy as np
import pytest

from zbot_amd import cstructs as cs
from zbot_amd import default_config

pytestmark = pytest.mark.gpu

N, T, STD = 512, 150, 0.2


@pytest.fixture(scope="module", params=[(True, False), (True, True)], ids=["push", "push_randomize"])
def runs(request, cmodel, oracle_mod):
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from zbot_amd.engine import HipEngine

    push, randomize = request.param
    cfg = default_config(solver="newton", push=push, randomize=randomize)
    ref = oracle_mod.OracleEnv(cmodel.cmodel, cfg, N, seed=11)
    ref.reset()
    eng = HipEngine(cmodel, cfg, N, seed=11)
    eng.reset()
    eng.set_state(torch.from_numpy(ref.state.copy()))
    rec = {"oracle": [], "engine": []}
    for t in range(T):
        a = oracle_mod.synthetic_actions(cmodel.cmodel, 3, N, 0, t, std=STD)
        r = ref.step(a)
        o = eng.step(torch.from_numpy(a).cuda())
        st_e = eng.get_state().cpu().numpy()
        for key, out, st in (("oracle", r, ref.state), ("engine", {k: v.cpu().numpy() for k, v in o.items() if v is not None}, st_e)):
            rec[key].append(dict(reward=out["reward"].astype(np.float64), terms=out["reward_terms"].astype(np.float64),
                                 done=out["done"].astype(np.float64), z=st[:, 2].astype(np.float64),
                                 qvel=np.abs(st[:, cs.S_QVEL:cs.S_QVEL + 26]).mean(axis=1).astype(np.float64)))
    return rec


def _mean(rec, key):
    return np.mean([r[key].mean() for r in rec])


def _sem(rec, key):
    # standard error of the time-averaged ensemble mean, envs as the independent unit
    per_env = np.mean([r[key] for r in rec], axis=0)
    return per_env.std() / np.sqrt(per_env.size)


@pytest.mark.parametrize("key", ["reward", "z", "qvel"])
def test_ensemble_means_match(runs, key):
    mo, me = _mean(runs["oracle"], key), _mean(runs["engine"], key)
    tol = 5.0 * np.hypot(_sem(runs["oracle"], key), _sem(runs["engine"], key)) + 1e-3 * abs(mo)
    print(f"{key}: oracle {mo:.6g} engine {me:.6g} tol {tol:.3g}")
    assert abs(me - mo) <= tol


def test_reward_terms_match(runs):
    to = np.mean([r["terms"].mean(axis=0) for r in runs["oracle"]], axis=0)
    te = np.mean([r["terms"].mean(axis=0) for r in runs["engine"]], axis=0)
    po = np.mean([r["terms"] for r in runs["oracle"]], axis=0)  # per env, time-averaged
    pe = np.mean([r["terms"] for r in runs["engine"]], axis=0)
    sem = np.hypot(po.std(axis=0), pe.std(axis=0)) / np.sqrt(N)
    tol = 5.0 * sem + 1e-3 * np.abs(to) + 1e-6
    for i in range(cs.NUM_TERMS):
        print(f"term {i}: oracle {to[i]:.6g} engine {te[i]:.6g} tol {tol[i]:.3g}")
    assert (np.abs(te - to) <= tol).all()


def test_episode_ends_match(runs):
    do = sum(r["done"].sum() for r in runs["oracle"])
    de = sum(r["done"].sum() for r in runs["engine"])
    print(f"episode ends: oracle {do:.0f} engine {de:.0f}")
    # counts of rare events: Poisson spread
    assert abs(de - do) <= 5.0 * np.sqrt(max(do, 1.0)) + 2


def test_long_soak_full_size(cmodel):
    """C5-shaped soak: 8192 envs, pushes and per-env randomization, noisy actions, 1500 control
    steps (30 000 physics substeps, many episodes per env). Nothing goes non-finite, no env
    raises the NaN flag, quaternions stay unit, episodes keep ending and restarting, and the
    per-step reward stays finite and bounded."""
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from zbot_amd.engine import HipEngine

    n, steps = 8192, 1500
    cfg = default_config(solver="newton", push=True, randomize=True)
    eng = HipEngine(cmodel, cfg, n, seed=5)
    eng.reset()
    g = torch.Generator(device="cuda")
    g.manual_seed(9)
    bias = torch.tensor([cmodel.cmodel.joint_bias[i] for i in range(20)], device="cuda")
    acts = [bias + 0.2 * torch.randn(n, 20, device="cuda", generator=g) for _ in range(16)]
    rmin, rmax, dones = float("inf"), float("-inf"), 0
    for t in range(steps):
        out = eng.step(acts[t % len(acts)])
        if t % 100 == 99:
            r = out["reward"]
            assert torch.isfinite(r).all()
            rmin, rmax = min(rmin, float(r.min())), max(rmax, float(r.max()))
    st = eng.get_state()
    stats = eng.get_stats(clear=True)
    dones = float(stats[:, cs.ST_DONE].sum())
    assert torch.isfinite(st[:, :58]).all() and torch.isfinite(out["obs_critic"]).all()
    assert (st[:, cs.S_NAN].view(torch.int32) == 0).all()
    assert torch.allclose(st[:, 3:7].norm(dim=1), torch.ones(n, device="cuda"), atol=2e-6)
    print(f"soak: {dones:.0f} episode ends over {n} envs x {steps} steps, reward range [{rmin:.3g}, {rmax:.3g}]")
    assert dones > n  # envs fall and restart, repeatedly
    assert -100.0 < rmin and rmax < 100.0
