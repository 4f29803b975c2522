"""The HIP engine's constrained acceleration minimizes MuJoCo's primal problem (GPU).

zb_debug_forward's qacc (fp32, the engine's own rows and Newton solve) against an independent
float64 BFGS minimizer of the oracle's statement of the same problem (tests/primal.py):
|qacc_gpu - a*| <= 1e-3 max(1, |a*|) (fp32 rows on both sides, contact stiffness amplifies them).
"""

import numpy as np
import pytest

import primal as P
from zbot_amd import default_config

pytestmark = pytest.mark.gpu


def test_engine_qacc_is_the_minimizer(cmodel, oracle_mod):
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from zbot_amd.engine import DBG, HipEngine

    cfg = default_config(solver="newton")
    st = P.states(oracle_mod, cmodel, cfg)
    n = st.shape[0]
    rng = np.random.default_rng(0)
    ctrl = (rng.normal(size=(n, 20)) * 1.5).astype(np.float32)
    eng = HipEngine(cmodel, cfg, n)
    dbg = eng.debug_forward(torch.from_numpy(st), torch.from_numpy(ctrl)).cpu().numpy()
    worst = 0.0
    for e in range(n):
        p = oracle_mod.constraint_problem(cmodel.cmodel, cfg, st[e, :27], st[e, 32:58], ctrl=ctrl[e],
                                          qaccw=st[e, 64:90])
        a_star = P.minimize(p)
        qa = dbg[e, DBG["qacc"]:DBG["qacc"] + 26].astype(np.float64)
        err = np.abs(qa - a_star).max() / max(1.0, np.abs(a_star).max())
        worst = max(worst, err)
        assert err <= 1e-3, (e, err)
    print(f"worst relative |qacc_gpu - a*| = {worst:.2e}")


def test_engine_cg_qacc_is_the_minimizer(cmodel, oracle_mod):
    """The CG kernel instantiation (ZbEnvConfig.solver = ZB_SOLVER_CG) with iterations to converge
    reaches the same minimizer (fp32 CG: 2e-3)."""
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from zbot_amd.engine import DBG, HipEngine

    cfg = default_config(solver="cg", iterations=200)
    st = P.states(oracle_mod, cmodel, cfg)
    n = st.shape[0]
    rng = np.random.default_rng(0)
    ctrl = (rng.normal(size=(n, 20)) * 1.5).astype(np.float32)
    eng = HipEngine(cmodel, cfg, n)
    dbg = eng.debug_forward(torch.from_numpy(st), torch.from_numpy(ctrl)).cpu().numpy()
    worst = 0.0
    for e in range(n):
        p = oracle_mod.constraint_problem(cmodel.cmodel, cfg, st[e, :27], st[e, 32:58], ctrl=ctrl[e],
                                          qaccw=st[e, 64:90])
        a_star = P.minimize(p)
        qa = dbg[e, DBG["qacc"]:DBG["qacc"] + 26].astype(np.float64)
        err = np.abs(qa - a_star).max() / max(1.0, np.abs(a_star).max())
        worst = max(worst, err)
        assert err <= 2e-3, (e, err)
    print(f"CG: worst relative |qacc_gpu - a*| = {worst:.2e}")
