"""The Newton solution is the minimizer of MuJoCo's primal problem (oracle, CPU).

Parity of the solver without trusting its own iteration: the oracle's fp32 qacc (8 Newton
iterations, exact line search, active-set Hessian) must agree with an independent float64 BFGS
minimizer of the same problem (tests/primal.py) on warm standing states, states pressed into the
floor and states past a joint limit. Tolerances: |qacc - a*| <= 1e-4 max|a*|, |grad| <= 1e-5 of
|M(a - a0)| + |J'f|, cost above the minimum by <= 1e-6 relative. The GPU engine's qacc is held to
the same minimizer in tests/test_gpu_solver_optimality.py.
"""

import numpy as np

import primal as P
from zbot_amd import default_config


def test_oracle_newton_solution_is_the_minimizer(oracle_mod, cmodel):
    cfg = default_config(solver="newton")
    st = P.states(oracle_mod, cmodel, cfg)
    rng = np.random.default_rng(0)
    kinds = np.zeros(3, int)
    for e in range(st.shape[0]):
        ctrl = (rng.normal(size=20) * 1.5).astype(np.float32)
        p = oracle_mod.constraint_problem(cmodel.cmodel, cfg, st[e, :27], st[e, 32:58], ctrl=ctrl,
                                          qaccw=st[e, 64:90])
        a_star = P.minimize(p)
        cg = P.cost_grad_fn(p)
        a = p["qacc"].astype(np.float64)
        c, g, scale = cg(a)
        c_star = cg(a_star)[0]
        assert np.abs(a - a_star).max() <= 1e-4 * max(1.0, np.abs(a_star).max()), e
        assert np.linalg.norm(g) <= 1e-5 * scale, e
        assert c - c_star <= 1e-6 * abs(c_star), e
        kinds += np.bincount(p["type"], minlength=3) > 0
    assert (kinds > 0).all(), kinds  # frictionloss, joint-limit and contact rows all exercised


def test_primal_helper_known_answer():
    """One dof, one contact row: a closed-form minimizer pins the helper itself."""
    p = dict(qM=np.array([[2.0]], np.float32), qacc_smooth=np.array([-1.0], np.float32),
             J=np.array([[1.0]], np.float32), D=np.array([6.0], np.float32), R=np.array([1 / 6.0], np.float32),
             aref=np.array([0.0], np.float32), floss=np.array([0.0], np.float32), type=np.array([2], np.int32))
    # minimize (a + 1)^2 + 3 a^2 for a < 0: a* = -1/4
    a = P.minimize(p)
    assert abs(a[0] + 0.25) < 1e-7


def test_oracle_cg_solution_is_the_minimizer(oracle_mod, cmodel):
    """The CG variant (mj_solCG: M^-1-preconditioned Polak-Ribiere, the same line search and
    termination; solver type [U]) converges to the same minimizer when given
    iterations (200 here; fp32 CG stalls a little above Newton's accuracy, hence 1e-3 / 1e-5), and
    with train.py's 8 iterations it never ends above the cost it started from."""
    cfg = default_config(solver="cg", iterations=200)
    cfg8 = default_config(solver="cg")
    st = P.states(oracle_mod, cmodel, cfg)
    rng = np.random.default_rng(1)
    gaps = []
    for e in range(st.shape[0]):
        ctrl = (rng.normal(size=20) * 1.5).astype(np.float32)
        p = oracle_mod.constraint_problem(cmodel.cmodel, cfg, st[e, :27], st[e, 32:58], ctrl=ctrl,
                                          qaccw=st[e, 64:90])
        a_star = P.minimize(p)
        cg = P.cost_grad_fn(p)
        c_star = cg(a_star)[0]
        a = p["qacc"].astype(np.float64)
        assert np.abs(a - a_star).max() <= 1e-3 * max(1.0, np.abs(a_star).max()), e
        assert cg(a)[0] - c_star <= 1e-5 * abs(c_star), e
        p8 = oracle_mod.constraint_problem(cmodel.cmodel, cfg8, st[e, :27], st[e, 32:58], ctrl=ctrl,
                                           qaccw=st[e, 64:90])
        c8 = cg(p8["qacc"].astype(np.float64))[0]
        c_ws = min(cg(st[e, 64:90].astype(np.float64))[0], cg(p["qacc_smooth"].astype(np.float64))[0])
        assert c8 <= c_ws + 1e-6 * abs(c_ws), e
        gaps.append((c8 - c_star) / abs(c_star))
    print(f"CG (8 iterations) cost above the minimum: median {np.median(gaps):.2e}, max {np.max(gaps):.2e}")
