"""MuJoCo's primal constrained-acceleration problem, restated in float64 numpy (test helper).

For one forward pass (oracle.constraint_problem): minimize over the acceleration a
    c(a) = 1/2 (a - a0)' M (a - a0) + sum_r s_r(J_r a - aref_r)
with a0 = qacc_smooth and, per row (mj_constraintUpdate's cost; oracle efc_eval):
  contact pyramid edge / joint limit:  s = 1/2 D x^2 for x < 0, else 0
  frictionloss (Huber, Rf = R floss):  x <= -Rf: -floss (Rf/2 + x);  x >= Rf: floss (x - Rf/2);
                                       else 1/2 D x^2
The gradient is M (a - a0) - J' f with f = -ds/dx. The minimizer found here by scipy's BFGS is
independent of the Newton solver (line search, Hessian factorization, active-set updates) that
the oracle and the HIP engine run.
"""

import numpy as np


def cost_grad_fn(p: dict):
    M = p["qM"].astype(np.float64)
    a0 = p["qacc_smooth"].astype(np.float64)
    J = p["J"].astype(np.float64)
    D = p["D"].astype(np.float64)
    R = p["R"].astype(np.float64)
    aref = p["aref"].astype(np.float64)
    fl = p["floss"].astype(np.float64)
    fr = p["type"] == 0

    def cg(a):
        da = a - a0
        Mda = M @ da
        x = J @ a - aref
        Rf = R * fl
        lo = fr & (x <= -Rf)
        hi = fr & (x >= Rf)
        quad = (fr & ~lo & ~hi) | (~fr & (x < 0))
        c = 0.5 * da @ Mda + np.sum(0.5 * D[quad] * x[quad] ** 2)
        c += np.sum(-fl[lo] * (0.5 * Rf[lo] + x[lo])) + np.sum(fl[hi] * (x[hi] - 0.5 * Rf[hi]))
        f = np.zeros_like(x)
        f[quad] = -D[quad] * x[quad]
        f[lo] = fl[lo]
        f[hi] = -fl[hi]
        Jf = J.T @ f
        return c, Mda - Jf, np.linalg.norm(Mda) + np.linalg.norm(Jf)

    return cg


def minimize(p: dict) -> np.ndarray:
    from scipy.optimize import minimize as sp_min

    cg = cost_grad_fn(p)
    res = sp_min(lambda a: cg(a)[:2], p["qacc_smooth"].astype(np.float64), jac=True, method="BFGS",
                 options=dict(gtol=1e-10, maxiter=20000))
    return res.x


def states(O, cm, cfg, n: int = 12, seed: int = 3):
    """Warm oracle states (standing on the sole contacts), a third pressed into the floor, a third
    with a knee past its lower limit and fast joints (limit rows)."""
    env = O.OracleEnv(cm.cmodel, cfg, n, seed=seed)
    env.reset()
    for t in range(24):
        env.step(O.synthetic_actions(cm.cmodel, seed, n, 0, t))
    st = env.state.copy()
    k = n // 3
    st[k:2 * k, 2] -= 0.003
    st[2 * k:, 7 + 3] = -2.3
    rng = np.random.default_rng(seed)
    st[2 * k:, 32 + 6:32 + 26] += rng.normal(scale=1.5, size=(n - 2 * k, 20)).astype(np.float32)
    return st
