"""Why CG's one-step contract is wider than Newton's, measured on the oracle alone:
the fp32 and fp64 oracles stepped from the same 64 warm states (test_gpu_parity's one-step states),
per solver, iteration cap and tolerances; counts of envs whose fp32 / fp64 qvel gap exceeds Newton's
qvel bound (2e-5), per step, and the gap's median / max. Writes profiles/r05_cg_sensitivity.json.

    python scripts/cg_sensitivity.py
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "ksim-gym-zbot_amd"), os.path.join(ROOT, "oracle")]
import oracle as O  # noqa: E402
from zbot_amd import compile_model, default_config  # noqa: E402


def run(cm, solver, iters, tol, ls_tol, n=64):
    cfg = default_config(solver=solver)
    cfg.iterations, cfg.tolerance, cfg.ls_tolerance = iters, tol, ls_tol
    env = O.OracleEnv(cm.cmodel, cfg, n, seed=7)
    env.reset()
    for t in range(12):
        env.step(O.synthetic_actions(cm.cmodel, 7, n, 0, t, std=0.05))
    gaps = []
    for t in range(3):
        e64 = O.OracleEnv(cm.cmodel, cfg, n, seed=7, precision="f64")
        e64.state[:] = env.state
        e64.rand[:] = env.rand
        a = O.synthetic_actions(cm.cmodel, 7, n, 0, 100 + t)
        e64.step(a)
        env.step(a)
        gaps.append(np.abs(e64.state[:, 32:58] - env.state[:, 32:58]).max(1))
    g = np.array(gaps)
    return {"solver": solver, "iterations": iters, "tolerance": tol, "ls_tolerance": ls_tol,
            "envs_over_newton_qvel_bound_per_step": [int((x > 2e-5).sum()) for x in g],
            "median_qvel_gap": float(np.median(g)), "max_qvel_gap": float(g.max())}


def main():
    cm = compile_model()
    rows = [run(cm, *a) for a in [("newton", 8, 1e-8, 0.01), ("newton", 32, 0.0, 0.0), ("cg", 8, 1e-8, 0.01),
                                   ("cg", 8, 0.0, 0.01), ("cg", 8, 1e-8, 0.0), ("cg", 8, 0.0, 0.0),
                                   ("cg", 16, 1e-8, 0.01), ("cg", 32, 1e-8, 0.01), ("cg", 100, 1e-8, 0.01)]]
    for r in rows:
        print(r)
    with open(os.path.join(ROOT, "profiles", "r05_cg_sensitivity.json"), "w") as f:
        json.dump({"what": __doc__.strip().splitlines()[0], "states": "64 envs, 12 warm steps (seed 7), 3 steps",
                   "rows": rows}, f, indent=1)


if __name__ == "__main__":
    main()
