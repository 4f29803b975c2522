"""Distribution of the CG one-step error against each env's fp32/fp64 oracle gap (diagnostic, GPU).

    python tests/diag_cg_contract.py [--eulerdamp] [--model limbs|cyl|mesh|pair] [--solver cg|newton]

For the one-step parity states (tests/test_gpu_parity.py: 64 envs warmed 12 steps, then 3 steps from
identical states), per output and step: the engine's |error| against the fp32 oracle and against the
fp64 oracle, the fp32/fp64 oracle gap, and how many envs exceed Newton's bound + k x gap for k = 1,
2, 3, 4 in both forms. This is what the CG contract (test_gpu_parity.py CG_CONTRACT) is chosen from.
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ksim-gym-zbot_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

import torch  # noqa: E402
import oracle as O  # noqa: E402
from test_gpu_parity import ONE_STEP_TOL, one_step_outputs, oracle_steps, warm_states  # noqa: E402
from zbot_amd import compile_model, default_config  # noqa: E402
from zbot_amd.engine import HipEngine  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--eulerdamp", action="store_true")
    ap.add_argument("--solver", default="cg")
    ap.add_argument("--push", type=int, default=1)
    ap.add_argument("--randomize", type=int, default=1)
    a = ap.parse_args()
    cm = compile_model()
    cfg = default_config(push=bool(a.push), randomize=bool(a.randomize), solver=a.solver, eulerdamp=a.eulerdamp)
    n = 64
    env = warm_states(O, cm, cfg, n, steps=12)
    eng = HipEngine(cm, cfg, n, seed=7)
    ks = (1, 2, 3, 4)
    for t in range(3):
        eng.set_state(torch.from_numpy(env.state.copy()))
        eng.set_rand(torch.from_numpy(env.rand.copy()))
        act = O.synthetic_actions(cm.cmodel, 7, n, 0, 100 + t)
        # the step's sensitivity to a rounding-level input change: the fp32 oracle from the state with
        # qvel scaled by 1 +- 2^-23 per component (3 draws), the largest output change per env
        pert = []
        rng = np.random.default_rng(100 + t)
        for _ in range(3):
            ep = O.OracleEnv(cm.cmodel, cfg, n, seed=7)
            ep.state[:] = env.state
            ep.rand[:] = env.rand
            sgn = rng.choice([-1.0, 1.0], size=(n, 26)).astype(np.float32)
            ep.state[:, 32:58] *= (1.0 + sgn * np.float32(2.0 ** -23))
            rp = ep.step(act)
            pert.append({k: want for k, _, want in one_step_outputs(ep.state, rp, ep.state, rp)})
        ref, ref64 = oracle_steps(O, cm, cfg, env, act, 7)
        out = eng.step(torch.from_numpy(act).cuda())
        torch.cuda.synchronize()
        gs = eng.get_state().cpu().numpy()
        for key, got, want in one_step_outputs(gs, out, env.state, ref):
            got = np.asarray(got, np.float64).reshape(n, -1)
            w32 = np.asarray(want, np.float64).reshape(n, -1)
            w64 = np.asarray(ref64[key], np.float64).reshape(n, -1)
            tol = ONE_STEP_TOL[key][0]
            gap = np.abs(w32 - w64).max(1)
            pg = np.max([np.abs(np.asarray(pp[key], np.float64).reshape(n, -1) - w32).max(1) for pp in pert], axis=0)
            sens = np.maximum(gap, pg)
            overs = [int((np.abs(got - w32).max(1) > tol + k * sens).sum()) for k in ks]
            e32 = np.abs(got - w32).max(1)
            e64 = np.abs(got - w64).max(1)
            over32 = [int((e32 > tol + k * gap).sum()) for k in ks]
            over64 = [int((e64 > tol + k * gap).sum()) for k in ks]
            ratio = np.max((e64 - tol) / np.maximum(gap, 1e-30))
            print(f"step {t} {key:12s} tol {tol:.0e} | max e32 {e32.max():.2e} e64 {e64.max():.2e} gap {gap.max():.2e} "
                  f"| over tol+k*gap vs f32 {over32} vs f64 {over64} | worst (e64-tol)/gap {ratio:.2f} "
                  f"| envs e64>tol+2gap {np.flatnonzero(e64 > tol + 2 * gap).tolist()[:8]} | pert {pg.max():.2e} over tol+k*sens vs f32 {overs} "
                  f"envs {np.flatnonzero(e32 > tol + 2 * sens).tolist()[:8]}")


if __name__ == "__main__":
    main()
