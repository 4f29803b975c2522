"""Per-step divergence of one env of the C1 golden rollout, engine vs the fp32 / fp64 oracles
(diagnostic for the env that needs test_golden_rollout's budget).

From the same reset and the fixture's actions, every step sets the engine to the fp32 oracle's
pre-step state (so each line is a one-step comparison along the oracle's own trajectory) and
prints, for the chosen env: qpos / qvel / planner errors, the joint with the largest qpos error,
the pre-step contact and row counts (engine and oracle), and the solver iterations.

    python scripts/diag_c1_env.py [--env 35] [--steps 8] [--tol 1e-8]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "ksim-gym-zbot_amd"), os.path.join(ROOT, "oracle"), ROOT]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--env", type=int, default=35)
    ap.add_argument("--steps", type=int, default=8)
    ap.add_argument("--tol", type=float, default=None)
    a = ap.parse_args()
    import numpy as np
    import torch

    import oracle as O
    from zbot_amd import compile_model, cstructs as cs, default_config
    from zbot_amd.engine import DBG, HipEngine

    O.build()
    g = dict(np.load(os.path.join(ROOT, "tests", "golden", "c1_64x128_seed0.npz")))
    n, seed = int(g["cfg_n"]), int(g["cfg_seed"])
    cm = compile_model()
    cfg = default_config(solver="newton")
    if a.tol is not None:
        cfg.tolerance = a.tol
    e32 = O.OracleEnv(cm.cmodel, cfg, n, seed=seed)
    e64 = O.OracleEnv(cm.cmodel, cfg, n, seed=seed, precision="f64")
    e32.reset()
    e64.reset()
    eng = HipEngine(cm, cfg, n, seed=seed)
    eng.reset()
    e = a.env
    P0, P1 = cs.S_PLAN_POS, cs.S_PLAN_TAU + 20
    for t in range(a.steps):
        st0 = e32.state.copy()
        eng.set_state(torch.from_numpy(st0.copy()))
        act = g["actions"][t]
        e64.state[:] = st0
        r64 = e64.step(act)
        r32 = e32.step(act)
        out = eng.step(torch.from_numpy(act).cuda())
        torch.cuda.synchronize()
        gs = eng.get_state().cpu().numpy()
        gi = eng.solver_iters().cpu().numpy()
        dq = np.abs(gs[e, :27] - e32.state[e, :27])
        dv = np.abs(gs[e, 32:58] - e32.state[e, 32:58]).max()
        dp = np.abs(gs[e, P0:P1] - e32.state[e, P0:P1])
        gap = np.abs(e32.state[e, :27] - e64.state[e, :27]).max()
        dbg = eng.debug_forward(torch.from_numpy(st0), torch.zeros(n, 20)).cpu().numpy()
        fd = O.forward_debug(cm.cmodel, cfg, st0[e, :27], st0[e, 32:58], None, precision="f32")
        dr = float(out["reward"][e]) - float(r32["reward"][e])
        print(f"step {t}: qpos err {dq.max():.2e} (dof {int(dq.argmax())}), qvel {dv:.2e}, planner pos/vel/tau "
              f"{dp[:20].max():.2e}/{dp[20:40].max():.2e}/{dp[40:].max():.2e} (slot {int(dp.argmax())}), "
              f"f32/f64 gap {gap:.2e}, reward err {dr:.2e} (f64 {float(r64['reward'][e]) - float(r32['reward'][e]):.2e}), "
              f"ncon gpu {int(dbg[e, DBG['misc'] + 1])} oracle {fd['ncon']}, nefc gpu {int(dbg[e, DBG['misc']])} "
              f"oracle {fd['nefc']}, iters gpu {int(gi[e])} oracle {int(e32.iters[e])} f64 {int(e64.iters[e])}",
              flush=True)


if __name__ == "__main__":
    main()
