"""Per-env one-step errors, GPU vs the fp32 / fp64 oracles, for one test_one_step_parity case
(diagnostic): the worst envs with their reward-term errors and the pre-step contact counts.

    python scripts/diag_onestep.py [--push] [--randomize] [--solver newton]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "ksim-gym-zbot_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests"), ROOT]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--push", action="store_true")
    ap.add_argument("--randomize", action="store_true")
    ap.add_argument("--solver", default="newton")
    ap.add_argument("--tol", type=float, default=None, help="solver tolerance of the GPU and fp32 oracle runs")
    a = ap.parse_args()
    import numpy as np
    import torch

    import oracle as O
    from zbot_amd import compile_model, default_config
    from zbot_amd.engine import DBG, HipEngine

    O.build()
    cm = compile_model()
    cfg = default_config(push=a.push, randomize=a.randomize, solver=a.solver)
    if a.tol is not None:
        cfg.tolerance = a.tol
    n = 64
    env = O.OracleEnv(cm.cmodel, cfg, n, seed=7)
    env.reset()
    for t in range(12):
        env.step(O.synthetic_actions(cm.cmodel, 7, n, 0, t, std=0.05))
    eng = HipEngine(cm, cfg, n, seed=7)
    for t in range(3):
        st0, rd0 = env.state.copy(), env.rand.copy()
        eng.set_state(torch.from_numpy(st0.copy()))
        eng.set_rand(torch.from_numpy(rd0.copy()))
        act = O.synthetic_actions(cm.cmodel, 7, n, 0, 100 + t)
        e64 = O.OracleEnv(cm.cmodel, cfg, n, seed=7, precision="f64")
        e64.state[:] = st0
        e64.rand[:] = rd0
        r64 = e64.step(act)
        ref = env.step(act)
        out = eng.step(torch.from_numpy(act).cuda())
        torch.cuda.synchronize()
        gs = eng.get_state().cpu().numpy()
        gi = eng.solver_iters().cpu().numpy()
        eq = np.abs(gs[:, :27] - env.state[:, :27]).max(1)
        gap = np.abs(env.state[:, :27] - e64.state[:, :27]).max(1)
        er = np.abs(out["reward"].cpu().numpy() - ref["reward"])
        et = np.abs(out["reward_terms"].cpu().numpy() - ref["reward_terms"])
        dbg = eng.debug_forward(torch.from_numpy(st0), torch.zeros(n, 20)).cpu().numpy()
        print(f"step {t}: max qpos err {eq.max():.2e}, reward {er.max():.2e}")
        for e in np.argsort(eq)[-4:][::-1]:
            fd = O.forward_debug(cm.cmodel, cfg, st0[e, :27], st0[e, 32:58], None, precision="f32")
            print(f"  env {e}: qpos err {eq[e]:.2e} (f32/f64 gap {gap[e]:.2e}), reward err {er[e]:.2e}, "
                  f"terms err {np.array2string(et[e], precision=1)}, done {int(ref['done'][e])}, "
                  f"pre-step ncon gpu {int(dbg[e, DBG['misc'] + 1])} oracle {fd['ncon']}, "
                  f"nefc gpu {int(dbg[e, DBG['misc']])} oracle {fd['nefc']}, iters gpu {int(gi[e])} oracle f32 "
                  f"{int(env.iters[e])} f64 {int(e64.iters[e])}")


if __name__ == "__main__":
    main()
