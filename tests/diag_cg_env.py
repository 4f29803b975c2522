"""Where a CG one-step outlier parts from the oracle (diagnostic, GPU).

    python tests/diag_cg_env.py --env 63 [--push 1 --randomize 1] [--t 0]

The one-step parity states (tests/test_gpu_parity.py: 64 envs warmed 12 steps; --t control steps
further), then for k = 1..20 physics substeps (ctrl_dt = k dt): the engine, the fp32 oracle and the
fp64 oracle from the same state, the env's qpos / qvel differences and solver iteration counts.
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
from test_gpu_parity import warm_states  # noqa: E402
from zbot_amd import compile_model, default_config  # noqa: E402
from zbot_amd.engine import HipEngine  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--env", type=int, action="append", required=True)
    ap.add_argument("--push", type=int, default=1)
    ap.add_argument("--randomize", type=int, default=1)
    ap.add_argument("--t", type=int, default=0)
    ap.add_argument("--solver", default="cg")
    ap.add_argument("--eulerdamp", action="store_true")
    a = ap.parse_args()
    cm = compile_model()
    kw = dict(push=bool(a.push), randomize=bool(a.randomize), solver=a.solver, eulerdamp=a.eulerdamp)
    cfg = default_config(**kw)
    n = 64
    env = warm_states(O, cm, cfg, n, steps=12)
    for t in range(a.t):
        env.step(O.synthetic_actions(cm.cmodel, 7, n, 0, 100 + t))
    act = O.synthetic_actions(cm.cmodel, 7, n, 0, 100 + a.t)
    for k in range(1, 21):
        ck = default_config(**kw, ctrl_dt=0.001 * k)
        e32 = O.OracleEnv(cm.cmodel, ck, n, seed=7)
        e64 = O.OracleEnv(cm.cmodel, ck, n, seed=7, precision="f64")
        for e in (e32, e64):
            e.state[:] = env.state
            e.rand[:] = env.rand
            e.step(act)
        eng = HipEngine(cm, ck, n, seed=7)
        eng.set_state(torch.from_numpy(env.state.copy()))
        eng.set_rand(torch.from_numpy(env.rand.copy()))
        eng.step(torch.from_numpy(act).cuda(), extras=False)
        torch.cuda.synchronize()
        gs = eng.get_state().cpu().numpy()
        gi = eng.solver_iters().cpu().numpy()
        for w in a.env:
            dq32 = np.abs(gs[w, :27] - e32.state[w, :27]).max()
            dq64 = np.abs(gs[w, :27] - e64.state[w, :27]).max()
            gap = np.abs(e32.state[w, :27] - e64.state[w, :27]).max()
            dv32 = np.abs(gs[w, 32:58] - e32.state[w, 32:58]).max()
            gapv = np.abs(e32.state[w, 32:58] - e64.state[w, 32:58]).max()
            print(f"env {w} substeps {k:2d}: |q-q32| {dq32:.2e} |q-q64| {dq64:.2e} gap {gap:.2e} | |v-v32| {dv32:.2e} "
                  f"gapv {gapv:.2e} | iters engine {int(gi[w])} f32 {int(e32.iters[w])} f64 {int(e64.iters[w])}")


if __name__ == "__main__":
    main()
