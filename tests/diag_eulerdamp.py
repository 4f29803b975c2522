"""Diagnostic (GPU box): where the implicit-damping step of one env parts from the oracle. Rebuilds the
one-step parity states (test_gpu_parity warm_states, seed 7, two one-step iterations), then runs the
third control step as 20 single-substep steps (ctrl_dt = dt) on the engine and the fp32 / fp64
oracles, re-synchronising the engine to the fp32 oracle after every substep, and prints per substep
the envs whose qvel increment (dt x the implicit qacc) differs most, with the solver iteration counts.

    python tests/diag_eulerdamp.py [eulerdamp 0|1] [env]
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "ksim-gym-zbot_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]
import torch  # noqa: E402

import oracle as O  # noqa: E402
from zbot_amd import compile_model, cstructs as cs, default_config  # noqa: E402
from zbot_amd.engine import HipEngine  # noqa: E402

ed = bool(int(sys.argv[1])) if len(sys.argv) > 1 else True
watch = int(sys.argv[2]) if len(sys.argv) > 2 else 23
cm = compile_model()
n = 64
cfg = default_config(solver="newton", eulerdamp=ed)
env = O.OracleEnv(cm.cmodel, cfg, n, seed=7)
env.reset()
for t in range(12):
    env.step(O.synthetic_actions(cm.cmodel, 7, n, 0, t, std=0.05))
for t in range(2):
    env.step(O.synthetic_actions(cm.cmodel, 7, n, 0, 100 + t))
a = O.synthetic_actions(cm.cmodel, 7, n, 0, 102)
c1 = default_config(solver="newton", eulerdamp=ed, ctrl_dt=0.001)
o32 = O.OracleEnv(cm.cmodel, c1, n, seed=7)
o64 = O.OracleEnv(cm.cmodel, c1, n, seed=7, precision="f64")
o32.state[:] = env.state
o32.rand[:] = env.rand
eng = HipEngine(cm, c1, n, seed=7)
eng.set_rand(torch.from_numpy(env.rand.copy()))
for ss in range(20):
    st = o32.state.copy()
    o64.state[:] = st
    o64.rand[:] = o32.rand
    eng.set_state(torch.from_numpy(st))
    eng.step(torch.from_numpy(a).cuda())
    g = eng.get_state().cpu().numpy()
    o64.step(a)
    o32.step(a)
    dv = np.abs(g[:, 32:58] - o32.state[:, 32:58]).max(1)
    d64 = np.abs(o64.state[:, 32:58] - o32.state[:, 32:58]).max(1)
    dq = np.abs(g[:, cs.S_QACCW:cs.S_QACCW + 26] - o32.state[:, cs.S_QACCW:cs.S_QACCW + 26]).max(1)
    it_g = eng.solver_iters().cpu().numpy()
    print(f"substep {ss:2d}: env {watch}: qvel err {dv[watch]:.2e} (fp64 gap {d64[watch]:.2e}), qacc err {dq[watch]:.2e}, "
          f"iters engine {it_g[watch]} oracle {o32.iters[watch]} f64 {o64.iters[watch]}; worst env {int(dv.argmax())} "
          f"{dv.max():.2e} (gap {d64[dv.argmax()]:.2e})")

# the substep with the largest error on the watched env, replayed with the damping switch on and off
worst = None
o32 = O.OracleEnv(cm.cmodel, c1, n, seed=7)
o32.state[:] = env.state
o32.rand[:] = env.rand
errs = []
for ss in range(20):
    st = o32.state.copy()
    eng.set_state(torch.from_numpy(st))
    eng.step(torch.from_numpy(a).cuda())
    g = eng.get_state().cpu().numpy()
    o32.step(a)
    errs.append((np.abs(g[watch, 32:58] - o32.state[watch, 32:58]).max(), ss, st))
_, ss, st = max(errs, key=lambda e: e[0])
np.set_printoptions(precision=5, suppress=True, linewidth=200)
print(f"replaying substep {ss}: touch {st[watch, cs.S_TOUCH:cs.S_TOUCH + 2]} prev contact "
      f"{st[watch, cs.S_PREV_CONT:cs.S_PREV_CONT + 2]} qpos z {st[watch, 2]:.5f}")
for e2 in (ed, not ed):
    c2 = default_config(solver="newton", eulerdamp=e2, ctrl_dt=0.001)
    oo = O.OracleEnv(cm.cmodel, c2, n, seed=7)
    oo.state[:] = st
    oo.rand[:] = o32.rand
    ee = HipEngine(cm, c2, n, seed=7)
    ee.set_rand(torch.from_numpy(oo.rand.copy()))
    ee.set_state(torch.from_numpy(st))
    ee.step(torch.from_numpy(a).cuda())
    oo.step(a)
    g = ee.get_state().cpu().numpy()
    qa_g = g[watch, cs.S_QACCW:cs.S_QACCW + 26]
    qa_o = oo.state[watch, cs.S_QACCW:cs.S_QACCW + 26]
    print(f"eulerdamp {int(e2)}: iters engine {ee.solver_iters().cpu().numpy()[watch]} oracle {oo.iters[watch]}")
    print("  engine qacc", qa_g)
    print("  oracle qacc", qa_o)
    print("  diff       ", qa_g - qa_o)
ctrl = st[:, cs.S_PLAN_TAU:cs.S_PLAN_TAU + 20].copy()
dbg = eng.debug_forward(torch.from_numpy(st), torch.from_numpy(ctrl)).cpu().numpy()[watch]
qa_e = dbg[1088:1088 + 26]
print(f"engine forward at the replayed state (ctrl = planner tau): nefc {int(dbg[1728])} ncon {int(dbg[1729])}")
print("  engine qacc", qa_e)
for prec in ("f32", "f64"):
    fd = O.forward_debug(cm.cmodel, c1, st[watch, :27], st[watch, 32:58], ctrl[watch], precision=prec)
    print(f"{prec} oracle forward: ncon {fd['ncon']} nefc {fd['nefc']}; engine - oracle qacc max "
          f"{np.abs(qa_e - fd['qacc']).max():.3e}")
    print("  oracle qacc", fd["qacc"])
