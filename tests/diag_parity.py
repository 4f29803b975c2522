"""Stage-by-stage GPU vs oracle diagnostics (run on a GPU box; prints a report).

    python tests/diag_parity.py [--n 64] [--steps 8]
"""

import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ksim-gym-zbot_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import oracle as O  # noqa: E402
import torch  # noqa: E402
from zbot_amd import compile_model, default_config  # noqa: E402
from zbot_amd import cstructs as cs  # noqa: E402
from zbot_amd.engine import DBG, HipEngine  # noqa: E402


def rel(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    d = np.abs(a - b)
    scale = np.maximum(np.abs(b), 1e-3)
    return float(d.max()), float((d / scale).max())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=16)
    ap.add_argument("--steps", type=int, default=8)
    ap.add_argument("--warm", type=int, default=20, help="oracle steps before comparing (contacts develop)")
    args = ap.parse_args()
    cm = compile_model()
    m = cm.cmodel
    cfg = default_config(solver="newton", obs_noise=True)
    n = args.n
    orc = O.OracleEnv(m, cfg, n, seed=7)
    orc.reset()
    for t in range(args.warm):
        orc.step(O.synthetic_actions(m, 7, n, 0, t))
    eng = HipEngine(cm, cfg, n, seed=7)
    nv, nb = m.nv, m.nbody

    # ---- stage check: debug forward on the oracle's states ----
    st = orc.state.copy()
    st[:, cs.S_QACCW:cs.S_QACCW + 32] = 0.0
    ctrl = O.synthetic_actions(m, 3, n, 0, 0, std=0.5) * 2.0  # arbitrary torques
    dbg = eng.debug_forward(torch.from_numpy(st), torch.from_numpy(ctrl)).cpu().numpy()
    worst = {}
    for e in range(n):
        ref = O.forward_debug(m, cfg, st[e, :27], st[e, 32:58], ctrl[e], precision="f64")
        g = dbg[e]
        qM = g[DBG["qM"]:DBG["qM"] + nv * nv].reshape(nv, nv)
        checks = dict(
            qM=(qM, ref["qM"]),
            bias=(g[DBG["bias"]:DBG["bias"] + nv], ref["qfrc_bias"]),
            qacc_smooth=(g[DBG["qacc_smooth"]:DBG["qacc_smooth"] + nv], ref["qacc_smooth"]),
            qacc=(g[DBG["qacc"]:DBG["qacc"] + nv], ref["qacc"]),
            xpos=(g[DBG["xpos"]:DBG["xpos"] + nb * 3].reshape(nb, 3), ref["xpos"]),
            cinert=(g[DBG["cinert"]:DBG["cinert"] + nb * 10].reshape(nb, 10), ref["cinert"]),
            cvel=(g[DBG["cvel"]:DBG["cvel"] + nb * 6].reshape(nb, 6), ref["cvel"]),
            touch=(g[DBG["misc"] + 2:DBG["misc"] + 4], ref["touch"]),
        )
        for k, (a, b) in checks.items():
            ad, rd = rel(a, b)
            if k not in worst or ad > worst[k][0]:
                worst[k] = (ad, rd, e)
        if e < 2:
            print(f"env {e}: nefc gpu={g[DBG['misc']]:.0f} oracle={ref['nefc']} ncon gpu={g[DBG['misc'] + 1]:.0f} "
                  f"oracle={ref['ncon']}")
    print("debug-forward stage errors vs fp64 oracle (max abs, max rel, env):")
    for k, v in worst.items():
        print(f"  {k:12s} abs={v[0]:.3e} rel={v[1]:.3e} env={v[2]}")

    # ---- one env-step from identical state ----
    eng.set_state(torch.from_numpy(orc.state.copy()))
    for t in range(args.steps):
        a = O.synthetic_actions(m, 7, n, 0, 100 + t)
        ref = orc.step(a)
        out = eng.step(torch.from_numpy(a).cuda())
        torch.cuda.synchronize()
        gs = eng.get_state().cpu().numpy()
        print(f"step {t}: qpos {rel(gs[:, :27], orc.state[:, :27])} qvel {rel(gs[:, 32:58], orc.state[:, 32:58])} "
              f"obs_actor {rel(out['obs_actor'].cpu().numpy(), ref['obs_actor'])} "
              f"critic {rel(out['obs_critic'].cpu().numpy(), ref['obs_critic'])} "
              f"reward {rel(out['reward'].cpu().numpy(), ref['reward'])} done "
              f"{int((out['done'].cpu().numpy() != ref['done']).sum())}")
        it = eng.solver_iters().cpu().numpy()
        print(f"   solver iters gpu mean={it.mean():.1f} oracle mean={orc.iters.mean():.1f}")
        # re-sync to keep comparing single-step errors
        eng.set_state(torch.from_numpy(orc.state.copy()))


if __name__ == "__main__":
    main()
