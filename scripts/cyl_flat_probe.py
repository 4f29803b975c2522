"""fp32 vs fp64 oracle on the cylinder-foot variant (tests/collider_util.py cyl_desc), CPU only
(diagnostic). A disk resting flat on the floor is a discontinuity of MuJoCo's plane-cylinder rule:
the contact triangle turns with the direction of a vanishing tilt. Prints, per env-step, how far the
two precisions' qpos apart after one step from the same state: (1) from the reset pose (the
cylinder foot exactly upright), (2) from the touching states of tests/test_gpu_colliders.py, where
the foot lands flat in the first step, with the limbs variant (boxes, capsule) beside it, and the
solver iterations of both precisions over that step.

    python scripts/cyl_flat_probe.py
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "ksim-gym-zbot_amd"), os.path.join(ROOT, "oracle")]
import collider_util as U  # noqa: E402
import oracle as O  # noqa: E402
from test_gpu_colliders import contact_env  # noqa: E402
from test_gpu_parity import oracle_steps  # noqa: E402
from zbot_amd import compile_model, default_config  # noqa: E402


def gap(env, ref64):
    g = np.abs(env.state[:, :27] - ref64["qpos"]).max(1)
    return f"qpos gap max {g.max():.1e}, envs > 1e-6: {(g > 1e-6).sum()} of {len(g)}"


def main():
    cfg = default_config(solver="newton")
    for name in ("limbs", "cyl"):
        cm = compile_model(getattr(U, name + "_desc")())
        env = O.OracleEnv(cm.cmodel, cfg, 16, seed=3)
        env.reset()
        for t in range(4):
            _, ref64 = oracle_steps(O, cm, cfg, env, O.synthetic_actions(cm.cmodel, 3, 16, 0, t), 3)
            print(f"{name} from reset, step {t}: {gap(env, ref64)}")
        env = contact_env(O, cm, cfg, 64, seed=11)
        for t in range(3):
            _, ref64 = oracle_steps(O, cm, cfg, env, O.synthetic_actions(cm.cmodel, 11, 64, 0, t), 11)
            it32, it64 = env.iters, ref64["_iters"]
            print(f"{name} from touching states, step {t}: {gap(env, ref64)}; solver iterations over the step "
                  f"fp32 {int(it32.min())}-{int(it32.max())}, fp64 {int(it64.min())}-{int(it64.max())}")


if __name__ == "__main__":
    main()
