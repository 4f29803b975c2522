"""fp32 against fp64 oracle along a rollout from reset (every step the fp64 oracle takes one step from
the fp32 oracle's state): per step, how many envs' rewards part by more than 1e-5, and the largest
gap. Diagnostic for the collider variants (tests/collider_util.py).

    python scripts/oracle_gap.py mjx_box_desc [steps]
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "ksim-gym-zbot_amd"), os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle")]
import collider_util as U  # noqa: E402
import oracle as O  # noqa: E402
from zbot_amd import compile_model, default_config  # noqa: E402

cm = compile_model(getattr(U, sys.argv[1])())
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 12
cfg = default_config(solver="newton", push=True)
n, seed = 64, 13
acts = np.stack([O.synthetic_actions(cm.cmodel, seed, n, 0, t, std=0.5) for t in range(steps)])
e32 = O.OracleEnv(cm.cmodel, cfg, n, seed=seed)
e64 = O.OracleEnv(cm.cmodel, cfg, n, seed=seed, precision="f64")
e32.reset()
print(f"# {sys.argv[1]}: fp32 vs fp64 oracle, {n} envs, pushes, action std 0.5, seed {seed} "
      "(the GPU rollout test's workload): step, envs with |reward gap| > 1e-5, max gap")
for t in range(steps):
    e64.state[:] = e32.state
    e64.rand[:] = e32.rand
    r64 = e64.step(acts[t])["reward"].copy()
    r32 = e32.step(acts[t])["reward"].copy()
    d = np.abs(r64 - r32)
    print(t, int((d > 1e-5).sum()), float(d.max()))
