"""Algorithmic FLOPs per env-step from the counting build of the CPU twin.

    python scripts/count_flops.py [--envs 64] [--steps 40] [--out profiles/flops_c2.json]

oracle/zb_flops.cpp compiles the fp32 oracle with every arithmetic operation of its physics
counted (FMA = 2: a multiply and an add). Two runs of the C2 workload (the standing task,
JOINT_BIASES + 0.05 N(0, 1) actions, Newton 8 / 8):
  * "as run": the solver's own early exits (tolerance 1e-8, ls_tolerance 0.01), the work the
    engine does per env-step;
  * "fixed iterations": tolerance and ls_tolerance set to -1, so every Newton solve runs its 8
    iterations and every line search its 8 evaluations unless the step vanishes (alpha = 0) —
    SURVEY §8(d)'s "fixed iteration counts".
Counts are per env-step after a 20-step warm-up from reset; compares are reported apart and
not included in the FLOPs.
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "ksim-gym-zbot_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import oracle as O  # noqa: E402
from zbot_amd import compile_model, default_config  # noqa: E402


def count(cm, cfg, n, steps, warm=20, seed=3):
    L = O.lib("flops")
    env = O.OracleEnv(cm.cmodel, cfg, n, seed=seed, precision="flops")
    env.reset()
    for t in range(warm):
        env.step(O.synthetic_actions(cm.cmodel, seed, n, 0, t))
    L.zbo_flops_reset()
    iters = 0
    for t in range(warm, warm + steps):
        env.step(O.synthetic_actions(cm.cmodel, seed, n, 0, t))
        iters += int(env.iters.sum())
    out = (np.ctypeslib.ctypes.c_uint64 * 6)()
    L.zbo_flops_get(out)
    add, mul, div, sqrt, trans, cmp = (int(x) for x in out)
    es = n * steps
    flops = add + mul + div + sqrt + trans
    return dict(env_steps=es, flops_per_env_step=flops / es, add=add / es, mul=mul / es, div=div / es,
                sqrt=sqrt / es, transcendental=trans / es, compares=cmp / es,
                newton_iters_per_env_step=iters / es)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=64)
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--out", default="")
    ap.add_argument("--solver", default="newton", choices=["newton", "cg"])
    ap.add_argument("--eulerdamp", action="store_true", help="mj_Euler's implicit joint damping (ZB_F_EULERDAMP)")
    ap.add_argument("--box-rule", default="mujoco", choices=["mujoco", "mjx"],
                    help="compile_model(box_rule=...): the soles by MJX's plane_convex manifold")
    ap.add_argument("--sole-pair", action="store_true",
                    help="the sole-pair model: the two box soles also collide with each other (DESIGN.md §4l)")
    args = ap.parse_args()
    if args.sole_pair:
        from zbot_amd.model import load_description  # noqa: PLC0415

        desc = load_description()
        desc["self_pairs"] = [["left_foot_sole", "right_foot_sole"]]
        cm = compile_model(desc, box_rule=args.box_rule)
    else:
        cm = compile_model(box_rule=args.box_rule)
    res = {"workload": f"C2 standing task, {args.envs} envs x {args.steps} env-steps after 20 warm-up steps, "
                       f"JOINT_BIASES + 0.05 N(0,1) actions (zbo_synthetic_actions), {args.solver} 8 / 8"
                       + (", implicit joint damping (eulerdamp)" if args.eulerdamp else "")
                       + (", box soles by MJX's plane_convex (box_rule mjx)" if args.box_rule == "mjx" else "")
                       + (", sole-pair model (the soles collide with each other)" if args.sole_pair else ""),
           "note": "FMA counted as a multiply and an add; compares listed apart and not in the FLOPs",
           "solver": args.solver, "eulerdamp": args.eulerdamp, "box_rule": args.box_rule,
           "sole_pair": args.sole_pair}
    res["as_run"] = count(cm, default_config(solver=args.solver, eulerdamp=args.eulerdamp), args.envs, args.steps)
    fixed = default_config(solver=args.solver, eulerdamp=args.eulerdamp)
    fixed.tolerance = -1.0
    fixed.ls_tolerance = -1.0
    res["fixed_iterations"] = count(cm, fixed, args.envs, args.steps)
    print(json.dumps(res, indent=1))
    if args.out:
        with open(args.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
