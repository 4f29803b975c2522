"""Per-phase cycle shares of the step kernel from the -DZB_STAMPS diagnostic build.

    make -C ksim-gym-zbot_amd/csrc stamps && python tests/diag_stamps.py [--n 8192]

Stamps fence the pipeline (s_waitcnt around s_memtime), so read the SHARES,
not the absolute time (cdna_hip_programming.md §7, In-kernel stamps).
"""

import argparse
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ksim-gym-zbot_amd"))

import torch  # noqa: E402
from zbot_amd import compile_model, default_config  # noqa: E402
from zbot_amd.engine import HipEngine  # noqa: E402

PHASES = ["feetech", "kinematics", "com_crb_M", "factor_M", "rne_bias", "solve_smooth", "constraints",
          "nw_warmstart", "nw_update0", "nw_hessian0", "nw_solve0", "line_search", "update_constraint",
          "hessian_refactor", "newton_solve", "newton_check", "sensors", "integrate", "step_end(obs/reward/reset)",
          "forward_entry"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=8192)
    ap.add_argument("--steps", type=int, default=4)
    ap.add_argument("--out", default="")
    ap.add_argument("--lib", default="libzbot_hip_stamps.so")
    ap.add_argument("--nslots", type=int, default=20, help="stamp slots of the build (ZB_NSTAMP)")
    ap.add_argument("--solver", default="cg", choices=["cg", "newton"])
    ap.add_argument("--names", default="", help="names of the extra slots (scripts/stamp_probe.py)")
    args = ap.parse_args()
    NS = args.nslots
    if args.names:
        PHASES.extend(args.names.split(","))
    lib = os.path.join(ROOT, "ksim-gym-zbot_amd", "zbot_amd", args.lib)
    cm = compile_model()
    eng = HipEngine(cm, default_config(solver=args.solver), args.n, lib_path=lib)
    eng.L.zb_get_stamps.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p]
    eng.reset()
    bias = torch.tensor([cm.cmodel.joint_bias[i] for i in range(20)], device="cuda")
    tot = torch.zeros(NS, dtype=torch.float64)
    calls = torch.zeros(NS, dtype=torch.float64)
    for t in range(args.steps):
        eng.step(bias + 0.05 * torch.randn(args.n, 20, device="cuda"))
        buf = torch.zeros(args.n, NS, dtype=torch.int64, device="cuda")
        eng.L.zb_get_stamps(eng.h, buf.data_ptr(), eng._stream())
        torch.cuda.synchronize()
        b = buf.cpu()
        tot += (b & ((1 << 44) - 1)).double().sum(0)
        calls += (b >> 44).double().sum(0)
    share = tot / tot.sum()
    res = {PHASES[i]: round(float(share[i]) * 100, 2) for i in range(NS)}
    res["cycles_per_env_step"] = float(tot.sum() / (args.n * args.steps))
    res["calls_per_env_step"] = {PHASES[i]: round(float(calls[i]) / (args.n * args.steps), 2) for i in range(NS)}
    res["cycles_per_call"] = {PHASES[i]: round(float(tot[i] / max(calls[i], 1)), 0) for i in range(NS)}
    print(json.dumps(res, indent=1))
    if args.out:
        with open(args.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
