"""Summarise rocprofv3 PMC counter CSVs for zb::step_kernel into profiles/.

    python scripts/pmc_summary.py --config c2 --envs 8192 \
        --fetch gpurun_out/pmc_fetch --write gpurun_out/pmc_write [--valu gpurun_out/pmc_valu]

Each directory holds the *_counter_collection.csv of one separate rocprofv3
--pmc pass over `bench.py --steps K` (FETCH_SIZE and WRITE_SIZE do not fit in
one TCC pass, MI355X_MICROARCH.md "rocprofv3 PMC slots"). Per launch of the
step kernel this reports:
  fetch_kb_raw / write_kb_raw   counter values (rocprofv3 reports KB units)
  hbm_bytes_per_launch          FETCH x2 (gfx950 correction: FETCH_SIZE counts
                                128-B requests at 64 B) + WRITE, in bytes
and, from the optional VALU pass, executed fp32 VALU instructions per launch
(wave-level) and the FLOP they issue (FMA = 2 x 64 lanes, ADD/MUL = 64 lanes).
Infinity-Cache hits are counted by FETCH_SIZE (guide, HBM section), so the
figure is an upper bound on DRAM bytes.
"""

from __future__ import annotations

import argparse
import csv
import glob
import json
import os
import statistics

KERNEL = "step_kernel"


def load(d: str) -> dict[str, list[float]]:
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection.csv under {d}")
    per: dict[tuple, dict[str, float]] = {}
    for fn in files:
        with open(fn, newline="") as f:
            for row in csv.DictReader(f):
                if KERNEL not in row["Kernel_Name"].split("(")[0]:
                    continue
                key = (fn, row["Dispatch_Id"])
                per.setdefault(key, {})
                per[key][row["Counter_Name"]] = per[key].get(row["Counter_Name"], 0.0) + float(row["Counter_Value"])
    out: dict[str, list[float]] = {}
    for vals in per.values():
        for k, v in vals.items():
            out.setdefault(k, []).append(v)
    return out


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c2")
    ap.add_argument("--envs", type=int, required=True)
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--write", required=True)
    ap.add_argument("--valu", default=None)
    ap.add_argument("--skip", type=int, default=2, help="drop the first launches (reset / warm-up)")
    ap.add_argument("--out", default=None)
    ap.add_argument("--kernel", default="step_kernel", help="kernel name substring (gae_kernel for the PPO leg)")
    ap.add_argument("--T", type=int, default=0, help="rollout length of a gae_kernel launch")
    ap.add_argument("--solver", default=None, help="the step kernel's solver (recorded; bench.py reads traffic only "
                                                   "for a matching --solver)")
    args = ap.parse_args()
    global KERNEL
    KERNEL = args.kernel

    def med(xs):
        xs = xs[args.skip:] if len(xs) > args.skip else xs
        return statistics.median(xs)

    fe = load(args.fetch)
    wr = load(args.write)
    fetch_kb = med(fe["FETCH_SIZE"])
    write_kb = med(wr["WRITE_SIZE"])
    hbm = 2.0 * fetch_kb * 1024.0 + write_kb * 1024.0
    res = {
        "kernel": "zb::" + args.kernel,
        "config": args.config,
        "envs": args.envs,
        "launches": len(fe["FETCH_SIZE"]),
        "fetch_kb_raw": fetch_kb,
        "write_kb_raw": write_kb,
        "hbm_bytes_per_launch": hbm,
        "hbm_bytes_per_env_step": hbm / args.envs,
        "correction": "FETCH_SIZE x2 (gfx950, MI355X_MICROARCH.md HBM section), WRITE_SIZE as read; "
                      "Infinity-Cache hits included (upper bound on DRAM bytes)",
    }
    if args.solver:
        res["solver"] = args.solver
    if args.T:
        res["T"] = args.T
        res["hbm_bytes_per_element"] = hbm / (args.T * args.envs)
    if args.valu:
        va = load(args.valu)
        fl = {}
        for name, mult in (("SQ_INSTS_VALU_FMA_F32", 128), ("SQ_INSTS_VALU_ADD_F32", 64),
                           ("SQ_INSTS_VALU_MUL_F32", 64), ("SQ_INSTS_VALU_TRANS_F32", 64)):
            if name in va:
                fl[name] = med(va[name])
        res["valu_insts_per_launch"] = {k: med(v) for k, v in va.items()}
        if "SQ_WAVES" in va:
            w = med(va["SQ_WAVES"])
            res["insts_per_wave"] = {k.replace("SQ_INSTS_", ""): med(v) / w for k, v in va.items() if k != "SQ_WAVES"}
        if fl:
            flop = sum(fl[k] * (128 if k.endswith("FMA_F32") else 64) for k in fl)
            res["issued_fp32_flop_per_launch"] = flop
            res["issued_fp32_flop_per_env_step"] = flop / args.envs
    out = args.out or os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles",
                                   f"pmc_traffic_{args.config}.json")
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
