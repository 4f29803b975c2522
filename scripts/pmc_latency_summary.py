"""Summarise scripts/pmc_latency.sh: per (solver, env count), the step kernel's SQ counters per wave
per launch (median over the step launches after the first two) and per physics substep, with the
issue floor: the quad-cycles a wave spends issuing (SQ_ACTIVE_INST_ANY), i.e. the wave's lifetime if
every dependency were already satisfied. latency_frac = issue floor / wave lifetime; lifetime / floor =
how much longer than its own instruction stream the wave lives (dependent chains: LDS round trips,
DPP / permlane stages, transcendental latencies, s_waitcnt; at 8192 envs also the partner wave's issue).

    python scripts/pmc_latency_summary.py gpurun_out/pmclat > gpurun_out/pmc_latency.json
"""
import csv
import glob
import json
import statistics
import sys

prefix = sys.argv[1]
SUBSTEPS = 20
out = {"note": __doc__.split("\n\n")[0].replace("\n", " "), "units": "quad-cycles (SQ counters count 4 shader cycles)"}
for d in sorted(glob.glob(prefix + "_*")):
    if d.endswith(".log"):
        continue
    tag = d[len(prefix) + 1:]
    per = {}
    for fn in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for row in csv.DictReader(open(fn)):
            if "step_kernel" not in row["Kernel_Name"]:
                continue
            per.setdefault(row["Dispatch_Id"], {}).setdefault(row["Counter_Name"], 0.0)
            per[row["Dispatch_Id"]][row["Counter_Name"]] += float(row["Counter_Value"])
    ks = sorted(per, key=int)[2:]
    if not ks:
        continue
    v = {c: statistics.median(per[k][c] for k in ks) for c in per[ks[0]]}
    w = v.pop("SQ_WAVES")
    pw = {c: v[c] / w for c in v}
    life, issue = pw["SQ_WAVE_CYCLES"], pw["SQ_ACTIVE_INST_ANY"]
    out[tag] = {
        "launches": len(ks), "waves": w,
        "per_wave": {c.replace("SQ_", ""): round(x, 1) for c, x in pw.items()},
        "per_substep": {"lifetime_quad_cycles": round(life / SUBSTEPS, 1), "issue_floor_quad_cycles": round(issue / SUBSTEPS, 1),
                        "lifetime_cycles": round(4 * life / SUBSTEPS), "issue_floor_cycles": round(4 * issue / SUBSTEPS)},
        "latency_frac": round(issue / life, 4),
        "lifetime_over_floor": round(life / issue, 3),
    }
print(json.dumps(out, indent=1))
