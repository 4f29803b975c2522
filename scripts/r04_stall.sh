#!/bin/bash
# Round 4: wave-state and LDS counters of the step kernel at C2 (one handle, headline only), one
# rocprofv3 --pmc pass each. Usage: bash scripts/r04_stall.sh <tag>
set -e -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
B="bench.py --steps 6 --warmup 2 --no-cpu-baseline --groups 1 --no-ppo --no-policy --no-pipeline --no-c2-rollout --no-extra-legs"
rm -rf gpurun_out/pmc_stall gpurun_out/pmc_lds
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_WAVES \
  --output-format csv -d gpurun_out/pmc_stall -o run -- python3 $B > $O/pmc_stall.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAVES SQ_INSTS_SMEM SQ_INSTS_VMEM SQ_ACTIVE_INST_SCA SQ_INSTS_SALU \
  --output-format csv -d gpurun_out/pmc_lds -o run -- python3 $B > $O/pmc_lds.log 2>&1
python3 - $O <<'PY'
import csv, glob, json, statistics, sys
out = {}
for d in ("pmc_stall", "pmc_lds"):
    per = {}
    for fn in glob.glob(f"gpurun_out/{d}/**/*counter_collection.csv", recursive=True):
        for row in csv.DictReader(open(fn)):
            if "step_kernel" not in row["Kernel_Name"]:
                continue
            per.setdefault(row["Dispatch_Id"], {}).setdefault(row["Counter_Name"], 0.0)
            per[row["Dispatch_Id"]][row["Counter_Name"]] += float(row["Counter_Value"])
    ks = sorted(per, key=int)
    vals = {c: statistics.median(per[k][c] for k in ks) for c in per[ks[0]]}
    w = vals["SQ_WAVES"]
    out[d] = {c: vals[c] / w for c in vals if c != "SQ_WAVES"}
    out[d]["launches"] = len(ks)
    out[d]["waves"] = w
json.dump(out, open(sys.argv[1] + "/pmc_stall_lds.json", "w"), indent=1)
print(json.dumps(out, indent=1))
PY
