#!/bin/bash
# Per-variant instruction counts of the step kernel (run on the GPU box; diagnostic only):
#   scripts/pmc_variants.sh evariants/libeng_a.so evariants/libeng_b.so ...
# One rocprofv3 --pmc pass per library over scripts/variant_driver.py; prints per-launch
# SQ_INSTS_VALU / SALU / LDS per wave (median over the step launches). PMC="<counters>" overrides
# the list (at most 8 SQ counters, one of them SQ_WAVES: values are printed per wave).
set -e -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
for lib in "$@"; do
  name=$(basename "$lib" .so)
  rm -rf "gpurun_out/pmcv_$name"
  timeout -k 10 120 rocprofv3 --pmc ${PMC:-SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32} \
    --output-format csv -d "gpurun_out/pmcv_$name" -o run -- python3 scripts/variant_driver.py "$lib" > "gpurun_out/pmcv_$name.log" 2>&1
  python3 - "$name" <<'PY'
import csv, glob, statistics, sys
name = sys.argv[1]
per = {}
for fn in glob.glob(f"gpurun_out/pmcv_{name}/**/*counter_collection.csv", recursive=True):
    for row in csv.DictReader(open(fn)):
        if "step_kernel" not in row["Kernel_Name"]:
            continue
        per.setdefault(row["Dispatch_Id"], {}).setdefault(row["Counter_Name"], 0.0)
        per[row["Dispatch_Id"]][row["Counter_Name"]] += float(row["Counter_Value"])
ks = sorted(per, key=int)
vals = {c: statistics.median(per[k][c] for k in ks) for c in per[ks[0]]}
w = vals["SQ_WAVES"]
it = open(f"gpurun_out/pmcv_{name}.log").read().strip().splitlines()[-1]
print(f"{name:24s} launches {len(ks)}  per wave: " + "  ".join(f"{c.replace('SQ_INSTS_', '')} {vals[c] / w:9.0f}" for c in sorted(vals) if c != "SQ_WAVES") + f"   [{it}]")
PY
done
