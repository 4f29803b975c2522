#!/bin/bash
# Latency profile of the step kernel (run on the GPU box): one rocprofv3 --pmc pass of the SQ wave-cycle
# counters per (solver, env count) over scripts/variant_driver.py on the product library, summarised by
# scripts/pmc_latency_summary.py into gpurun_out/pmc_latency.json (copied to profiles/ by the caller).
# 512 envs = train.py's size: 256 waves on 256 CUs, every wave alone on its SIMD, so its lifetime is its
# own instruction stream: issuing (SQ_ACTIVE_INST_ANY) or stalled on its dependencies (the rest).
set -e -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
LIB=ksim-gym-zbot_amd/zbot_amd/libzbot_hip.so
for solver in cg newton; do
  for n in 512 8192; do
    d=gpurun_out/pmclat_${solver}_$n
    rm -rf $d
    SOLVER=$solver N=$n timeout -k 10 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY \
      SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_WAVES --output-format csv -d $d -o run -- \
      python3 scripts/variant_driver.py $LIB 6 > $d.log 2>&1
  done
done
python3 scripts/pmc_latency_summary.py gpurun_out/pmclat > gpurun_out/pmc_latency.json
cat gpurun_out/pmc_latency.json
