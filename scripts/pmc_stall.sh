#!/bin/bash
# One rocprofv3 --pmc pass of SQ wave-state counters over a short C2 bench
# (run on the GPU box): where the step kernel's wave time goes
# (WAIT_ANY = parked at s_waitcnt / barrier, WAIT_INST_ANY = issue stalls,
# ACTIVE_INST_* = issuing), summarised by scripts/pmc_summary.py --valu.
set -e -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
STEPS=${STEPS:-6}
mkdir -p gpurun_out
rm -rf gpurun_out/pmc_stall
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_SCA \
  --output-format csv -d gpurun_out/pmc_stall -o run -- python3 bench.py --steps $STEPS --warmup 2 --no-cpu-baseline > gpurun_out/pmc_stall.log 2>&1
