#!/bin/bash
# One rocprofv3 --pmc pass over the policy kernels (run on the GPU box): matrix-core busy cycles
# against the GPU's active cycles per dispatch, summarised by scripts/pmc_policy_summary.py.
set -e -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf gpurun_out/pmc_policy
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE \
  --output-format csv -d gpurun_out/pmc_policy -o run -- python3 scripts/policy_driver.py 8192 10 > gpurun_out/pmc_policy.log 2>&1
python3 scripts/pmc_policy_summary.py gpurun_out/pmc_policy > gpurun_out/pmc_policy_summary.json
cat gpurun_out/pmc_policy_summary.json
