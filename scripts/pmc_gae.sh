#!/bin/bash
# HBM traffic of zb::gae_kernel (PPO inputs leg) at the C2 rollout shape [256, 8192]:
# separate rocprofv3 --pmc passes for FETCH_SIZE and WRITE_SIZE, plus a kernel trace.
set -e -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
for pass in fetch:FETCH_SIZE write:WRITE_SIZE; do
  name=${pass%%:*}; ctrs=${pass#*:}
  rm -rf gpurun_out/pmcg_$name
  timeout -s KILL 120 rocprofv3 --pmc $ctrs --output-format csv -d gpurun_out/pmcg_$name -o run -- python3 scripts/gae_driver.py 256 8192 12 > gpurun_out/pmcg_$name.log 2>&1
done
rm -rf gpurun_out/trace_gae
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/trace_gae -o run -- python3 scripts/gae_driver.py 256 8192 12 > gpurun_out/trace_gae.log 2>&1
python3 scripts/pmc_summary.py --config gae --kernel gae_kernel --envs 8192 --T 256 --fetch gpurun_out/pmcg_fetch \
  --write gpurun_out/pmcg_write --out gpurun_out/pmc_traffic_gae.json
