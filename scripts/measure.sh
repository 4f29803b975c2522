#!/bin/bash
# One measurement round on the GPU box: PMC traffic passes, kernel-trace stats,
# and the default bench line (which picks up the fresh PMC traffic figure).
set -e -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
bash scripts/pmc_traffic.sh > gpurun_out/pmc.log 2>&1
bash scripts/pmc_gae.sh > gpurun_out/pmc_gae.log 2>&1
cp gpurun_out/pmc_traffic_gae.json profiles/pmc_traffic_gae.json
rm -rf gpurun_out/trace
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/trace -o run -- python3 bench.py --steps 32 --warmup 4 --no-cpu-baseline --no-ppo --no-policy --no-pipeline --no-c2-rollout --no-extra-legs > gpurun_out/trace_bench.log 2>&1
timeout -k 10 400 python3 bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
cat gpurun_out/bench.json
timeout -k 10 300 python3 bench.py --config c3 --no-cpu-baseline > gpurun_out/bench_c3.json 2> gpurun_out/bench_c3.err
timeout -k 10 300 python3 bench.py --config c5 --no-cpu-baseline > gpurun_out/bench_c5.json 2> gpurun_out/bench_c5.err
