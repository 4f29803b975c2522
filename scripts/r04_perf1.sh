#!/bin/bash
# Round 4: C1 env-35 divergence diagnosis, the step-gap probe, a kernel trace of the headline
# command and the default bench line with the new legs. Usage: bash scripts/r04_perf1.sh <tag>
set -e -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 200 python3 -u scripts/diag_c1_env.py > $O/diag_c1_env35.log 2>&1
timeout -k 10 200 python3 -u scripts/diag_c1_env.py --tol 0 > $O/diag_c1_env35_tol0.log 2>&1
timeout -k 10 300 python3 -u scripts/gap_probe.py --steps 200 --reps 5 > $O/gap_probe.json 2> $O/gap_probe.err
rm -rf gpurun_out/trace_$1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/trace_$1 -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-ppo --no-policy --no-pipeline --no-c2-rollout --no-extra-legs > $O/trace_bench.json 2> $O/trace_bench.err
timeout -k 10 400 python3 bench.py > $O/bench.json 2> $O/bench.err
