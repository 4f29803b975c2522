#!/bin/bash
# The driver's own bench invocations on one box (N=1 with its short window, twice), for the
# headline's robustness to the window length. Usage: bash scripts/r03_driver_cmd.sh <tag>
set -e -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_s20w5_a.json 2> $O/bench_s20w5_a.err
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_s20w5_b.json 2> $O/bench_s20w5_b.err
timeout -k 10 300 python3 bench.py --gpus 1 --steps 200 --warmup 10 --no-cpu-baseline --no-ppo --no-policy --no-pipeline --no-c2-rollout > $O/bench_s200.json 2> $O/bench_s200.err
