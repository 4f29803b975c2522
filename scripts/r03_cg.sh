#!/bin/bash
# Round 3: the -m gpu suite (with the CG solver tests), then bench lines for both solvers.
set -e -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-ppo --no-policy --no-pipeline --solver newton > $O/bench_newton.json 2> $O/bench_newton.err
timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-ppo --no-policy --no-pipeline --solver cg > $O/bench_cg.json 2> $O/bench_cg.err
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > $O/bench_driver_cmd.json 2> $O/bench_driver_cmd.err
