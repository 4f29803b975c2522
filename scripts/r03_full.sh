#!/bin/bash
# Round 3 full pass: -m gpu suite, smoke, default bench, chunked partial-round bench, C3 / C5 lines.
set -e -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
T=$1
bash scripts/r03_check.sh $T
O=gpurun_out/$T
L="--no-cpu-baseline --no-ppo --no-policy --no-pipeline --no-c2-rollout"
timeout -k 10 300 python3 bench.py --envs 5120 --groups 1 $L > $O/bench_5120_chunked.json 2> $O/bench_5120.err
ZB_STEP_CHUNKS=1 timeout -k 10 300 python3 bench.py --envs 5120 --groups 1 $L > $O/bench_5120_unchunked.json 2> $O/bench_5120u.err
timeout -k 10 300 python3 bench.py --config c3 --no-cpu-baseline > $O/bench_c3.json 2> $O/bench_c3.err
timeout -k 10 300 python3 bench.py --config c5 --no-cpu-baseline > $O/bench_c5.json 2> $O/bench_c5.err
