#!/bin/bash
# Round 4: the new / changed GPU tests (ksim API over groups, INTEGRATION binding, parity contract
# with the bounded slack and the tolerance-0 cause test, the 64 x 128 C1 fixture), the step-gap
# probe, a kernel trace of the headline command, and the default bench line with the new legs.
# Usage: bash scripts/r04_check2.sh <tag>
set -e -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_task_groups.py tests/test_gpu_integration.py tests/test_gpu_parity.py -x -v -s --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
timeout -k 10 300 python3 -u scripts/gap_probe.py --steps 200 --reps 5 > $O/gap_probe.json 2> $O/gap_probe.err
rm -rf gpurun_out/trace_$1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/trace_$1 -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-ppo --no-policy --no-pipeline --no-c2-rollout --no-extra-legs > $O/trace_bench.json 2> $O/trace_bench.err
timeout -k 10 400 python3 bench.py > $O/bench.json 2> $O/bench.err
