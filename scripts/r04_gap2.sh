#!/bin/bash
# Round 4: group layouts against the step gap (G x chunks), and a kernel trace at 3 groups.
set -e -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 400 python3 -u scripts/gap_probe.py --steps 100 --reps 3 --variants noev --configs 1x0,1x1,2x1,2x2,3x1,4x1 > $O/gap_probe2.json 2> $O/gap_probe2.err
rm -rf gpurun_out/trace3_$1
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/trace3_$1 -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --groups 3 --no-cpu-baseline --no-ppo --no-policy --no-pipeline --no-c2-rollout --no-extra-legs > $O/trace3_bench.json 2> $O/trace3_bench.err
