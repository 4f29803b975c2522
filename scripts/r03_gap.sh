#!/bin/bash
# Round 3: the driver's headline command, the per-launch timeline probe and a runtime trace.
set -e -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out/r03
O=gpurun_out/r03
timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $O/drv1.json 2> $O/drv1.err
timeout -k 10 200 python3 scripts/headline_probe.py --steps 20 --warmup 5 --groups 2 --reps 4 > $O/probe_g2.json 2> $O/probe_g2.err
timeout -k 10 200 python3 scripts/headline_probe.py --steps 20 --warmup 5 --groups 1 --reps 2 > $O/probe_g1.json 2> $O/probe_g1.err
timeout -k 10 300 rocprofv3 --kernel-trace --hip-runtime-trace --stats --output-format csv -d $O/trace -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-ppo --no-policy --no-pipeline --no-c2-rollout > $O/trace_bench.json 2> $O/trace_bench.err
timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/drv2.json 2> $O/drv2.err
