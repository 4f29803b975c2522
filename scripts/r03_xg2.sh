#!/bin/bash
# Round 3: the general-collider tests and the limbs-model bench only. Usage: bash scripts/r03_xg2.sh <tag>
set -e -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_colliders.py -m gpu -v -s --timeout 120 --timeout-method thread > $O/gpu_colliders.log 2>&1
L="--no-cpu-baseline --no-ppo --no-policy --no-pipeline --no-c2-rollout"
timeout -k 10 300 python3 bench.py --model ksim-gym-zbot_amd/assets/zbot_like_limbs.xml $L > $O/bench_limbs.json 2> $O/bench_limbs.err
timeout -k 10 300 python3 bench.py --model ksim-gym-zbot_amd/assets/zbot_like_limbs.xml $L --groups 1 > $O/bench_limbs_g1.json 2> $O/bench_limbs_g1.err
