#!/bin/bash
# Round 3: the general-collider kernels on the GPU box. The collider parity tests first (their
# failures do not stop the run; a fault, abort or time limit does), then the rest of the -m gpu
# suite, smoke and the default bench line. Usage: bash scripts/r03_xg.sh <tag>
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_colliders.py -m gpu -v -s --timeout 120 --timeout-method thread > $O/gpu_colliders.log 2>&1
rc=$?
echo "colliders rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
set -e
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread --deselect tests/test_gpu_colliders.py > $O/gpu_tests.log 2>&1
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 300 python3 bench.py > $O/bench.json 2> $O/bench.err
L="--no-cpu-baseline --no-ppo --no-policy --no-pipeline --no-c2-rollout"
timeout -k 10 300 python3 bench.py --model ksim-gym-zbot_amd/assets/zbot_like_limbs.xml $L > $O/bench_limbs.json 2> $O/bench_limbs.err
