#!/bin/bash
# Round 4: the solo step layout on one box: its GPU tests, then the train.py-size legs (512 envs)
# and a layout sweep over small env counts. Usage: bash scripts/r04_solo.sh <tag>
set -e -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_layout.py tests/test_gpu_parity.py -v -s --timeout 200 --timeout-method thread -k "layout or solo or cg_conditioned or golden" > $O/gpu_tests_layout.log 2>&1
timeout -k 10 300 python3 -u scripts/layout_sweep.py > $O/layout_sweep.json 2> $O/layout_sweep.err
