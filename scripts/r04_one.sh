#!/bin/bash
# One GPU test selection with printed output. Usage: bash scripts/r04_one.sh <tag> <pytest -k expr> [files]
set -e -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
K=$2; shift 2
timeout -k 10 400 python3 -u -m pytest ${@:-tests/test_gpu_parity.py} -v -s --timeout 300 --timeout-method thread -k "$K" > $O/gpu_tests.log 2>&1
