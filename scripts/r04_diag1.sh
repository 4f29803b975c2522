#!/bin/bash
# Round 4, first lease: the INTEGRATION binding test, the one-step parity suite with its printed
# errors, the randomized-Newton outlier diagnosis at the default and zero solver tolerance, and the
# default bench line. Usage: bash scripts/r04_diag1.sh <tag>
set -e -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_integration.py tests/test_gpu_parity.py -x -v -s --timeout 200 --timeout-method thread -k "integration or one_step" > $O/gpu_tests.log 2>&1
timeout -k 10 200 python3 -u scripts/diag_onestep.py --randomize > $O/diag_rand.log 2>&1
timeout -k 10 200 python3 -u scripts/diag_onestep.py --randomize --tol 0 > $O/diag_rand_tol0.log 2>&1
timeout -k 10 300 python3 bench.py > $O/bench.json 2> $O/bench.err
