#!/bin/bash
# Round 4 on one box: an A/B of engine variants in one process (grouped, as the headline runs),
# then the -m gpu suite, smoke and the default bench line of the product library.
# Usage: bash scripts/r04_check_ab.sh <tag> lib...   (no libs: skip the A/B)
set -e -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/$1; shift
mkdir -p $O
if [ $# -gt 0 ]; then
  timeout -k 10 300 python3 -u tests/diag_variants.py "$@" --groups 2 --rounds ${ROUNDS:-7} --steps 24 > $O/ab.log 2>&1
fi
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
  timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
fi
timeout -k 10 300 python3 bench.py > $O/bench.json 2> $O/bench.err
