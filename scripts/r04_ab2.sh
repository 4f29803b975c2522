#!/bin/bash
# Round 4: grouped and one-stream A/B of engine variants, then the two-rank rehearsal test.
# Usage: bash scripts/r04_ab2.sh <tag> lib...
set -e -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/$1; shift
mkdir -p $O
timeout -k 10 300 python3 -u tests/diag_variants.py "$@" --groups 2 --rounds ${ROUNDS:-9} --steps 24 > $O/ab_g2.log 2>&1
timeout -k 10 300 python3 -u tests/diag_variants.py "$@" --rounds 5 --steps 24 > $O/ab_g1.log 2>&1
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_distributed.py -v -s --timeout 350 --timeout-method thread > $O/dist.log 2>&1
