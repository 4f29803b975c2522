#!/bin/bash
# Round 4: A/B of engine variants (grouped and one stream) in one process, then PMC VALU counts.
# Usage: bash scripts/r04_ab3w.sh <tag> lib...
set -e -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/$1; shift
mkdir -p $O
timeout -k 10 300 python3 -u tests/diag_variants.py "$@" --groups 2 --rounds 7 --steps 24 > $O/ab_g2.log 2>&1
timeout -k 10 300 python3 -u tests/diag_variants.py "$@" --rounds 5 --steps 24 > $O/ab_g1.log 2>&1
timeout -k 10 400 bash scripts/pmc_variants.sh "$@" > $O/pmc_variants.log 2>&1
