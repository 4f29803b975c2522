#!/bin/bash
# Round 3 A/B: engine variants (evariants/libeng_*.so, scripts/ab_build.sh) timed round-robin in one
# process, then the PMC traffic passes of the product library. Usage: bash scripts/r03_ab.sh <tag> lib...
set -e -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/$1; shift
mkdir -p $O
timeout -k 10 300 python3 tests/diag_variants.py "$@" --rounds 5 --steps 24 > $O/ab.log 2>&1
if [ -z "$NO_PMC" ]; then
  timeout -k 10 600 bash scripts/pmc_traffic.sh > $O/pmc.log 2>&1
  cp gpurun_out/pmc_traffic_c2.json $O/
fi
