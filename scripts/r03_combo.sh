#!/bin/bash
# check (tests, smoke, bench) then A/B + PMC in one call: bash scripts/r03_combo.sh <tag> lib...
set -e -o pipefail
cd "$(dirname "$0")/.."
T=$1; shift
bash scripts/r03_check.sh $T
bash scripts/r03_ab.sh $T "$@"
timeout -k 10 120 python3 scripts/pairing_probe.py > gpurun_out/$T/pairing.json 2>&1
