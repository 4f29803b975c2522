#!/bin/bash
# Round 4: VALU per wave of engine variants (PMC), slot occupancy / hand-over of the grouped
# headline and the placement of train.py's 512 envs (wavetime build). Usage: bash scripts/r04_probe1.sh <tag> lib...
set -e -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/$1; shift
mkdir -p $O
timeout -k 10 500 bash scripts/pmc_variants.sh "$@" > $O/pmc_variants.log 2>&1
timeout -k 10 200 python3 -u scripts/groups_wavetime.py --groups 2 --out $O/wavetime_g2.json > $O/wavetime_g2.log 2>&1
timeout -k 10 200 python3 -u scripts/groups_wavetime.py --groups 1 --out $O/wavetime_g1.json > $O/wavetime_g1.log 2>&1
timeout -k 10 200 python3 -u scripts/groups_wavetime.py --groups 1 --n 512 --out $O/wavetime_512.json > $O/wavetime_512.log 2>&1
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -v -s --timeout 200 --timeout-method thread -k "cg" > $O/gpu_tests_cg.log 2>&1
