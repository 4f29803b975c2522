#!/bin/bash
# Marginal phase costs of the current kernel (dup probes, scripts/dup_probes.py) on the GPU box:
# one-process A/B timing of evariants/libeng_cur.so against every libeng_d_*.so, then one PMC pass
# per library (VALU / SALU / LDS per wave). Usage: bash scripts/r03_probes.sh <tag>
set -e -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 400 python3 -u tests/diag_variants.py evariants/libeng_cur.so evariants/libeng_d_*.so --rounds 5 --steps 16 > $O/dup_probes.log 2>&1
timeout -k 10 400 bash scripts/pmc_variants.sh evariants/libeng_cur.so evariants/libeng_d_*.so > $O/dup_probes_pmc.log 2>&1
