#!/bin/bash
# A/B of engine variants in one process (first library = reference for the screening parity),
# then the marginal phase costs (dup probes) of the current kernel: bash scripts/r03_ab3.sh <tag> lib...
set -e -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/$1; shift
mkdir -p $O
timeout -k 10 300 python3 -u tests/diag_variants.py "$@" --rounds ${ROUNDS:-7} --steps 24 ${AB_ARGS:-} > $O/ab${AB_TAG:-}.log 2>&1
if [ -n "$PROBES" ]; then
  timeout -k 10 400 python3 -u tests/diag_variants.py evariants/libeng_cur.so evariants/libeng_d_*.so --rounds 5 --steps 16 > $O/dup_probes.log 2>&1
  timeout -k 10 500 bash scripts/pmc_variants.sh evariants/libeng_cur.so evariants/libeng_d_*.so > $O/dup_probes_pmc.log 2>&1
fi
