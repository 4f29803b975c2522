#!/bin/bash
# round-6 pass 11: policy A/B (round-5 build, one-step form split out with the cross-layer W_hh overlap,
# split only), the whole GPU suite, the bench line, the CG / Newton PMC traffic passes
set -e -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r06_p11; mkdir -p $O
timeout -k 10 400 python3 -u scripts/policy_ab.py pvariants/libpol_old.so pvariants/libpol_new3.so pvariants/libpol_split.so pvariants/libpol_new3.so pvariants/libpol_split.so pvariants/libpol_old.so > $O/policy_ab.log 2>&1
cat $O/policy_ab.log
rc=0
timeout -k 10 900 python3 -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || rc=$?
tail -3 $O/gpu_tests.log
[ $rc -le 1 ]
timeout -k 10 600 python3 -u bench.py > $O/bench.json 2> $O/bench.err
tail -c 300 $O/bench.json
SOLVER=cg bash scripts/pmc_traffic.sh > $O/pmc_cg.log 2>&1
cp gpurun_out/pmc_traffic_c2.json $O/pmc_traffic_c2_cg.json
SOLVER=newton bash scripts/pmc_traffic.sh > $O/pmc_newton.log 2>&1
cp gpurun_out/pmc_traffic_c2.json $O/pmc_traffic_c2_newton.json
