#!/bin/bash
# round-6 pass 10: the block-layout policy kernel with layer l+1's W_hh products beside layer l's epilogue
# (policy tests + A/B against the previous build), the CG contract at slack 2.5x
set -e -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r06_p10; mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_policy.py tests/test_gpu_policy_layouts.py -v --timeout 120 --timeout-method thread > $O/policy_tests.log 2>&1
tail -3 $O/policy_tests.log
timeout -k 10 300 python3 -u scripts/policy_ab.py pvariants/libpol_old.so pvariants/libpol_new.so pvariants/libpol_new2.so pvariants/libpol_old.so pvariants/libpol_new2.so > $O/policy_ab.log 2>&1
cat $O/policy_ab.log
rc=0
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_sole_pair.py tests/test_gpu_colliders.py -v -s --timeout 300 --timeout-method thread -k "one_step" > $O/contract_tests.log 2>&1 || rc=$?
tail -3 $O/contract_tests.log
[ $rc -le 1 ]
