#!/bin/bash
# round-6 pass 9: the CG contract at budget 1, slack 2x; the touchdown cause tests; the debug forwards
set -e -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r06_p9; mkdir -p $O
rc=0
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_sole_pair.py tests/test_gpu_colliders.py -v -s --timeout 300 --timeout-method thread -k "one_step or touchdown or debug_forward" > $O/contract_tests.log 2>&1 || rc=$?
tail -5 $O/contract_tests.log
[ $rc -le 1 ]
