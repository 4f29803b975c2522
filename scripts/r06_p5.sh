#!/bin/bash
# round-6 pass 5: the CG contract tests again (slack 3 x sensitivity), the touchdown cause test, the
# latency profile (PMC at 512 and 8192 envs, both solvers), CG / Newton stamps at 512 and 8192 envs
set -e -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r06_p5; mkdir -p $O
rc=0
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_sole_pair.py tests/test_gpu_colliders.py -v -s --timeout 300 --timeout-method thread -k "one_step or touchdown" > $O/contract_tests.log 2>&1 || rc=$?
tail -3 $O/contract_tests.log
[ $rc -le 1 ]
bash scripts/pmc_latency.sh > $O/pmc_latency.log 2>&1
cp gpurun_out/pmc_latency.json $O/
for s in cg newton; do for n in 512 8192; do
  timeout -k 10 120 python3 -u tests/diag_stamps.py --solver $s --n $n --out $O/stamps_${s}_$n.json > $O/stamps_${s}_$n.log 2>&1
done; done
