#!/bin/bash
# round-6 pass 3: CG A/B (v4: one-round-trip solve), VALU per wave, the CG outlier envs, the CG contract
# diag on v4, then the whole GPU suite on the product build (v4)
set -e -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r06_p3; mkdir -p $O
timeout -k 10 400 python3 -u tests/diag_variants.py evariants/libeng_base.so evariants/libeng_v3.so evariants/libeng_v4.so --groups 2 --rounds 9 --steps 32 > $O/ab.log 2>&1
bash scripts/pmc_variants.sh evariants/libeng_v4.so > $O/pmc_variants.log 2>&1
timeout -k 10 300 python3 -u tests/diag_cg_env.py --env 63 --env 47 --t 0 > $O/cg_env_pr_t0.log 2>&1
timeout -k 10 300 python3 -u tests/diag_cg_env.py --env 12 --env 23 --env 59 --t 1 --push 0 --randomize 0 > $O/cg_env_flat_t1.log 2>&1
timeout -k 10 300 python3 -u tests/diag_cg_contract.py > $O/cg_contract_pr.log 2>&1
timeout -k 10 300 python3 -u tests/diag_cg_contract.py --push 0 --randomize 0 > $O/cg_contract_flat.log 2>&1
timeout -k 10 300 python3 -u tests/diag_cg_contract.py --eulerdamp > $O/cg_contract_ed_pr.log 2>&1
rc=0
timeout -k 10 1200 python3 -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || rc=$?
tail -3 $O/gpu_tests.log
[ $rc -le 1 ]
