#!/bin/bash
# round-6 pass 2: CG A/B (v1 merged sums, v2 root coupling, v3 no Hessian stores), VALU per wave,
# the CG contract with input-perturbation sensitivity, the bank-2 cap probe, CG parity on v3
set -e -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r06_p2; mkdir -p $O
timeout -k 10 400 python3 -u tests/diag_variants.py evariants/libeng_base.so evariants/libeng_v1.so evariants/libeng_v2.so evariants/libeng_v3.so --groups 2 --rounds 9 --steps 32 > $O/ab.log 2>&1
bash scripts/pmc_variants.sh evariants/libeng_base.so evariants/libeng_v3.so > $O/pmc_variants.log 2>&1
timeout -k 10 300 python3 -u tests/diag_cg_contract.py > $O/cg_contract_pr.log 2>&1
timeout -k 10 300 python3 -u tests/diag_cg_contract.py --push 0 --randomize 0 > $O/cg_contract_flat.log 2>&1
timeout -k 10 300 python3 -u tests/diag_cg_contract.py --eulerdamp > $O/cg_contract_ed_pr.log 2>&1
timeout -k 10 300 python3 -u tests/diag_bank2_overflow.py > $O/bank2_c3.log 2>&1
timeout -k 10 300 python3 -u tests/diag_bank2_overflow.py --sigma 0.2 > $O/bank2_c3_s02.log 2>&1
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -x -v -s --timeout 200 --timeout-method thread -k "cg or golden" > $O/parity_cg.log 2>&1
