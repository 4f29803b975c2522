#!/bin/bash
# round-6 pass 1: CG A/B (merged reductions), CG / Newton phase stamps, CG parity subset
set -e -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r06_p1; mkdir -p $O
timeout -k 10 300 python3 -u tests/diag_variants.py evariants/libeng_base.so evariants/libeng_v1.so --groups 2 --rounds 7 --steps 32 > $O/ab_v1.log 2>&1
timeout -k 10 120 python3 -u tests/diag_stamps.py --solver cg --out $O/stamps_cg.json > $O/stamps_cg.log 2>&1
timeout -k 10 120 python3 -u tests/diag_stamps.py --solver newton --out $O/stamps_newton.json > $O/stamps_newton.log 2>&1
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -x -v -s --timeout 200 --timeout-method thread -k "cg or golden" > $O/parity_cg.log 2>&1
timeout -k 10 300 python3 -u tests/diag_cg_contract.py > $O/cg_contract_pr.log 2>&1
timeout -k 10 300 python3 -u tests/diag_cg_contract.py --push 0 --randomize 0 > $O/cg_contract_flat.log 2>&1
timeout -k 10 300 python3 -u tests/diag_cg_contract.py --eulerdamp > $O/cg_contract_ed_pr.log 2>&1
timeout -k 10 300 python3 -u tests/diag_cg_contract.py --eulerdamp --solver newton > $O/newton_contract_ed_pr.log 2>&1
