#!/bin/bash
# round-6 pass 14: the env row index from its LDS copy (fewer spilled VGPRs in the CG kernels): A/B on the
# headline model, bit-identity, and the PMC HBM traffic of the variant
set -e -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r06_p14; mkdir -p $O
timeout -k 10 400 python3 -u tests/diag_variants.py evariants/libeng_base.so evariants/libeng_envx.so --groups 2 --rounds 7 --steps 32 > $O/ab.log 2>&1
tail -3 $O/ab.log
timeout -k 10 400 python3 -u tests/diag_variants.py evariants/libeng_base.so evariants/libeng_envx.so --model ksim-gym-zbot_amd/assets/zbot_like_limbs.xml --groups 2 --rounds 5 --steps 32 > $O/ab_limbs.log 2>&1
tail -3 $O/ab_limbs.log
PMC="WRITE_SIZE SQ_WAVES" bash scripts/pmc_variants.sh evariants/libeng_base.so evariants/libeng_envx.so > $O/pmc_write.log 2>&1
cat $O/pmc_write.log
