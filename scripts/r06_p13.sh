#!/bin/bash
# round-6 pass 13: the second bank's empty-bank exit ahead of its row-chain shuffles (A/B on the limbs
# model), then the closing pass (GPU suite + smoke, PMC, kernel trace, bench, C3 / C5)
set -e -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r06_p13; mkdir -p $O
timeout -k 10 400 python3 -u tests/diag_variants.py evariants/libeng_base.so evariants/libeng_early.so --model ksim-gym-zbot_amd/assets/zbot_like_limbs.xml --groups 2 --rounds 7 --steps 32 > $O/ab_limbs.log 2>&1
tail -3 $O/ab_limbs.log
bash scripts/gpu_pass.sh r06_v2 check pmc trace bench c3c5
