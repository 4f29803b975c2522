#!/bin/bash
# Round 4: instruction counts and wave-state counters of the two-sole and the general-collider
# (limbs model) step kernels, one rocprofv3 --pmc pass per counter set and model (diagnostic).
#   bash scripts/r04_pmc_xg.sh <tag>
set -e -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
LIB=ksim-gym-zbot_amd/zbot_amd/libzbot_hip.so
STALL="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_WAVES"
for m in default limbs; do
  if [ $m = limbs ]; then export MODEL=ksim-gym-zbot_amd/assets/zbot_like_limbs.xml; else unset MODEL; fi
  cp $LIB gpurun_out/lib_$m.so
  bash scripts/pmc_variants.sh gpurun_out/lib_$m.so >> $O/pmc_xg_insts.log 2>&1
  PMC="$STALL" bash scripts/pmc_variants.sh gpurun_out/lib_$m.so >> $O/pmc_xg_stall.log 2>&1
done
