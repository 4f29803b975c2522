#!/bin/bash
# Separate rocprofv3 PMC passes over a short C2 bench (run on the GPU box):
#   FETCH_SIZE, WRITE_SIZE (cannot share a TCC pass) and fp32 VALU instruction
#   counts; summarised into gpurun_out/pmc_traffic_c2.json (copied into
#   profiles/ so a following bench.py run in the same call reports it).
set -e -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
STEPS=${STEPS:-6}
SOLVER=${SOLVER:-cg}
B="bench.py --solver $SOLVER --steps $STEPS --warmup 2 --no-cpu-baseline --groups 1 --no-ppo --no-policy --no-pipeline --no-c2-rollout --no-extra-legs"
mkdir -p gpurun_out
for pass in fetch:FETCH_SIZE write:WRITE_SIZE "valu:SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES"; do
  name=${pass%%:*}; ctrs=${pass#*:}
  rm -rf gpurun_out/pmc_$name
  timeout -k 10 300 rocprofv3 --pmc $ctrs --output-format csv -d gpurun_out/pmc_$name -o run -- python3 $B > gpurun_out/pmc_$name.log 2>&1
done
python3 scripts/pmc_summary.py --config c2 --envs 8192 --fetch gpurun_out/pmc_fetch --write gpurun_out/pmc_write \
  --valu gpurun_out/pmc_valu --solver $SOLVER --out gpurun_out/pmc_traffic_c2.json
[ "$SOLVER" = cg ] && cp gpurun_out/pmc_traffic_c2.json profiles/pmc_traffic_c2.json || cp gpurun_out/pmc_traffic_c2.json profiles/pmc_traffic_c2_$SOLVER.json
