#!/bin/bash
# full -m gpu suite + smoke + bench + headline probes at 2/3/4 groups: bash scripts/r03_check2.sh <tag>
set -e -o pipefail
cd "$(dirname "$0")/.."
T=$1
bash scripts/r03_check.sh $T
O=gpurun_out/$T
for G in 2 3 4; do
  timeout -k 10 200 python3 scripts/headline_probe.py --steps 20 --warmup 5 --groups $G --reps 4 > $O/probe20_g$G.json 2> $O/probe20_g$G.err
done
