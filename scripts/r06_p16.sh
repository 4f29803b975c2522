#!/bin/bash
# round-6 pass 16: the headline's env-group count (2 = bench.py's default) against 3 and 4, alternating
set -e -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r06_p16; mkdir -p $O
for rep in 1 2 3; do for g in 2 3 4; do
  timeout -k 10 200 python3 -u bench.py --groups $g --steps 64 --warmup 8 --no-cpu-baseline --no-ppo --no-policy --no-pipeline --no-c2-rollout --no-extra-legs > $O/g${g}_$rep.json 2> $O/g${g}_$rep.err
  python3 -c "import json; d=json.loads(open('$O/g${g}_$rep.json').read().strip().splitlines()[-1]); print($g, $rep, d['value'], d['ms_per_step'], d['roofline']['kernel_avg_ms'])" | tee -a $O/summary.txt
done; done
