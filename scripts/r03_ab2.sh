#!/bin/bash
# A/B of engine variants + a kernel trace of the default headline: bash scripts/r03_ab2.sh <tag> lib...
set -e -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/$1; shift
mkdir -p $O
timeout -k 10 300 python3 tests/diag_variants.py "$@" --rounds 7 --steps 24 > $O/ab.log 2>&1
rm -rf $O/trace
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 bench.py --no-cpu-baseline --no-ppo --no-policy --no-pipeline --no-c2-rollout > $O/trace_bench.json 2> $O/trace_bench.err
