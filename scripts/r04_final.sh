#!/bin/bash
# Round-4 full pass on one box: -m gpu suite, smoke, PMC traffic / VALU passes, kernel-trace stats
# of the headline, the default bench line, C3 and C5. Usage: bash scripts/r04_final.sh <tag>
set -e -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
T=$1
O=gpurun_out/$T
mkdir -p $O
bash scripts/r03_check.sh $T
bash scripts/measure.sh
for f in bench.json bench_c3.json bench_c5.json trace_bench.log pmc_traffic_c2.json pmc_traffic_gae.json; do cp gpurun_out/$f $O/; done
cp gpurun_out/trace/run_kernel_stats.csv $O/kernel_stats.csv
