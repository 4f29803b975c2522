#!/bin/bash
# round-6 pass 7: the whole GPU suite (the CG contract with the qpos+qvel sensitivity, the sole pair's
# manifold-tie ensemble, XG 4), then the default bench line
set -e -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r06_p7; mkdir -p $O
rc=0
timeout -k 10 900 python3 -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || rc=$?
tail -5 $O/gpu_tests.log
[ $rc -le 1 ]
timeout -k 10 600 python3 -u bench.py > $O/bench.json 2> $O/bench.err
tail -c 600 $O/bench.json
