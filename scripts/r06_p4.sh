#!/bin/bash
# round-6 pass 4: the whole GPU suite on the CG-contract tests, smoke, then the default bench line
set -e -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r06_p4; mkdir -p $O
rc=0
timeout -k 10 1200 python3 -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || rc=$?
tail -3 $O/gpu_tests.log
[ $rc -le 1 ]
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 600 python3 bench.py > $O/bench.json 2> $O/bench.err
