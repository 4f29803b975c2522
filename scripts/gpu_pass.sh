#!/bin/bash
# One GPU-box pass, parametrized (replaces rounds 3-4's per-lease r0N_*.sh drivers):
#   bash scripts/gpu_pass.sh <tag> [check] [pmc] [trace] [bench] [c3c5]
# check: the -m gpu suite (prints the measured parity errors) and smoke
# pmc:   PMC traffic / VALU passes of the step kernel and the GAE kernel (refreshes profiles/pmc_*)
# trace: rocprofv3 kernel trace + stats of the headline's command
# bench: the default bench line (the driver's N = 1 command)
# c3c5:  bench lines at C3 and C5
# Every step has its own time limit; the first failure ends the pass. Outputs: gpurun_out/<tag>/.
set -e -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
T=$1; shift
O=gpurun_out/$T
mkdir -p $O
for step in "$@"; do
  case $step in
    check)
      # a failed assertion (rc 1) does not end the pass; a crash, abort or time limit does
      rc=0
      timeout -k 10 900 python3 -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || rc=$?
      tail -3 $O/gpu_tests.log
      [ $rc -le 1 ] || exit $rc
      timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 ;;
    pmc)
      bash scripts/pmc_traffic.sh > $O/pmc.log 2>&1
      bash scripts/pmc_gae.sh > $O/pmc_gae.log 2>&1
      cp gpurun_out/pmc_traffic_gae.json profiles/pmc_traffic_gae.json
      cp gpurun_out/pmc_traffic_c2.json gpurun_out/pmc_traffic_gae.json $O/ ;;
    trace)
      rm -rf gpurun_out/trace
      timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/trace -o run -- python3 bench.py \
        --steps 32 --warmup 4 --no-cpu-baseline --no-ppo --no-policy --no-pipeline --no-c2-rollout --no-extra-legs > $O/trace_bench.log 2>&1
      cp gpurun_out/trace/run_kernel_stats.csv $O/kernel_stats.csv ;;
    bench)
      timeout -k 10 600 python3 bench.py > $O/bench.json 2> $O/bench.err
      cat $O/bench.json ;;
    c3c5)
      timeout -k 10 300 python3 bench.py --config c3 --no-cpu-baseline --no-extra-legs > $O/bench_c3.json 2> $O/bench_c3.err
      timeout -k 10 300 python3 bench.py --config c5 --no-cpu-baseline --no-extra-legs > $O/bench_c5.json 2> $O/bench_c5.err ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
