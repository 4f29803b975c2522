#!/bin/bash
# round-6 pass 15: the actor in the rollout loop by layout and group count (after the one-step block split)
set -e -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r06_p15; mkdir -p $O
timeout -k 10 400 python3 -u scripts/policy_loop_probe.py --layouts block,wave2,wave4 --groups 1,2,3 > $O/loop_probe.log 2>&1
cat $O/loop_probe.log
