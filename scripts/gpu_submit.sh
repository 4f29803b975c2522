#!/bin/bash
# Submit one command to the GPU box through gpurun, retrying ONLY while the pool has no free slot
# (gpurun's "transient" status: nothing ran, nothing was charged), at most 12 times, 4 min apart.
# A command that ran (whatever its exit status) is never resubmitted.
#   scripts/gpu_submit.sh <timeout-seconds> <log> '<command>'
T=$1; LOG=$2; shift 2
for try in $(seq 1 12); do
  /usr/local/graft/bin/gpurun --timeout "$T" -- "$@" > "$LOG" 2>&1
  rc=$?
  if grep -q "status=transient" "$LOG" || [ $rc -eq 3 ]; then
    echo "[gpu_submit] no free slot (try $try), waiting" >> "$LOG.tries"
    sleep 240
    continue
  fi
  echo "[gpu_submit] done rc=$rc" >> "$LOG"
  exit $rc
done
echo "[gpu_submit] gave up" >> "$LOG"
exit 3
