"""Where do the grouped headline's step launches stop overlapping?

Reads a rocprofv3 --kernel-trace CSV of `bench.py --steps K --warmup W --groups G` (no other legs)
and takes the last K x G step_kernel launches (the timed window). Prints one JSON object:
  * per stream: the launches' average duration and the gaps between consecutive launches;
  * the window: its span (first start to last end), the time with no step kernel running at all,
    the time with only one running, and the span per step against the average launch duration.

    python scripts/trace_gaps.py gpurun_out/trace_x/run_kernel_trace.csv --steps 20 --groups 2
"""

from __future__ import annotations

import argparse
import csv
import json
import statistics


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--groups", type=int, default=2)
    ap.add_argument("--kernel", default="step_kernel")
    args = ap.parse_args()
    rows = []
    with open(args.csv) as f:
        for r in csv.DictReader(f):
            if args.kernel in r["Kernel_Name"]:
                sid = r.get("Stream_Id") or r.get("Queue_Id") or "0"
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), sid))
    rows.sort()
    win = rows[-args.steps * args.groups:]
    streams: dict = {}
    for s, e, sid in win:
        streams.setdefault(sid, []).append((s, e))
    per = {}
    for sid, ls in streams.items():
        gaps = [b[0] - a[1] for a, b in zip(ls[:-1], ls[1:])]
        per[sid] = {"launches": len(ls), "avg_ms": statistics.mean(e - s for s, e in ls) / 1e6,
                    "gap_us_mean": statistics.mean(gaps) / 1e3 if gaps else None,
                    "gap_us_max": max(gaps) / 1e3 if gaps else None}
    # sweep: how many step kernels run at each instant of the window
    ev = sorted([(s, 1) for s, _, _ in win] + [(e, -1) for _, e, _ in win])
    t0, t1 = ev[0][0], ev[-1][0]
    idle = single = 0
    cur, last = 0, t0
    for t, d in ev:
        if cur == 0:
            idle += t - last
        elif cur == 1:
            single += t - last
        cur += d
        last = t
    span = t1 - t0
    avg = statistics.mean(e - s for s, e, _ in win) / 1e6
    print(json.dumps({
        "launches": len(win), "streams": per, "span_ms": span / 1e6,
        "ms_per_step_span": span / 1e6 / args.steps, "avg_launch_ms": avg,
        "idle_ms": idle / 1e6, "one_running_ms": single / 1e6,
        "span_over_launch": span / 1e6 / args.steps / avg,
    }, indent=1))


if __name__ == "__main__":
    main()
