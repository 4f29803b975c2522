"""Per-pair start / end times of the step kernel from the -DZB_WAVETIME diagnostic build, and
what a cost-ordered dispatch could save on the last round of waves.

    make -C ksim-gym-zbot_amd/csrc wavetime && python tests/diag_wavetime.py [--n 8192]

Each pair of envs (one wave) records its start and end on the 100 MHz constant clock, its CU and
its Newton iterations. The script reports the duration spread, how well a pair's duration at step
t - 1 predicts it at step t, and the makespan of a greedy list schedule over the resident slots
for three dispatch orders (index order as launched, longest-predicted-first from step t - 1, and
longest-first with the true durations as the bound).
"""

import argparse
import ctypes as C
import heapq
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ksim-gym-zbot_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402
from zbot_amd import compile_model, default_config  # noqa: E402
from zbot_amd.engine import HipEngine  # noqa: E402


def list_schedule(dur, order, slots):
    """Makespan of handing the units out in `order` to `slots` identical slots as they free up."""
    h = [0.0] * slots
    for i in order:
        t = heapq.heappop(h)
        heapq.heappush(h, t + dur[i])
    return max(h)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=8192)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--steps", type=int, default=24)
    ap.add_argument("--slots", type=int, default=2048, help="resident workgroups (8 per CU)")
    ap.add_argument("--out", default="")
    ap.add_argument("--raw", default="", help="npz of the per-unit records")
    args = ap.parse_args()
    lib = os.path.join(ROOT, "ksim-gym-zbot_amd", "zbot_amd", "libzbot_hip_wavetime.so")
    cm = compile_model()
    eng = HipEngine(cm, default_config(solver="newton"), args.n, lib_path=lib)
    eng.L.zb_get_stamps.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p]
    eng.reset()
    npair = (args.n + 1) // 2
    g = torch.Generator(device="cuda").manual_seed(0)
    bias = torch.tensor([cm.cmodel.joint_bias[i] for i in range(20)], device="cuda")
    acts = bias + 0.05 * torch.randn(64, args.n, 20, device="cuda", generator=g)
    buf = torch.zeros(args.n, 20, dtype=torch.int64, device="cuda")
    rec = []
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for t in range(args.warmup + args.steps):
        ev0.record()
        eng.step(acts[t % 64])
        ev1.record()
        eng.L.zb_get_stamps(eng.h, buf.data_ptr(), eng._stream())
        torch.cuda.synchronize()
        if t >= args.warmup:
            K = int(os.environ.get("ZB_STEP_CHUNKS", "1"))  # the bench sizes here are unchunked by default
            w = buf.view(-1)[: K * npair * 4].view(K * npair, 4).cpu().numpy().astype(np.int64)
            rec.append((w, ev0.elapsed_time(ev1)))
    if args.raw:
        np.savez_compressed(args.raw, w=np.stack([r[0] for r in rec]), ms=np.array([r[1] for r in rec]))
    if rec[0][0].shape[0] != npair:
        print("chunked launch: raw records only")
        return
    res = {"n": args.n, "pairs": npair, "slots": args.slots, "steps": args.steps, "clock": "100 MHz", "per_step": []}
    ratios = {"index": [], "lpt_prev": [], "lpt_true": [], "mean_bound": []}
    corr, corr_it = [], []
    prev = None
    for k, (w, ms) in enumerate(rec):
        t0, t1, cu, it = w[:, 0], w[:, 1], w[:, 2], w[:, 3]
        base = t0.min()
        dur = (t1 - t0).astype(np.float64) / 100.0  # us
        span = (t1.max() - base) / 100.0
        start_rank = np.argsort(np.argsort(t0))
        first = (t0 - base) < (dur.min() * 100 * 0.5)
        row = {"event_ms": round(ms, 4), "span_us": round(float(span), 1), "dur_mean_us": round(float(dur.mean()), 1),
               "dur_std_us": round(float(dur.std()), 1), "dur_min_us": round(float(dur.min()), 1),
               "dur_max_us": round(float(dur.max()), 1), "first_round_pairs": int(first.sum()),
               "first_start_spread_us": round(float((t0[first].max() - base) / 100.0), 2),
               "last_end_minus_p90_end_us": round(float((t1.max() - np.percentile(t1, 90)) / 100.0), 1),
               "start_order_vs_index_rank_corr": round(float(np.corrcoef(start_rank, np.arange(npair))[0, 1]), 4),
               "cus_used": int(len(np.unique(cu)))}
        sim_index = list_schedule(dur, range(npair), args.slots)
        sim_true = list_schedule(dur, np.argsort(-dur, kind="stable"), args.slots)
        ratios["index"].append(sim_index / span)
        ratios["lpt_true"].append(sim_true / sim_index)
        ratios["mean_bound"].append(dur.sum() / args.slots / sim_index)
        row["sim_index_us"] = round(sim_index, 1)
        row["sim_lpt_true_us"] = round(sim_true, 1)
        if prev is not None:
            pdur, pit = prev
            sim_prev = list_schedule(dur, np.argsort(-pdur, kind="stable"), args.slots)
            sim_prev_it = list_schedule(dur, np.argsort(-pit, kind="stable"), args.slots)
            ratios["lpt_prev"].append(sim_prev / sim_index)
            row["sim_lpt_prev_dur_us"] = round(sim_prev, 1)
            row["sim_lpt_prev_iters_us"] = round(sim_prev_it, 1)
            corr.append(float(np.corrcoef(pdur, dur)[0, 1]))
        corr_it.append(float(np.corrcoef(it.astype(np.float64), dur)[0, 1]))
        prev = (dur, it.astype(np.float64))
        res["per_step"].append(row)
    res["summary"] = {
        "sim_index_over_measured_span": round(float(np.mean(ratios["index"])), 4),
        "sim_lpt_prev_over_index": round(float(np.mean(ratios["lpt_prev"])), 4),
        "sim_lpt_true_over_index": round(float(np.mean(ratios["lpt_true"])), 4),
        "perfect_balance_over_index": round(float(np.mean(ratios["mean_bound"])), 4),
        "corr_dur_prev_step": round(float(np.mean(corr)), 4),
        "corr_dur_iters": round(float(np.mean(corr_it)), 4),
    }
    print(json.dumps(res["summary"], indent=1))
    print(json.dumps(res["per_step"][:3], indent=1))
    if args.out:
        with open(args.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
