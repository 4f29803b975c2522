"""Where does the grouped headline step lose time? Slot occupancy of the env groups (diagnostic).

    make -C ksim-gym-zbot_amd/csrc wavetime && python scripts/groups_wavetime.py [--groups 2 --steps 24]

The -DZB_WAVETIME build records every pair's start / end on the 100 MHz constant clock. With G env
groups (bench.py's headline) each group's records are copied out on the group's own
stream right after its launch (no host sync in the loop, so the groups keep running into each
other's drain as in the bench). Over the steady-state window the script reports:
  * slot occupancy: sum of pair durations / (resident slots x window), where the slots are the
    8 one-wave workgroups per CU the occupancy API gives (2048 on 256 CUs);
  * per group and step, the hand-over on its stream: first pair start of launch k + 1 minus the
    last pair end of launch k (the "gap" a kernel trace shows between a stream's launches), and
    how many slots the other group's launch held at that moment;
  * the wall time per step against the mean launch span (first start to last end).
"""

import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ksim-gym-zbot_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402
from zbot_amd import compile_model, default_config  # noqa: E402
from zbot_amd.engine import EnvGroups  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=8192)
    ap.add_argument("--groups", type=int, default=2)
    ap.add_argument("--warmup", type=int, default=8)
    ap.add_argument("--steps", type=int, default=24)
    ap.add_argument("--slots", type=int, default=2048, help="resident one-wave workgroups (8 per CU)")
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    lib = os.path.join(ROOT, "ksim-gym-zbot_amd", "zbot_amd", "libzbot_hip_wavetime.so")
    cm = compile_model()
    eg = EnvGroups(cm, default_config(), a.n, groups=a.groups, lib_path=lib, seed=0)
    import ctypes as C  # noqa: PLC0415

    for e in eg.engines:
        e.L.zb_get_stamps.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p]
    eg.reset()
    g = torch.Generator(device="cuda").manual_seed(0)
    bias = torch.tensor([cm.cmodel.joint_bias[i] for i in range(20)], device="cuda")
    acts = bias + 0.05 * torch.randn(64, a.n, 20, device="cuda", generator=g)
    npairs = [(hi - lo + 1) // 2 for lo, hi in eg.bounds]
    T = a.warmup + a.steps
    # zb_get_stamps copies n x ZB_NSTAMP (20) words per handle; the records are the first 4 per pair
    nst = 20
    bufs = [torch.zeros(T, (hi - lo) * nst, dtype=torch.int64, device="cuda") for lo, hi in eg.bounds]
    torch.cuda.synchronize()
    import time  # noqa: PLC0415

    t_wall = None
    for t in range(T):
        if t == a.warmup:
            eg.join()
            torch.cuda.synchronize()
            t_wall = time.perf_counter()
        eg.step(acts[t % 64], extras=False)
        for gi, (e, s) in enumerate(zip(eg.engines, eg.streams)):
            # the copy is enqueued on the group's stream behind its launch (no host sync)
            rc = e.L.zb_get_stamps(e.h, C.c_void_p(bufs[gi][t].data_ptr()), C.c_void_p(s.cuda_stream))
            assert rc == 0, rc
    eg.join()
    torch.cuda.synchronize()
    wall_ms = (time.perf_counter() - t_wall) * 1e3 / a.steps
    rec = [b[a.warmup:, : p * 4].reshape(a.steps, p, 4).cpu().numpy().astype(np.int64)
           for b, p in zip(bufs, npairs)]  # [steps, pairs, 4]
    t_lo = min(int(r[0, :, 0].min()) for r in rec)
    t_hi = max(int(r[-1, :, 1].max()) for r in rec)
    # steady-state window: from the last group's first launch start to the first group's last launch end
    w0 = max(int(r[0, :, 0].min()) for r in rec)
    w1 = min(int(r[-1, :, 1].max()) for r in rec)
    busy = 0.0
    for r in rec:
        s0 = np.clip(r[:, :, 0], w0, w1)
        s1 = np.clip(r[:, :, 1], w0, w1)
        busy += float((s1 - s0).sum())
    occ = busy / (a.slots * (w1 - w0))
    spans = [(r[:, :, 1].max(1) - r[:, :, 0].min(1)) / 100.0 for r in rec]  # us per launch
    handover = []
    for gi, r in enumerate(rec):
        for k in range(a.steps - 1):
            end_k = int(r[k, :, 1].max())
            start_next = int(r[k + 1, :, 0].min())
            # slots the other groups held at the moment launch k of group gi ended
            held = 0
            for gj, q in enumerate(rec):
                if gj == gi:
                    continue
                held += int(((q[:, :, 0] <= end_k) & (q[:, :, 1] > end_k)).sum())
            handover.append({"group": gi, "step": k, "gap_us": (start_next - end_k) / 100.0, "other_held": held})
    gaps = np.array([h["gap_us"] for h in handover])
    held = np.array([h["other_held"] for h in handover])
    dur = np.concatenate([((r[:, :, 1] - r[:, :, 0]) / 100.0).ravel() for r in rec])
    # placement: distinct CUs (hardware ids from __smid) per step, and the most pairs one CU ran at once
    cus, crowd = [], []
    for k in range(a.steps):
        ids = np.concatenate([r[k, :, 2] for r in rec])
        t0 = np.concatenate([r[k, :, 0] for r in rec])
        t1 = np.concatenate([r[k, :, 1] for r in rec])
        cus.append(len(np.unique(ids)))
        mid = np.median(t0)  # a moment inside the first round
        live = (t0 <= mid) & (t1 > mid)
        _, cnt = np.unique(ids[live], return_counts=True)
        crowd.append(int(cnt.max()) if cnt.size else 0)
    res = {
        "n": a.n, "groups": a.groups, "steps": a.steps, "slots": a.slots,
        "wall_ms_per_step": round(wall_ms, 4),
        "records_span_ms_per_step": round((t_hi - t_lo) / 1e5 / a.steps, 4),
        "launch_span_us_mean": round(float(np.mean(np.concatenate(spans))), 1),
        "pair_us_mean": round(float(dur.mean()), 1),
        "slot_occupancy_steady": round(occ, 4),
        "handover_gap_us_mean": round(float(gaps.mean()), 2),
        "handover_gap_us_max": round(float(gaps.max()), 2),
        "handover_gap_note": "includes the zb_get_stamps copy enqueued between a group's launches (a few us)",
        "other_groups_slots_held_at_handover_mean": round(float(held.mean()), 1) if held.size else None,
        "distinct_cus_per_step_mean": round(float(np.mean(cus)), 1),
        "max_pairs_on_one_cu_at_once_mean": round(float(np.mean(crowd)), 2),
        "note": "slot occupancy = sum of pair durations / (slots x steady window); a hand-over gap with the other "
                "groups holding ~all slots is queueing behind them, not idle hardware",
    }
    print(json.dumps(res, indent=1))
    if a.out:
        with open(a.out, "w") as f:
            json.dump({**res, "handover": handover}, f, indent=1)


if __name__ == "__main__":
    main()
