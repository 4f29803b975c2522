"""Where does the headline's wall time go? (VERDICT r02 "What's weak" 3.)

Replays bench.py's headline loop (C2, EnvGroups, --steps K --warmup W) with every group launch
bracketed by timing events and one origin event recorded on the caller's stream before the first
timed step, so each launch's GPU start / end lands on one timeline; the host's enqueue time of
every step is taken beside it. Prints one JSON object.

    python scripts/headline_probe.py --steps 20 --warmup 5 --groups 2
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ksim-gym-zbot_amd"))


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--groups", type=int, default=2)
    ap.add_argument("--envs", type=int, default=8192)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--mode", default="py", help="py: EnvGroups.step; c: zb_step_groups (one C call per step)")
    args = ap.parse_args()

    import torch  # noqa: PLC0415
    from zbot_amd import compile_model, default_config  # noqa: PLC0415
    from zbot_amd import cstructs as cs  # noqa: PLC0415
    from zbot_amd.constants import JOINT_BIASES  # noqa: PLC0415
    from zbot_amd.engine import EnvGroups, HipEngine  # noqa: PLC0415

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    cm = compile_model()
    cfg = default_config()
    n, G = args.envs, args.groups
    eng = EnvGroups(cm, cfg, n, groups=G, device=0) if G > 1 else HipEngine(cm, cfg, n, device=0)
    T = args.warmup + args.steps
    g = torch.Generator(device=dev)
    g.manual_seed(1234)
    bias = torch.tensor([b for _, b, _ in JOINT_BIASES], device=dev)
    acts = bias + 0.05 * torch.randn(min(T, 64), n, cs.NJ, device=dev, generator=g)
    stream = torch.cuda.current_stream(dev)
    out = {"args": vars(args), "reps": []}
    for rep in range(args.reps):
        eng.reset()
        for t in range(args.warmup):
            eng.step(acts[t % acts.shape[0]], extras=False)
        if G > 1:
            eng.join()
        eng.get_stats(clear=True)
        torch.cuda.synchronize(dev)
        origin = torch.cuda.Event(enable_timing=True)
        ev = [[(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(G)]
              for _ in range(args.steps)]
        host = []
        t0 = time.perf_counter()
        origin.record(stream)
        for t in range(args.steps):
            a_t = acts[(args.warmup + t) % acts.shape[0]]
            if G > 1:
                if args.mode == "c":
                    eng.step_fused(a_t, extras=False, events=ev[t])
                else:
                    eng.step(a_t, extras=False, events=ev[t])
            else:
                ev[t][0][0].record(stream)
                eng.step(a_t, extras=False)
                ev[t][0][1].record(stream)
            host.append(time.perf_counter() - t0)
        if G > 1:
            eng.join()
        t_enq = time.perf_counter() - t0
        torch.cuda.synchronize(dev)
        wall = time.perf_counter() - t0
        starts = [[origin.elapsed_time(ev[t][k][0]) for k in range(G)] for t in range(args.steps)]
        ends = [[origin.elapsed_time(ev[t][k][1]) for k in range(G)] for t in range(args.steps)]
        dur = [e - s for st, en in zip(starts, ends) for s, e in zip(st, en)]
        out["reps"].append({
            "wall_ms": wall * 1e3, "ms_per_step": wall * 1e3 / args.steps, "enqueue_ms": t_enq * 1e3,
            "host_enqueue_ms": [round(h * 1e3, 3) for h in host],
            "gpu_start_ms": [[round(x, 3) for x in s] for s in starts],
            "gpu_end_ms": [[round(x, 3) for x in e] for e in ends],
            "launch_avg_ms": sum(dur) / len(dur),
            "last_end_ms": max(max(e) for e in ends),
        })
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
