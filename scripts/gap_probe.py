"""Where does the grouped headline step lose time outside the kernels?

Runs the C2 headline loop (8192 envs, 2 EnvGroups) in variants that strip one per-step packet at a
time from the group streams, and times each over the same window:
  bench      EnvGroups.step with the bench's per-launch timing events (fork, 2 x (start, launch,
             end), 2 x tail mark per step)
  noev       no timing events
  nomark     no timing events, tails recorded only at the final join
  nofork     no timing events, no tails, the group streams forked from the caller once
  graph      the nofork loop captured once per window as a HIP graph and replayed
Prints one JSON object: ms per step (median over reps) per variant.

    python scripts/gap_probe.py --steps 200 --reps 5
"""

from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ksim-gym-zbot_amd"))


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--envs", type=int, default=8192)
    ap.add_argument("--variants", default="bench,noev,nomark,nofork,graph")
    ap.add_argument("--configs", default="",
                    help="extra group layouts timed with plain EnvGroups.step, e.g. '1x0,2x2,3x1,4x1' "
                         "(groups x chunks per group launch; chunks 0 = zb_create's automatic choice)")
    args = ap.parse_args()

    import torch  # noqa: PLC0415
    from zbot_amd import compile_model, default_config  # noqa: PLC0415
    from zbot_amd import cstructs as cs  # noqa: PLC0415
    from zbot_amd.constants import JOINT_BIASES  # noqa: PLC0415
    from zbot_amd.engine import EnvGroups  # noqa: PLC0415

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    n = args.envs
    eng = EnvGroups(compile_model(), default_config(), n, groups=2, device=0)
    g = torch.Generator(device=dev)
    g.manual_seed(1234)
    bias = torch.tensor([b for _, b, _ in JOINT_BIASES], device=dev)
    acts = bias + 0.05 * torch.randn(64, n, cs.NJ, device=dev, generator=g)
    K = args.steps
    ev = [[(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(2)]
          for _ in range(K)]
    cur = torch.cuda.current_stream(dev)
    for evt in ev:
        for a, b in evt:
            a.record(cur)
            b.record(cur)

    def raw_steps(t0):
        for t in range(K):
            a_t = acts[(t0 + t) % 64]
            for e, s, (lo, hi) in eng.groups():
                with torch.cuda.stream(s):
                    e.step(a_t[lo:hi], extras=False)

    def run(variant, t0):
        if variant == "bench":
            for t in range(K):
                eng.step(acts[(t0 + t) % 64], extras=False, events=ev[t])
        elif variant == "noev":
            for t in range(K):
                eng.step(acts[(t0 + t) % 64], extras=False)
        elif variant == "nomark":
            eng.fork()
            for t in range(K):
                eng.fork()
                for e, s, (lo, hi) in eng.groups():
                    with torch.cuda.stream(s):
                        e.step(acts[(t0 + t) % 64][lo:hi], extras=False)
            for gi in range(2):
                eng.mark(gi)
        elif variant == "nofork":
            eng.fork()
            raw_steps(t0)
            for gi in range(2):
                eng.mark(gi)
        eng.join()

    out = {"args": vars(args), "ms_per_step": {}, "kernel_avg_ms": None}
    eng.reset()
    for t in range(8):
        eng.step(acts[t], extras=False)
    eng.join()
    torch.cuda.synchronize()
    for variant in args.variants.split(","):
        times = []
        graph = None
        if variant == "graph":
            # capture K steps of both groups: the group streams fork from the capture stream and join back
            side = torch.cuda.Stream(device=dev)
            side.wait_stream(cur)
            graph = torch.cuda.CUDAGraph()
            with torch.cuda.stream(side):
                with torch.cuda.graph(graph, stream=side):
                    cap = torch.cuda.current_stream(dev)
                    fe = torch.cuda.Event()
                    fe.record(cap)
                    for s in eng.streams:
                        s.wait_event(fe)
                    raw_steps(0)
                    for s in eng.streams:
                        je = torch.cuda.Event()
                        je.record(s)
                        cap.wait_event(je)
            torch.cuda.synchronize()
        for rep in range(args.reps):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            if graph is not None:
                graph.replay()
            else:
                run(variant, 8 + rep * K)
            torch.cuda.synchronize()
            times.append((time.perf_counter() - t0) * 1e3 / K)
        out["ms_per_step"][variant] = {"median": statistics.median(times), "min": min(times), "all": times}
        if variant == "bench":
            ks = [a.elapsed_time(b) for evt in ev for a, b in evt]
            out["kernel_avg_ms"] = sum(ks) / len(ks)
        print(variant, out["ms_per_step"][variant]["median"], flush=True, file=sys.stderr)
    eng.check()
    for spec in filter(None, args.configs.split(",")):
        G, ch = (int(x) for x in spec.split("x"))
        if G == 1:
            from zbot_amd.engine import HipEngine  # noqa: PLC0415

            e2 = HipEngine(compile_model(), default_config(), n, device=0)
            e2.set_step_chunks(ch)
        else:
            e2 = EnvGroups(compile_model(), default_config(), n, groups=G, device=0, chunks=ch)
        e2.reset()
        for t in range(8):
            e2.step(acts[t], extras=False)
        e2.join()
        torch.cuda.synchronize()
        times = []
        for rep in range(args.reps):
            t0 = time.perf_counter()
            for t in range(K):
                e2.step(acts[(8 + t) % 64], extras=False)
            e2.join()
            torch.cuda.synchronize()
            times.append((time.perf_counter() - t0) * 1e3 / K)
        e2.check()
        out["ms_per_step"][f"G{G}_chunks{ch}"] = {"median": statistics.median(times), "min": min(times), "all": times}
        print(spec, statistics.median(times), flush=True, file=sys.stderr)
        del e2
    print(json.dumps(out))


if __name__ == "__main__":
    main()
