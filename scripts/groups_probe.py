"""Env groups on their own HIP streams: does splitting one GPU's envs into G engine handles, each
stepping on its own stream, fill the drain at the end of every step launch?

    python scripts/groups_probe.py [--n 8192] [--config c2]

For G in --groups, the same envs (global ids kept through env_offset, so every RNG stream is the
same) run as G handles of n/G envs; step t of group g waits only on step t - 1 of group g. The
script times --steps control steps after --warmup, and checks that the final states of every G
are bit-identical to G = 1.
"""

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ksim-gym-zbot_amd"))

import torch  # noqa: E402
from zbot_amd import compile_model, default_config  # noqa: E402
from zbot_amd import cstructs as cs  # noqa: E402
from zbot_amd.constants import JOINT_BIASES  # noqa: E402
from zbot_amd.engine import HipEngine  # noqa: E402


def run(cm, cfg, n, G, acts, warmup, steps, reps, prio=0):
    ng = n // G
    engs = [HipEngine(cm, cfg, ng, env_offset=g * ng) for g in range(G)]
    streams = [torch.cuda.Stream(priority=prio) for _ in range(G)]
    for e, s in zip(engs, streams):
        with torch.cuda.stream(s):
            e.reset()
    torch.cuda.synchronize()

    def steps_(t0, k):
        for t in range(t0, t0 + k):
            a = acts[t % acts.shape[0]]
            for g, (e, s) in enumerate(zip(engs, streams)):
                with torch.cuda.stream(s):
                    e.step(a[g * ng:(g + 1) * ng], extras=False)

    steps_(0, warmup)
    torch.cuda.synchronize()
    best = []
    t = warmup
    for _ in range(reps):
        w0 = time.perf_counter()
        steps_(t, steps)
        torch.cuda.synchronize()
        best.append(time.perf_counter() - w0)
        t += steps
    st = []
    for e, s in zip(engs, streams):
        with torch.cuda.stream(s):
            st.append(e.get_state())
    torch.cuda.synchronize()
    return n * steps / min(best), n * steps / (sum(best) / len(best)), torch.cat(st)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=8192)
    ap.add_argument("--config", default="c2")
    ap.add_argument("--groups", default="1,2,4")
    ap.add_argument("--warmup", type=int, default=8)
    ap.add_argument("--steps", type=int, default=64)
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    cm = compile_model()
    cfg = default_config(push=args.config == "c3", randomize=args.config == "c5")
    g = torch.Generator(device="cuda").manual_seed(1234)
    bias = torch.tensor([b for _, b, _ in JOINT_BIASES], device="cuda")
    acts = bias + 0.05 * torch.randn(64, args.n, cs.NJ, device="cuda", generator=g)
    ref = None
    out = {}
    for GG in args.groups.split(","):
        G = int(GG.rstrip("p"))  # "4p": high-priority streams
        best, mean, st = run(cm, cfg, args.n, G, acts, args.warmup, args.steps, args.reps, -1 if GG.endswith("p") else 0)
        same = None
        if ref is None:
            ref = st
        else:
            same = bool(torch.equal(st.view(torch.int32), ref.view(torch.int32)))
        out[GG] = dict(best=round(best / 1e6, 4), mean=round(mean / 1e6, 4), bit_identical_to_G1=same)
        print(json.dumps({"n": args.n, "config": args.config, "groups": GG, **out[GG]}), flush=True)


if __name__ == "__main__":
    main()
