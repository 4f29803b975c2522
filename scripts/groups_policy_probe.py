"""Actor-in-the-loop with env groups: which stream arrangement keeps the GRU actor launches from
stalling the step launches of the other group?

    python scripts/groups_policy_probe.py [--n 8192] [--steps 48]

Variants (each: 2 warm-up control steps, then --steps timed, best of --reps):
  one      one handle, actor -> zb_step on the current stream (PolicyRollout on a HipEngine)
  groups   EnvGroups(G): each group's actor -> zb_step chain on the group's stream
  prio     as groups, the group streams created with high priority
  actprio  as groups, each group's actor on its own high-priority stream (event hand-offs)
A "+wave" suffix runs the actor in the one-wave layout (ZB_POL_LAYOUT_WAVE); "priostag" / "groupsstag"
stagger the groups' first actor launches (PolicyRollout(stagger=True)).
"""

import argparse
import gc
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ksim-gym-zbot_amd"))

import torch  # noqa: E402
from zbot_amd import compile_model, default_config  # noqa: E402
from zbot_amd import policy as P  # noqa: E402
from zbot_amd.engine import EnvGroups, HipEngine  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=8192)
    ap.add_argument("--steps", type=int, default=48)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--groups", type=int, default=2)
    ap.add_argument("--variants", default="one,groups,prio,actprio")
    ap.add_argument("--chunks", type=int, default=1, help="EnvGroups chunks (0: automatic)")
    args = ap.parse_args()
    cm = compile_model()
    cfg = default_config()
    n, T = args.n, args.steps
    actor = P.GruPolicy(P.ACTOR, P.init_params(P.ACTOR, seed=0))
    for vv in args.variants.split(","):
        # drop the previous variant's handles first: a handle freed later by the garbage collector
        # (hipFree synchronizes the device) would stall the next variant's timed loop
        eng = ro = run = None
        gc.collect()
        torch.cuda.synchronize()
        v, _, lay = vv.partition("+")  # "+wave": the one-wave actor layout
        actor.set_layout({"wave": P.LAYOUT_WAVE, "wave2": P.LAYOUT_WAVE2, "wave4": P.LAYOUT_WAVE4}.get(lay, P.LAYOUT_BLOCK))
        if v == "one":
            eng = HipEngine(cm, cfg, n, seed=1)
        else:
            eng = EnvGroups(cm, cfg, n, groups=args.groups, seed=1, priority=-1 if v.startswith("prio") else 0,
                            chunks=args.chunks)
        if v == "actprio":
            astreams = [torch.cuda.Stream(priority=-1) for _ in range(eng.G)]
            carry = actor.initial_carry(n)
            eng.reset(extras=False)
            acts = torch.empty(n, P.JOINTS, device="cuda")
            obs = eng.obs_actor

            def run(k, t0):
                eng.fork()
                for t in range(t0, t0 + k):
                    for g, (e, s, (lo, hi)) in enumerate(eng.groups()):
                        a_s = astreams[g]
                        ev = torch.cuda.Event()
                        ev.record(s)
                        a_s.wait_event(ev)
                        with torch.cuda.stream(a_s):
                            actor.actor(obs[lo:hi], carry[lo:hi], reset=eng.done[lo:hi] if t > 0 else None,
                                        seed=1, env_offset=lo, step=t, actions=acts[lo:hi])
                        ev2 = torch.cuda.Event()
                        ev2.record(a_s)
                        s.wait_event(ev2)
                        with torch.cuda.stream(s):
                            e.step(acts[lo:hi], extras=False)
                        eng.mark(g)
                eng.join()
        else:
            ro = P.PolicyRollout(eng, actor, seed=1, stagger=v.endswith("stag"))
            ro.reset()

            def run(k, t0):
                ro.run(k)
        run(2, 0)
        torch.cuda.synchronize()
        best = 1e9
        t = 2
        for _ in range(args.reps):
            w0 = time.perf_counter()
            run(T, t)
            torch.cuda.synchronize()
            best = min(best, time.perf_counter() - w0)
            t += T
        print(json.dumps({"variant": vv, "n": n, "groups": 1 if v == "one" else args.groups,
                          "env_steps_per_s": round(n * T / best / 1e6, 4)}), flush=True)


if __name__ == "__main__":
    main()
