"""The actor in the rollout loop by policy layout and env-group count (diagnostic, GPU): C2's 8192 envs,
PolicyRollout over EnvGroups (or one HipEngine for one group), 48 timed control steps after 2, best of
3; env-steps/s per (layout, groups).

    python scripts/policy_loop_probe.py [--layouts block,wave2] [--groups 1,2,3]
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
from zbot_amd import policy as P  # noqa: E402
from zbot_amd.engine import EnvGroups, HipEngine  # noqa: E402

LAYOUTS = {"block": P.LAYOUT_BLOCK, "wave": P.LAYOUT_WAVE, "wave2": P.LAYOUT_WAVE2, "wave4": P.LAYOUT_WAVE4}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--layouts", default="block,wave2")
    ap.add_argument("--groups", default="1,2,3")
    ap.add_argument("--n", type=int, default=8192)
    ap.add_argument("--steps", type=int, default=48)
    a = ap.parse_args()
    cm = compile_model()
    cfg = default_config()
    for lay in a.layouts.split(","):
        for g in (int(x) for x in a.groups.split(",")):
            eng = HipEngine(cm, cfg, a.n, seed=3) if g == 1 else EnvGroups(cm, cfg, a.n, groups=g, seed=3)
            actor = P.GruPolicy(P.ACTOR, P.init_params(P.ACTOR, seed=0), layout=LAYOUTS[lay])
            ro = P.PolicyRollout(eng, actor, seed=1)
            ro.reset()
            ro.run(2)
            torch.cuda.synchronize()
            best = 0.0
            for _ in range(3):
                t0 = time.perf_counter()
                ro.run(a.steps)
                torch.cuda.synchronize()
                best = max(best, a.n * a.steps / (time.perf_counter() - t0))
            print(json.dumps({"layout": lay, "groups": g, "env_steps_per_s": best}), flush=True)
            del ro, actor, eng
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
