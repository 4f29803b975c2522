"""Step layouts against the env count (diagnostic): env-steps/s of zb_step with two
envs per wave (pairs) and one (solo), one handle, C2 workload, for the latency-bound small counts
(train.py's 512 among them) and a few above one wave per SIMD. Each point alternates the layouts
over rounds in one process; final states are compared (the layouts give the same bits).

    python scripts/layout_sweep.py [--sizes 128,256,512,1024,1536,2048,4096] [--steps 40 --rounds 5]
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
from zbot_amd.engine import HipEngine, LAYOUT_PAIRS, LAYOUT_SOLO  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="128,256,512,1024,1536,2048,4096")
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--rounds", type=int, default=5)
    a = ap.parse_args()
    cm = compile_model()
    bias = torch.tensor([cm.cmodel.joint_bias[i] for i in range(20)], device="cuda")
    out = {"steps": a.steps, "rounds": a.rounds, "points": []}
    for n in [int(x) for x in a.sizes.split(",")]:
        g = torch.Generator(device="cuda").manual_seed(n)
        acts = [bias + 0.05 * torch.randn(n, 20, device="cuda", generator=g) for _ in range(8)]
        engs = {}
        for name, lay in (("pairs", LAYOUT_PAIRS), ("solo", LAYOUT_SOLO)):
            e = HipEngine(cm, default_config(), n, seed=0)
            e.set_step_layout(lay)
            e.reset()
            for t in range(4):
                e.step(acts[t % 8], extras=False)
            engs[name] = e
        torch.cuda.synchronize()
        same = bool(torch.equal(engs["pairs"].get_state(), engs["solo"].get_state()))
        res = {k: [] for k in engs}
        for _ in range(a.rounds):
            for k, e in engs.items():
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for t in range(a.steps):
                    e.step(acts[t % 8], extras=False)
                torch.cuda.synchronize()
                res[k].append(n * a.steps / (time.perf_counter() - t0))
        med = {k: sorted(v)[len(v) // 2] for k, v in res.items()}
        pt = {"n": n, "same_bits_after_4_steps": same, "pairs_env_steps_per_s": med["pairs"],
              "solo_env_steps_per_s": med["solo"], "solo_over_pairs": med["solo"] / med["pairs"],
              "pairs_ms_per_step": 1e3 * n / med["pairs"], "solo_ms_per_step": 1e3 * n / med["solo"]}
        out["points"].append(pt)
        print(json.dumps(pt), file=sys.stderr, flush=True)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
