"""How much do the two envs of a wave differ in Newton iterations? (diagnostic, round 3)

A wave runs two envs (teams 2k, 2k+1) in lockstep: every Newton / line-search loop runs until both
teams leave it, so per control step the wave pays about max(it_2k, it_2k+1) where each env needs
its own count. This measures, at C2 with the bench's actions, the step-level ratio
sum_k max(it_2k, it_2k+1) / (sum_e it_e / 2), how well an env's count predicts its next one, and
the same ratio if the pairs were formed by sorting the envs on their previous step's count.
(Step-level sums hide the per-substep mismatch, so the true lockstep overhead is larger.)

    python scripts/pairing_probe.py [--n 8192 --steps 24]
"""

from __future__ import annotations

import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ksim-gym-zbot_amd"))


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=8192)
    ap.add_argument("--steps", type=int, default=24)
    ap.add_argument("--sigma", type=float, default=0.05)
    a = ap.parse_args()
    import numpy as np
    import torch
    from zbot_amd import compile_model, default_config
    from zbot_amd import cstructs as cs
    from zbot_amd.constants import JOINT_BIASES
    from zbot_amd.engine import HipEngine

    eng = HipEngine(compile_model(), default_config(), a.n, seed=0)
    eng.reset()
    g = torch.Generator(device="cuda").manual_seed(1234)
    bias = torch.tensor([b for _, b, _ in JOINT_BIASES], device="cuda")
    its = []
    for t in range(a.steps):
        eng.step(bias + a.sigma * torch.randn(a.n, cs.NJ, device="cuda", generator=g), extras=False)
        its.append(eng.solver_iters().cpu().numpy().astype(np.float64))
    it = np.stack(its[4:])  # skip the settling after reset
    pair = it.reshape(it.shape[0], -1, 2)
    lock = pair.max(-1).sum(-1) / (it.sum(-1) / 2)
    corr = [float(np.corrcoef(it[t], it[t + 1])[0, 1]) for t in range(it.shape[0] - 1)]
    sorted_lock = []
    for t in range(1, it.shape[0]):
        order = np.argsort(it[t - 1], kind="stable")
        p = it[t][order].reshape(-1, 2)
        sorted_lock.append(p.max(-1).sum() / (it[t].sum() / 2))
    out = {"envs": a.n, "steps": a.steps, "mean_iters_per_env_step": float(it.mean()),
           "lockstep_ratio_env_pairs": float(lock.mean()),
           "lockstep_ratio_sorted_by_previous_step": float(np.mean(sorted_lock)),
           "step_to_step_corr": float(np.mean(corr)),
           "iters_percentiles": {str(q): float(np.percentile(it, q)) for q in (5, 25, 50, 75, 95)}}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
