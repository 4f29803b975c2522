"""Diagnostic: how much Newton work two envs sharing a wavefront waste on each other (the wave
runs the larger iteration count), and whether pairing envs by the previous step's counts would
recover it (GPU box: python scripts/iters_probe.py)."""
import sys, os
sys.path.insert(0, "ksim-gym-zbot_amd")
import torch
from zbot_amd import compile_model, default_config
from zbot_amd.engine import HipEngine
cm = compile_model(); n = 8192
eng = HipEngine(cm, default_config(), n, seed=1)
eng.reset()
bias = torch.tensor([cm.cmodel.joint_bias[i] for i in range(20)], device="cuda")
g = torch.Generator(device="cuda"); g.manual_seed(0)
tot_rand = tot_sorted = tot_mean = 0.0
prev = None
for t in range(40):
    eng.step(bias + 0.05 * torch.randn(n, 20, device="cuda", generator=g), extras=False)
    it = eng.solver_iters().float()
    if t >= 8:
        pairs = it.view(-1, 2)
        tot_rand += pairs.max(1).values.sum().item()
        tot_mean += it.sum().item() / 2
        if prev is not None:
            # pairing by the previous step's counts (what a per-step permutation could do)
            order = torch.argsort(prev)
            sp = it[order].view(-1, 2)
            tot_sorted += sp.max(1).values.sum().item()
        else:
            tot_sorted += pairs.max(1).values.sum().item()
    prev = it.clone()
print(f"sum of wave max (current pairing) {tot_rand:.0f}; ideal (no waste) {tot_mean:.0f}; "
      f"sorted by previous step {tot_sorted:.0f}; waste now {(tot_rand - tot_mean) / tot_rand:.3%}, "
      f"with sorting {(tot_sorted - tot_mean) / tot_sorted:.3%}")
print("iters per env-step: mean", it.mean().item(), "std", it.std().item(), "min", it.min().item(), "max", it.max().item())
