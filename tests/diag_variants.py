"""A/B timing of library variants (same sources, different build flags) in ONE process.

    python tests/diag_variants.py lib1.so lib2.so ... [--n 8192 --steps 16 --rounds 3]
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ksim-gym-zbot_amd"))
import torch  # noqa: E402
from zbot_amd import compile_model, default_config  # noqa: E402
from zbot_amd.engine import EnvGroups, HipEngine  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs="+")
    ap.add_argument("--n", type=int, default=8192)
    ap.add_argument("--steps", type=int, default=16)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--groups", type=int, default=1, help="env groups on their own streams (EnvGroups)")
    ap.add_argument("--model", default=None, help="an MJCF file (e.g. the limbs asset) instead of the default model")
    ap.add_argument("--box-rule", default="mujoco", choices=["mujoco", "mjx"], help="compile_model(box_rule=...)")
    ap.add_argument("--solver", default="cg", choices=["cg", "newton"])
    a = ap.parse_args()
    if a.model:
        from zbot_amd.mjcf import load_mjcf  # noqa: PLC0415

        cm = compile_model(load_mjcf(a.model), box_rule=a.box_rule)
    else:
        cm = compile_model(box_rule=a.box_rule)
    bias = torch.tensor([cm.cmodel.joint_bias[i] for i in range(20)], device="cuda")
    acts = [bias + 0.05 * torch.randn(a.n, 20, device="cuda") for _ in range(8)]
    if a.groups > 1:
        engs = [EnvGroups(cm, default_config(solver=a.solver), a.n, groups=a.groups, lib_path=os.path.abspath(p), seed=0)
                for p in a.libs]
    else:
        engs = [HipEngine(cm, default_config(solver=a.solver), a.n, lib_path=os.path.abspath(p), seed=0) for p in a.libs]
    for e in engs:
        e.reset()
        for t in range(3):
            e.step(acts[t])
    torch.cuda.synchronize()
    # screening parity: every variant against the first library after the same 3 steps
    ref = engs[0].get_state()
    for p, e in zip(a.libs[1:], engs[1:]):
        st = e.get_state()
        dq = (st[:, :27] - ref[:, :27]).abs().max().item()
        dv = (st[:, 32:58] - ref[:, 32:58]).abs().max().item()
        bad = int((~torch.isfinite(st[:, :58])).sum().item())
        print(f"{os.path.basename(p):32s} vs {os.path.basename(a.libs[0])}: max|dqpos| {dq:.2e} max|dqvel| {dv:.2e} nonfinite {bad}")
    res = {p: [] for p in a.libs}
    for r in range(a.rounds):
        for p, e in zip(a.libs, engs):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for t in range(a.steps):
                e.step(acts[t % 8], extras=False)
            if a.groups > 1:
                e.join()
            torch.cuda.synchronize()
            res[p].append(a.n * a.steps / (time.perf_counter() - t0))
    for p in a.libs:
        v = sorted(res[p])
        print(f"{os.path.basename(p):32s} median {v[len(v)//2]:.0f} env-steps/s  all {[round(x) for x in v]}")


if __name__ == "__main__":
    main()
