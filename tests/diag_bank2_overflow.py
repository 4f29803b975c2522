"""How often the second contact-row bank's two-geom cap binds on the task (diagnostic, GPU).

    python tests/diag_bank2_overflow.py [--n 32768] [--steps 256] [--sigma 0.05] [--model many]

The nine-collider model (assets/zbot_like_many.xml) at C3 (pushes) stepped from reset with actions
JOINT_BIASES + sigma N(0,1): per step, the envs whose bank-2 selection found more than two colliders
within reach of the floor in some substep of that step (flag bit 1 of ZB_S_NAN, cleared with the
episode), and of those how many end their episode in that same step. Prints the totals.
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ksim-gym-zbot_amd"))

import torch  # noqa: E402
from zbot_amd import compile_model, cstructs as cs, default_config  # noqa: E402
from zbot_amd.engine import HipEngine  # noqa: E402
from zbot_amd.mjcf import load_mjcf  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=32768)
    ap.add_argument("--steps", type=int, default=256)
    ap.add_argument("--sigma", type=float, default=0.05)
    ap.add_argument("--model", default="zbot_like_many.xml")
    ap.add_argument("--push", type=int, default=1)
    a = ap.parse_args()
    cm = compile_model(load_mjcf(os.path.join(ROOT, "ksim-gym-zbot_amd", "assets", a.model)))
    eng = HipEngine(cm, default_config(push=bool(a.push)), a.n, seed=11)
    bias = torch.tensor([cm.cmodel.joint_bias[i] for i in range(20)], device="cuda")
    g = torch.Generator(device="cuda")
    g.manual_seed(5)
    eng.reset()
    flagged_steps = flagged_ending = ends = 0
    prev = torch.zeros(a.n, dtype=torch.bool, device="cuda")
    for t in range(a.steps):
        out = eng.step(bias + a.sigma * torch.randn(a.n, 20, device="cuda", generator=g), extras=False)
        st = eng.get_state()
        flag = (st[:, cs.S_NAN].view(torch.int32) & 2) != 0
        done = out["done"].bool()
        flagged_steps += int(flag.sum())
        flagged_ending += int((flag & done).sum())
        ends += int(done.sum())
        prev = flag
    torch.cuda.synchronize()
    print(f"{a.model} n={a.n} steps={a.steps} sigma={a.sigma} push={a.push}: episode ends {ends}; env-steps with the "
          f"bank-2 overflow flag {flagged_steps} ({flagged_steps / (a.n * a.steps):.2e} of all), of them in a "
          f"terminating step {flagged_ending}; still flagged at the end {int(prev.sum())}")


if __name__ == "__main__":
    main()
