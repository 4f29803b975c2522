"""Fixed C2 workload on one library build (diagnostic only): reset + N zb_step launches.

    [MODEL=path.xml] python scripts/variant_driver.py evariants/libeng_x.so [steps]
Used under rocprofv3 --pmc by scripts/pmc_variants.sh to count the step kernel's instructions.
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ksim-gym-zbot_amd"))
import torch  # noqa: E402
from zbot_amd import compile_model, default_config  # noqa: E402
from zbot_amd.engine import HipEngine  # noqa: E402

lib = os.path.abspath(sys.argv[1])
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 4
if os.environ.get("MODEL"):  # an MJCF file, e.g. the limbs asset (the general-collider kernels)
    from zbot_amd.mjcf import load_mjcf  # noqa: E402

    cm = compile_model(load_mjcf(os.environ["MODEL"]))
else:
    cm = compile_model()
g = torch.Generator(device="cuda")
g.manual_seed(0)
bias = torch.tensor([cm.cmodel.joint_bias[i] for i in range(20)], device="cuda")
n = int(os.environ.get("N", "8192"))  # 512: train.py's size, one wave per CU (scripts/pmc_latency.sh)
eng = HipEngine(cm, default_config(solver=os.environ.get("SOLVER", "cg")), n, seed=1, lib_path=lib)
eng.reset()
for t in range(steps):
    eng.step(bias + 0.05 * torch.randn(n, 20, device="cuda", generator=g), extras=False)
torch.cuda.synchronize()
print("iters/env-step", eng.solver_iters().float().mean().item())
