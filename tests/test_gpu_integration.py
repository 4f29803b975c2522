"""INTEGRATION.md's reference-side binding runs as documented.

The `ZbotHipEnv` code block of INTEGRATION.md §2 — the ctypes stub a ksim maintainer would put next
to train.py — is executed verbatim (only the library path is made absolute) and stepped on 8 envs.
Its observations, rewards, done and success flags must be the bits of the package's HipEngine on the
same seed and actions: both are the same C-ABI entry points, bound twice.
"""

import os
import re

import numpy as np
import pytest

from zbot_amd import default_config

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _binding_block() -> str:
    txt = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    blocks = [b for b in re.findall(r"```python\n(.*?)```", txt, flags=re.S) if "class ZbotHipEnv" in b]
    assert len(blocks) == 1
    return blocks[0]


def test_documented_binding_steps_like_hipengine(cmodel):
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from zbot_amd.engine import LIB_PATH, HipEngine, load_library

    load_library()  # builds nothing; raises if the library is missing
    src = _binding_block().replace('C.CDLL("libzbot_hip.so")', f"C.CDLL({LIB_PATH!r})")
    ns: dict = {}
    exec(compile(src, "INTEGRATION.md:ZbotHipEnv", "exec"), ns)  # noqa: S102 - our own document
    n, T = 8, 12
    env = ns["ZbotHipEnv"](n, seed=5)
    ref = HipEngine(cmodel, default_config(), n, seed=5)  # zb_default_config: CG, as default_config()
    oa, oc = env.reset()
    r = ref.reset()
    torch.cuda.synchronize()
    np.testing.assert_array_equal(oa.cpu().numpy(), r["obs_actor"].cpu().numpy())
    np.testing.assert_array_equal(oc.cpu().numpy(), r["obs_critic"].cpu().numpy())
    g = torch.Generator(device="cuda").manual_seed(1)
    bias = torch.tensor([cmodel.cmodel.joint_bias[a] for a in range(20)], device="cuda")
    for t in range(T):
        a = (bias + 0.2 * torch.randn(n, 20, device="cuda", generator=g)).contiguous()
        oa, oc, rew, done, succ = env.step(a, 1.0)
        r = ref.step(a, curriculum=1.0)
        torch.cuda.synchronize()
        for got, k in ((oa, "obs_actor"), (oc, "obs_critic"), (rew, "reward"), (done, "done"), (succ, "success")):
            np.testing.assert_array_equal(got.cpu().numpy(), r[k].cpu().numpy(), err_msg=f"{k} at step {t}")
    assert torch.isfinite(rew).all()
