"""The handle's kernel instantiation is fixed at zb_create: ZB_FORCE_XG, the
profiling switch that runs a two-sole model on the general-collider kernels, is read once when the
handle is created (zb_capi.cpp: ZbHandle.xg), so setting it afterwards neither launches the XG
kernel on a handle without its second-bank scratch nor changes any result."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch_gpu():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch


def _run(torch, cm, force_after_create: bool):
    from zbot_amd import default_config
    from zbot_amd.engine import HipEngine

    eng = HipEngine(cm, default_config(push=True, randomize=True), 64, seed=3)
    g = torch.Generator(device="cuda").manual_seed(11)
    acts = 0.05 * torch.randn(4, 64, 20, device="cuda", generator=g)
    if force_after_create:
        os.environ["ZB_FORCE_XG"] = "1"
    try:
        outs = [eng.step(acts[t])["reward"].clone() for t in range(4)]
        torch.cuda.synchronize()
    finally:
        os.environ.pop("ZB_FORCE_XG", None)
    return eng.get_state().cpu().numpy(), torch.stack(outs).cpu().numpy()


def test_force_xg_after_create_changes_nothing(torch_gpu, cmodel):
    assert "ZB_FORCE_XG" not in os.environ
    st0, r0 = _run(torch_gpu, cmodel, False)
    st1, r1 = _run(torch_gpu, cmodel, True)
    assert np.array_equal(st0.view(np.uint32), st1.view(np.uint32))
    assert np.array_equal(r0.view(np.uint32), r1.view(np.uint32))
