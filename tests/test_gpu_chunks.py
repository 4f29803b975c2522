"""Chunked step (zb_step's substeps split into work units handed between workgroups inside one
launch) against the unchunked step: bit for bit, with odd env counts (a ghost
team), pushes, randomization and automatic resets. ZB_STEP_CHUNKS is read when an engine is
created."""
import os

import pytest

from zbot_amd import default_config

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch_gpu():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch


def make(cm, cfg, n, k):
    from zbot_amd.engine import HipEngine

    old = os.environ.get("ZB_STEP_CHUNKS")
    os.environ["ZB_STEP_CHUNKS"] = str(k)
    try:
        return HipEngine(cm, cfg, n, seed=3)
    finally:
        if old is None:
            os.environ.pop("ZB_STEP_CHUNKS")
        else:
            os.environ["ZB_STEP_CHUNKS"] = old


def same(torch, a, b):
    if a.dtype == torch.float32:
        return torch.equal(a.view(torch.int32), b.view(torch.int32))
    return torch.equal(a, b)


@pytest.mark.parametrize("n,k,push", [(37, 2, True), (37, 7, True), (64, 20, False), (1, 3, True)])
def test_chunked_step_bit_exact(torch_gpu, cmodel, n, k, push):
    torch = torch_gpu
    cfg = default_config(solver="newton", push=push, randomize=push)
    ref, chk = make(cmodel, cfg, n, 1), make(cmodel, cfg, n, k)
    ref.reset()
    chk.reset()
    g = torch.Generator(device="cuda")
    g.manual_seed(5)
    bias = torch.tensor([cmodel.cmodel.joint_bias[i] for i in range(20)], device="cuda")
    dones = 0
    for t in range(60):
        # large action noise: the robot falls, so automatic resets happen inside chunks' launches
        act = bias + 0.4 * torch.randn(n, 20, device="cuda", generator=g)
        o1 = {k_: v.clone() for k_, v in ref.step(act, curriculum=0.5).items()}
        o2 = chk.step(act, curriculum=0.5)
        for name in o1:
            assert same(torch, o1[name], o2[name]), (t, name)
        assert same(torch, ref.get_state(), chk.get_state()), t
        assert torch.equal(ref.solver_iters(), chk.solver_iters()), t
        dones += int(o1["done"].sum().item())
    assert same(torch, ref.get_stats(), chk.get_stats())
    assert same(torch, ref.get_rand(), chk.get_rand())
    if push:
        assert dones > 0  # the resets were exercised


@pytest.mark.parametrize("n,push,steps", [(8192, False, 6), (6144, False, 6), (5121, True, 40)])
def test_default_chunking(torch_gpu, cmodel, n, push, steps):
    """The library's own chunk choice (whole rounds of resident workgroups: unchunked, as at the
    C2 bench size of 8192 envs; a partial last round: 2 or 4 chunks) against unchunked; at 5121
    envs (4 chunks) with pushes, per-env randomization and resets."""
    torch = torch_gpu
    from zbot_amd.engine import HipEngine

    cfg = default_config(solver="newton", push=push, randomize=push)
    old = os.environ.pop("ZB_STEP_CHUNKS", None)
    try:
        auto = HipEngine(cmodel, cfg, n, seed=3)
    finally:
        if old is not None:
            os.environ["ZB_STEP_CHUNKS"] = old
    ref = make(cmodel, cfg, n, 1)
    auto.reset()
    ref.reset()
    bias = torch.tensor([cmodel.cmodel.joint_bias[i] for i in range(20)], device="cuda")
    std = 0.4 if push else 0.05
    for t in range(steps):
        act = bias + std * torch.randn(n, 20, device="cuda")
        o1 = {k_: v.clone() for k_, v in ref.step(act).items()}
        o2 = auto.step(act)
        for name in o1:
            assert same(torch, o1[name], o2[name]), (t, name)
    assert same(torch, ref.get_state(), auto.get_state())
    assert torch.equal(ref.solver_iters(), auto.solver_iters())
    assert same(torch, ref.get_stats(), auto.get_stats())


@pytest.mark.parametrize("variant", ["limbs", "mesh"])
def test_chunked_step_bit_exact_general_colliders(torch_gpu, oracle_mod, variant):
    """The general-collider kernels (a shin box and a hand capsule beside the soles, DESIGN.md
    §4j; or the convex mesh sole, shin and hand, round 5) chunked against unchunked, from states where
    those colliders touch the floor, so that the second contact bank and its global-scratch rows are
    in use across the hand-offs."""
    torch = torch_gpu
    import numpy as np

    import collider_util as U
    from zbot_amd import compile_model
    from zbot_amd import cstructs as cs

    cm = compile_model(getattr(U, f"{variant}_desc")())
    cfg = default_config(solver="newton", push=True, randomize=True)
    n = 37
    ref, chk = make(cm, cfg, n, 1), make(cm, cfg, n, 5)
    env = oracle_mod.OracleEnv(cm.cmodel, cfg, n, seed=3)
    env.reset()
    g = torch.Generator(device="cuda")
    g.manual_seed(9)
    bias = torch.tensor([cm.cmodel.joint_bias[i] for i in range(20)], device="cuda")
    names = [gd["name"] for gd in cm.desc["geoms"]]  # collider_util's order (document order)
    extra = [names.index("right_shin"), names.index("left_hand")]
    touched = 0
    for t in range(3):
        st = env.state.copy()
        st[:, :27] = U.touching_states(cm, n, seed=20 + t).astype(np.float32)
        st[:, 32:58] = 0.0
        st[:, cs.S_QACCW:cs.S_QACCW + 32] = 0.0
        touched += sum(any(len(c[i]) for i in extra) for c in
                       (U.contacts(cm, q) for q in st[:, :27].astype(np.float64)))
        for h in (ref, chk):
            h.set_state(torch.from_numpy(st.copy()))
            h.set_rand(torch.from_numpy(env.rand.copy()))
        act = bias + 0.3 * torch.randn(n, 20, device="cuda", generator=g)
        o1 = {k_: v.clone() for k_, v in ref.step(act).items()}
        o2 = chk.step(act)
        for name in o1:
            assert same(torch, o1[name], o2[name]), (t, name)
        assert same(torch, ref.get_state(), chk.get_state()), t
        assert torch.equal(ref.solver_iters(), chk.solver_iters()), t
    assert touched > 0  # the shin or the hand touches in some of the states
