"""The solo step layout (one env per wave, the other team a ghost of the same env; zb_set_step_layout,
DESIGN.md §4k) gives the bits of the paired layout: every output and the state after steps with
pushes, per-env randomization, observation noise and automatic resets, the open-loop rollout, and
the general-collider kernels; the automatic choice picks solo while the launch has at most one wave
per SIMD."""

import numpy as np
import pytest

import collider_util as U
from zbot_amd import compile_model, default_config
from zbot_amd import cstructs as cs

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch_gpu():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch


def run(torch, cm, cfg, n, layout, acts, seed=3, force_reset=True):
    from zbot_amd.engine import HipEngine

    eng = HipEngine(cm, cfg, n, seed=seed)
    eng.set_step_layout(layout)
    eng.reset()
    outs = []
    for t, a in enumerate(acts):
        if force_reset and t == 2:
            st = eng.get_state()
            st[::5, 2] = 0.7  # BadZ (train.py:1590): automatic resets of a fifth of the envs
            eng.set_state(st)
        o = eng.step(a)
        outs.append({k: v.cpu().numpy().copy() for k, v in o.items() if v is not None})
    torch.cuda.synchronize()
    return eng, outs, eng.get_state().cpu().numpy(), eng.get_rand().cpu().numpy(), eng.get_stats().cpu().numpy()


@pytest.mark.parametrize("n", [64, 33, 1])
def test_solo_equals_pairs(torch_gpu, cmodel, oracle_mod, n):
    torch = torch_gpu
    from zbot_amd.engine import LAYOUT_PAIRS, LAYOUT_SOLO

    cfg = default_config(push=True, randomize=True)
    acts = [torch.from_numpy(oracle_mod.synthetic_actions(cmodel.cmodel, 3, n, 0, t, std=0.2)).cuda() for t in range(6)]
    ea, oa, sa, ra, ta = run(torch, cmodel, cfg, n, LAYOUT_PAIRS, acts)
    eb, ob, sb, rb, tb = run(torch, cmodel, cfg, n, LAYOUT_SOLO, acts)
    assert ea.step_layout == LAYOUT_PAIRS and eb.step_layout == LAYOUT_SOLO
    assert int(sum(o["done"].sum() for o in oa)) > 0  # the resets happened
    for t, (x, y) in enumerate(zip(oa, ob)):
        for k in x:
            assert np.array_equal(x[k], y[k]), (t, k)
    assert np.array_equal(sa, sb) and np.array_equal(ra, rb) and np.array_equal(ta, tb)
    assert np.array_equal(ea.solver_iters().cpu().numpy(), eb.solver_iters().cpu().numpy())


def test_solo_rollout_equals_steps(torch_gpu, cmodel, oracle_mod):
    """zb_rollout under the solo layout = T x zb_step under the paired one."""
    torch = torch_gpu
    from zbot_amd.engine import HipEngine, LAYOUT_PAIRS, LAYOUT_SOLO

    cfg = default_config(push=True)
    n, T = 48, 5
    A = torch.from_numpy(np.stack([oracle_mod.synthetic_actions(cmodel.cmodel, 9, n, 0, t) for t in range(T)])).cuda()
    a = HipEngine(cmodel, cfg, n, seed=9)
    b = HipEngine(cmodel, cfg, n, seed=9)
    a.set_step_layout(LAYOUT_PAIRS)
    b.set_step_layout(LAYOUT_SOLO)
    a.reset()
    b.reset()
    for t in range(T):
        a.step(A[t])
    b.rollout(A)
    torch.cuda.synchronize()
    assert np.array_equal(a.get_state().cpu().numpy(), b.get_state().cpu().numpy())
    assert np.array_equal(a.obs_actor.cpu().numpy(), b.obs_actor.cpu().numpy())


def test_solo_general_colliders(torch_gpu, oracle_mod):
    """The general-collider kernels (second contact bank in global scratch, shared by a solo ghost
    with its env) under both layouts, from touching states."""
    torch = torch_gpu
    from zbot_amd.engine import HipEngine, LAYOUT_PAIRS, LAYOUT_SOLO

    cm = compile_model(U.limbs_desc())
    cfg = default_config(randomize=True)
    n = 40
    st0 = oracle_mod.OracleEnv(cm.cmodel, cfg, n, seed=5)
    st0.reset()
    st0.state[:, :27] = U.touching_states(cm, n, 5).astype(np.float32)
    st0.state[:, 32:58] = 0.0
    st0.state[:, cs.S_QACCW:cs.S_QACCW + 32] = 0.0
    res = []
    for layout in (LAYOUT_PAIRS, LAYOUT_SOLO):
        eng = HipEngine(cm, cfg, n, seed=5)
        eng.set_step_layout(layout)
        eng.reset()
        eng.set_state(torch.from_numpy(st0.state.copy()))
        for t in range(3):
            o = eng.step(torch.from_numpy(oracle_mod.synthetic_actions(cm.cmodel, 5, n, 0, t)).cuda())
        torch.cuda.synchronize()
        res.append((eng.get_state().cpu().numpy(), o["obs_critic"].cpu().numpy().copy()))
    assert np.array_equal(res[0][0], res[1][0]) and np.array_equal(res[0][1], res[1][1])


def test_auto_layout(torch_gpu, cmodel):
    """LAYOUT_AUTO: solo up to one wave per SIMD (n <= 4 x CUs), pairs above; ZB_STEP_LAYOUT is not
    set in the test environment."""
    torch = torch_gpu
    from zbot_amd.engine import HipEngine, LAYOUT_PAIRS, LAYOUT_SOLO, ZbError

    simds = 4 * torch.cuda.get_device_properties(0).multi_processor_count
    cfg = default_config()
    assert HipEngine(cmodel, cfg, 512).step_layout == LAYOUT_SOLO  # train.py's num_envs
    assert HipEngine(cmodel, cfg, simds).step_layout == LAYOUT_SOLO
    assert HipEngine(cmodel, cfg, simds + 1).step_layout == LAYOUT_PAIRS
    assert HipEngine(cmodel, cfg, 8192).step_layout == LAYOUT_PAIRS
    e = HipEngine(cmodel, cfg, 8192)
    e.set_step_layout(LAYOUT_SOLO)
    assert e.step_layout == LAYOUT_SOLO
    with pytest.raises(ZbError):
        e.set_step_layout(7)
