"""EnvGroups: N envs as G handles on G HIP streams give bit-identical results to one
handle over all N envs — every output of every step, the engine state, the open-loop rollout, and
PolicyRollout's actor-in-the-loop trajectories — with pushes, per-env randomization and automatic
resets on, at env counts that leave odd groups and ghost teams.
"""

import numpy as np
import pytest

from zbot_amd import default_config

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch_gpu():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch


def _actions(torch, cm, T, n, seed):
    g = torch.Generator(device="cuda").manual_seed(seed)
    bias = torch.tensor([cm.cmodel.joint_bias[a] for a in range(20)], device="cuda")
    return bias + 0.3 * torch.randn(T, n, 20, device="cuda", generator=g)


def _bits(t):
    return t.contiguous().view(-1).cpu().numpy().view(np.uint8)


@pytest.mark.parametrize("n,G", [(517, 2), (300, 3), (64, 4)])
def test_grouped_steps_bit_identical(torch_gpu, cmodel, n, G):
    torch = torch_gpu
    from zbot_amd.engine import EnvGroups, HipEngine

    cfg = default_config(solver="newton", push=True, randomize=True, max_episode_sec=0.3)
    one = HipEngine(cmodel, cfg, n, seed=7)
    grp = EnvGroups(cmodel, cfg, n, groups=G, seed=7)
    assert [b - a for a, b in grp.bounds] and grp.bounds[-1][1] == n
    one.reset()
    grp.reset()
    torch.cuda.synchronize()
    np.testing.assert_array_equal(_bits(grp.get_rand()), _bits(one.get_rand()))
    acts = _actions(torch, cmodel, 24, n, 3)
    ends = 0
    for t in range(24):
        o1 = one.step(acts[t])
        o2 = grp.step(acts[t])
        grp.join()
        torch.cuda.synchronize()
        for k in ("obs_actor", "obs_critic", "obs_extra", "reward_terms", "reward", "done", "success"):
            np.testing.assert_array_equal(_bits(o2[k]), _bits(o1[k]), err_msg=f"{k} at step {t}")
        ends += int(o1["done"].sum())
    np.testing.assert_array_equal(_bits(grp.get_state()), _bits(one.get_state()))
    np.testing.assert_array_equal(grp.solver_iters().cpu().numpy(), one.solver_iters().cpu().numpy())
    np.testing.assert_array_equal(_bits(grp.get_stats()), _bits(one.get_stats()))
    assert ends > 0  # automatic resets were exercised


def test_grouped_rollout_and_state_io(torch_gpu, cmodel):
    torch = torch_gpu
    from zbot_amd.engine import EnvGroups, HipEngine

    cfg = default_config(solver="newton", push=True)
    n = 130
    one = HipEngine(cmodel, cfg, n, seed=4)
    grp = EnvGroups(cmodel, cfg, n, groups=2, seed=4)
    one.reset()
    grp.reset()
    acts = _actions(torch, cmodel, 6, n, 5)
    r1 = torch.empty(n, device="cuda")
    r2 = torch.empty(n, device="cuda")
    o1 = one.rollout(acts, reward_sum=r1)
    o2 = grp.rollout(acts, reward_sum=r2)
    grp.join()
    torch.cuda.synchronize()
    np.testing.assert_array_equal(_bits(r2), _bits(r1))
    np.testing.assert_array_equal(_bits(o2["obs_actor"]), _bits(o1["obs_actor"]))
    np.testing.assert_array_equal(_bits(grp.get_state()), _bits(one.get_state()))
    # set_state through the groups, then one more step each
    st = one.get_state()
    st[:, 2] += 0.01
    one.set_state(st)
    grp.set_state(st)
    o1 = one.step(acts[0])
    o2 = grp.step(acts[0])
    grp.join()
    torch.cuda.synchronize()
    np.testing.assert_array_equal(_bits(o2["obs_critic"]), _bits(o1["obs_critic"]))


def test_grouped_policy_rollout_bit_identical(torch_gpu, cmodel):
    torch = torch_gpu
    from zbot_amd import policy as P
    from zbot_amd.engine import EnvGroups, HipEngine

    cfg = default_config(solver="newton", max_episode_sec=0.2)
    n, T = 200, 14
    actor = P.GruPolicy(P.ACTOR, P.init_params(P.ACTOR, seed=0))
    outs = []
    for eng in (HipEngine(cmodel, cfg, n, seed=9), EnvGroups(cmodel, cfg, n, groups=2, seed=9)):
        ro = P.PolicyRollout(eng, actor, seed=2)
        ro.reset()
        a = ro.run(T, record_critic=True)
        b = ro.run(3, record_critic=True)  # continues across run() calls: carry, done, step counter
        torch.cuda.synchronize()
        outs.append((a, b, ro.carry.clone()))
    (a1, b1, c1), (a2, b2, c2) = outs
    for k in a1:
        np.testing.assert_array_equal(_bits(a2[k]), _bits(a1[k]), err_msg=k)
        np.testing.assert_array_equal(_bits(b2[k]), _bits(b1[k]), err_msg=k)
    np.testing.assert_array_equal(_bits(c2), _bits(c1))
    assert int(a1["done"].sum()) > 0


@pytest.mark.parametrize("G", [1, 3])
def test_in_loop_critic_matches_post_hoc(torch_gpu, cmodel, G):
    """PolicyRollout's in-loop critic (V(s_t) after each step launch, per group, one-wave layout)
    equals the critic run over the recorded observations afterwards (8-wave layout)."""
    torch = torch_gpu
    from zbot_amd import policy as P
    from zbot_amd.engine import EnvGroups, HipEngine

    cfg = default_config(solver="newton", max_episode_sec=0.2)
    n, T = 150, 12
    actor = P.GruPolicy(P.ACTOR, P.init_params(P.ACTOR, seed=0), layout=P.LAYOUT_WAVE)
    crit_in = P.GruPolicy(P.CRITIC, P.init_params(P.CRITIC, seed=1), layout=P.LAYOUT_WAVE)
    crit_ph = P.GruPolicy(P.CRITIC, P.init_params(P.CRITIC, seed=1), layout=P.LAYOUT_BLOCK)
    eng = HipEngine(cmodel, cfg, n, seed=3) if G == 1 else EnvGroups(cmodel, cfg, n, groups=G, seed=3, priority=-1)
    ro = P.PolicyRollout(eng, actor, seed=2)
    ro.reset()
    ro.run(2, record_critic=True)
    cc = crit_in.initial_carry(n)
    traj = ro.run(T, record_critic=True, critic=crit_in, critic_carry=cc)
    cp = crit_ph.initial_carry(n)
    zeros = torch.zeros(1, n, dtype=torch.uint8, device="cuda")
    v = crit_ph.critic(traj["obs_critic"], cp, reset=torch.cat([zeros, traj["done"][:-1]]))
    b = crit_ph.critic(traj["obs_critic_next"], cp, reset=traj["done"][-1])
    torch.cuda.synchronize()
    np.testing.assert_array_equal(_bits(traj["value"]), _bits(v))
    np.testing.assert_array_equal(_bits(traj["value_next"]), _bits(b))
    np.testing.assert_array_equal(_bits(cc), _bits(cp))
    assert int(traj["done"].sum()) > 0


def test_set_step_chunks_same_bits(torch_gpu, cmodel):
    torch = torch_gpu
    from zbot_amd.engine import HipEngine, ZbError

    cfg = default_config(solver="newton", push=True, max_episode_sec=0.3)
    n = 90
    acts = _actions(torch, cmodel, 8, n, 11)
    states = []
    for k in (1, 3, 0):
        e = HipEngine(cmodel, cfg, n, seed=12)
        e.set_step_chunks(k)
        e.reset()
        for t in range(8):
            e.step(acts[t])
        states.append(e.get_state())
    torch.cuda.synchronize()
    for st in states[1:]:
        np.testing.assert_array_equal(_bits(st), _bits(states[0]))
    with pytest.raises(ZbError):
        e.set_step_chunks(-1)


def test_converted_actions_outlive_step_without_join(torch_gpu, cmodel):
    """A float64 action converted inside EnvGroups.step is read on the group streams after step()
    returns; allocations right after step() (no join) must not reuse its block before the groups
    are done with it (record_stream). Same bits as float32 actions on one handle."""
    torch = torch_gpu
    from zbot_amd.engine import EnvGroups, HipEngine

    n = 256
    cfg = default_config(solver="newton", push=True)
    one = HipEngine(cmodel, cfg, n, seed=5)
    grp = EnvGroups(cmodel, cfg, n, groups=2, seed=5)
    one.reset()
    grp.reset()
    acts = _actions(torch, cmodel, 6, n, 9)
    junk = []
    for t in range(6):
        one.step(acts[t])
        grp.step(acts[t].double())  # converted copy, dropped when step() returns
        # same-size allocations on the caller's stream, written at once
        junk.append(torch.full((n, 20), float("nan"), dtype=torch.float32, device="cuda"))
        junk.append(torch.full((n, 20), float("nan"), dtype=torch.float64, device="cuda"))
    grp.join()
    torch.cuda.synchronize()
    np.testing.assert_array_equal(_bits(grp.get_state()), _bits(one.get_state()))


def test_airtime_patch_orders_after_caller_writes(torch_gpu, cmodel):
    """the row-0 FeetAirtime patch runs on the group streams; a trajectory buffer the
    caller fills on its own stream after the last step() (here: stacked behind a long sleep kernel)
    must be written before the patch adds to it. One handle on one stream is the reference."""
    torch = torch_gpu
    from zbot_amd.engine import EnvGroups, HipEngine

    n, T = 300, 12
    cfg = default_config(solver="newton", push=True)
    acts = _actions(torch, cmodel, T, n, 5)
    out = {}
    for name, eng in (("one", HipEngine(cmodel, cfg, n, seed=11)), ("grp", EnvGroups(cmodel, cfg, n, groups=3, seed=11))):
        eng.reset()
        for t in range(10):  # the feet are down at the rollout's first step (its contact bits are set)
            eng.step(acts[t])
        eng.mark_rollout_start()
        rows = []
        for t in range(T):
            o = eng.step(acts[t])
            eng.join()
            rows.append(o["reward"].clone())
        torch.cuda._sleep(50_000_000)  # the caller's stream is busy: the stack below lands late
        traj = torch.stack(rows)
        eng.feet_airtime_exact(traj[0], None)
        eng.join()
        torch.cuda.synchronize()
        out[name] = traj.cpu().numpy()
        out[name + "_causal0"] = rows[0].cpu().numpy()
    np.testing.assert_array_equal(out["grp"].view(np.uint32), out["one"].view(np.uint32))
    # the patch changed row 0 for the envs whose feet touched down over the rollout
    assert not np.array_equal(out["one"][0], out["one_causal0"])
