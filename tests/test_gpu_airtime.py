"""ksim's FeetAirtimeReward over whole rollouts on the GPU (train.py:503-546).

The fused step computes the causal per-step form; zb_mark_rollout_start + zb_feet_airtime_exact
(include/zbot.h) patch row 0 to ksim's trajectory semantics (prev contact False at t = 0, airtime
roll -> air[T-1]). Checked against the oracle's numpy restatement of get_reward_stateful on the
contact / done sequence the engine itself produced.
"""

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

TERM = 6  # ZB_T_FEET_AIRTIME


def _rollout(eng, cs, T, seed, push_noise=0.2, mark=True):
    from zbot_amd.constants import JOINT_BIASES

    n = eng.n
    g = torch.Generator(device="cuda")
    g.manual_seed(seed)
    bias = torch.tensor([b for _, b, _ in JOINT_BIASES], device="cuda")
    terms = torch.empty(T, n, cs.NUM_TERMS, device="cuda")
    rew = torch.empty(T, n, device="cuda")
    done = torch.empty(T, n, dtype=torch.uint8, device="cuda")
    cont = torch.empty(T, n, 2, dtype=torch.bool, device="cuda")
    carry0 = eng.get_state()[:, cs.S_AIRTIME:cs.S_AIRTIME + 2].clone()
    if mark:
        eng.mark_rollout_start()
    for t in range(T):
        a = bias + push_noise * torch.randn(n, cs.NJ, device="cuda", generator=g)
        out = eng.step(a, extras=False)
        terms[t].copy_(out["reward_terms"])
        rew[t].copy_(out["reward"])
        done[t].copy_(out["done"])
        # the contact flags the step's reward used (touch > 0.1), kept in the state row
        cont[t].copy_(eng.get_state()[:, cs.S_PREV_CONT:cs.S_PREV_CONT + 2] > 0.5)
    return terms, rew, done, cont, carry0


def test_feet_airtime_exact_rollout_matches_ksim(oracle_mod):
    """200-step rollout of 256 envs with pushes and sigma = 0.2 action noise (touchdowns and
    resets inside): after the patch, the FeetAirtime column of every row equals the oracle's
    get_reward_stateful restatement bit for bit; rows t >= 1 and the 11 other terms are unchanged
    (the causal form is ksim's there); reward[0] moves by exactly scale * (ksim - causal) (fp32,
    one fused multiply-add: atol 1e-6)."""
    from zbot_amd import compile_model, default_config
    from zbot_amd import cstructs as cs
    from zbot_amd.engine import HipEngine

    cfg = default_config(solver="newton", push=True)
    eng = HipEngine(compile_model(), cfg, 256, seed=11)
    eng.reset()
    _rollout(eng, cs, 5, seed=1, mark=False)  # airtime carries and contact history from a first rollout
    T = 200
    eng.get_stats(clear=True)
    terms, rew, done, cont, carry0 = _rollout(eng, cs, T, seed=2)
    before_t, before_r = terms.clone(), rew.clone()
    eng.feet_airtime_exact(rew[0], terms[0], curriculum=1.0)
    # the statistics' reward sum follows the patched row 0 (fp32 running sums: rtol 1e-5)
    np.testing.assert_allclose(eng.get_stats()[:, cs.ST_REWARD].double().cpu().numpy(),
                               rew.double().sum(0).cpu().numpy(), rtol=1e-5, atol=1e-4)
    final_air = eng.get_state()[:, cs.S_AIRTIME:cs.S_AIRTIME + 2]
    torch.cuda.synchronize()
    ref, carry = oracle_mod.feet_airtime_traj(cont.cpu().numpy(), done.cpu().numpy().astype(bool),
                                              carry0.cpu().numpy(), cfg.ctrl_dt, cfg.feet_airtime_touchdown_penalty)
    got = terms[:, :, TERM].cpu().numpy()
    print(f"max |ksim - engine| FeetAirtime over [{T}, 256]: {np.abs(got - ref).max():.3e}; "
          f"touchdowns {int((got != 0).sum())}, episode ends {int(done.sum())}, "
          f"row-0 changes {int((before_t[0, :, TERM] != terms[0, :, TERM]).sum())}")
    np.testing.assert_array_equal(got, ref)
    np.testing.assert_array_equal(final_air.cpu().numpy(), carry)
    # the rollout exercises what it claims to: touchdowns after t = 0, resets, a changed row 0
    assert (got[1:] != 0).sum() > 20 and int(done.sum()) > 5
    assert int((before_t[0, :, TERM] != terms[0, :, TERM]).sum()) > 100
    assert torch.equal(terms[1:], before_t[1:]) and torch.equal(rew[1:], before_r[1:])
    other = [i for i in range(cs.NUM_TERMS) if i != TERM]
    assert torch.equal(terms[0][:, other], before_t[0][:, other])
    scale = cfg.reward_scale[TERM]
    exp0 = before_r[0].cpu().numpy() + scale * (ref[0] - before_t[0, :, TERM].cpu().numpy())
    np.testing.assert_allclose(rew[0].cpu().numpy(), exp0, rtol=0, atol=1e-6)


def test_feet_airtime_exact_needs_a_marked_step():
    from zbot_amd import compile_model, default_config
    from zbot_amd.engine import HipEngine, ZbError

    eng = HipEngine(compile_model(), default_config(solver="newton"), 8, seed=1)
    eng.reset()
    r = torch.zeros(8, device="cuda")
    with pytest.raises(ZbError):
        eng.feet_airtime_exact(r)
    eng.mark_rollout_start()
    with pytest.raises(ZbError):  # marked, but no step ran yet
        eng.feet_airtime_exact(r)
    eng.step(torch.zeros(8, 20, device="cuda"))
    eng.feet_airtime_exact(r)
    with pytest.raises(ZbError):  # patched once already
        eng.feet_airtime_exact(r)


def test_policy_rollout_rows_are_ksim_feet_airtime(oracle_mod):
    """PolicyRollout patches every run() (one ksim trajectory) by default: its reward rows equal
    the same rollout with exact_airtime=False except row 0, which moves by scale * (ksim - causal)
    with ksim's row 0 from the restatement (the run's contacts from the recorded obs would need
    extras; here the causal rows come from a second, unpatched run of the same seeds)."""
    from zbot_amd import compile_model, default_config
    from zbot_amd import cstructs as cs
    from zbot_amd import policy as P
    from zbot_amd.engine import HipEngine

    cm = compile_model()
    outs = []
    for exact in (True, False):
        eng = HipEngine(cm, default_config(solver="newton"), 64, seed=3)
        ro = P.PolicyRollout(eng, P.GruPolicy(P.ACTOR, P.init_params(P.ACTOR, seed=4)), seed=6, exact_airtime=exact)
        ro.reset()
        ro.run(12)  # from the reset pose the feet touch down during the first steps: warm up first
        air0 = eng.get_state()[:, cs.S_AIRTIME:cs.S_AIRTIME + 2].clone()
        out = ro.run(12)
        st = eng.get_state()
        torch.cuda.synchronize()
        outs.append((out["reward"].cpu().numpy(), st.cpu().numpy(), air0.cpu().numpy()))
    (r_ex, st_ex, _), (r_c, st_c, _) = outs
    np.testing.assert_array_equal(r_ex[1:], r_c[1:])
    np.testing.assert_array_equal(st_ex[:, :cs.S_AIR0_CONT], st_c[:, :cs.S_AIR0_CONT])
    bits = np.ascontiguousarray(st_ex[:, cs.S_AIR0_CONT]).view(np.uint32)
    air = st_ex[:, cs.S_AIRTIME:cs.S_AIRTIME + 2]
    f = np.float32
    k0 = ((air[:, 0] - f(0.3)) * (bits & 1).astype(f)).astype(f)
    k0 = (f(0) + k0 + ((air[:, 1] - f(0.3)) * ((bits >> 1) & 1).astype(f))).astype(f)
    causal0 = st_ex[:, cs.S_AIR0_TERM]
    np.testing.assert_allclose(r_ex[0], r_c[0] + f(2.5) * (k0 - causal0), rtol=0, atol=1e-6)
    assert (bits != 0).any()
