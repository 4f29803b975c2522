"""Floor colliders beyond the two box soles on the GPU (the general-collider kernels, XG): a right
shin box and a left hand capsule beside the soles ("limbs"), capsule feet with a head sphere
("round"), and a cylinder right foot, a cylinder shin and an ellipsoid hand beside the left box sole
("cyl", round 4), in states where the colliders touch the floor (tests/collider_util.py), against the
oracle on the same model and state."""

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


DESCS = {"limbs": U.limbs_desc, "round": U.round_desc, "cyl": U.cyl_desc, "mesh": U.mesh_desc, "mjxbox": U.mjx_box_desc}


@pytest.fixture(scope="module", params=list(DESCS))
def variant(request):
    return request.param, compile_model(DESCS[request.param]())


def contact_env(O, cm, cfg, n, seed):
    """An oracle env whose qpos are touching_states (at rest, no warm start)."""
    env = O.OracleEnv(cm.cmodel, cfg, n, seed=seed)
    env.reset()
    env.state[:, :27] = U.touching_states(cm, n, seed).astype(np.float32)
    env.state[:, 32:58] = 0.0
    env.state[:, cs.S_QACCW:cs.S_QACCW + 32] = 0.0
    return env


def test_debug_forward_matches_oracle(torch_gpu, variant, oracle_mod):
    """One forward pass: contact and constraint counts exact, constrained acceleration and touch
    within the stage test's bounds (test_forward_stages_match_oracle)."""
    torch = torch_gpu
    from zbot_amd.engine import DBG, HipEngine

    name, cm = variant
    cfg = default_config(solver="newton")
    n = 64
    env = contact_env(oracle_mod, cm, cfg, n, seed=5)
    st = env.state.copy()
    ctrl = (np.random.default_rng(2).normal(size=(n, 20)) * 0.5).astype(np.float32)
    eng = HipEngine(cm, cfg, n)
    g = eng.debug_forward(torch.from_numpy(st), torch.from_numpy(ctrl)).cpu().numpy()
    worst = 0.0
    for e in range(n):
        ref = oracle_mod.forward_debug(cm.cmodel, cfg, st[e, :27], st[e, 32:58], ctrl[e], precision="f64")
        assert int(g[e, DBG["misc"] + 1]) == ref["ncon"], (name, e)
        assert int(g[e, DBG["misc"]]) == ref["nefc"], (name, e)
        qa = g[e, DBG["qacc"]:DBG["qacc"] + 26]
        err = np.abs(qa - ref["qacc"]).max() / max(1.0, np.abs(ref["qacc"]).max())
        worst = max(worst, err)
        assert err <= 1e-3, (name, e, err)
        np.testing.assert_allclose(g[e, DBG["misc"] + 2:DBG["misc"] + 4], ref["touch"], rtol=1e-3, atol=1e-3)
    print(f"\n[{name} debug forward] max relative qacc error {worst:.2e}")


# One env-step from a touching state at rest (the contacts' first impulses), fp32 engine vs fp32
# oracle, about 5x the max error measured on MI355X (round 3, profiles/r03_v12_gpu_colliders.log:
# Newton qpos 3.0e-7, qvel 3.6e-5, planner 2.2e-5, obs_critic 1.4e-4, obs_extra 4.2e-3, reward
# 1.6e-6, terms 9.0e-7).
COLLIDER_TOL = {
    "qpos": (2e-6, 0.0),
    "qvel": (2e-4, 0.0),
    "planner": (1e-4, 0.0),
    "obs_actor": (2e-4, 0.0),
    "obs_critic": (1e-3, 0.0),
    "obs_extra": (2e-2, 0.0),
    "reward": (1e-5, 0.0),
    "reward_terms": (5e-6, 0.0),
}
# CG: the CG contract of tests/test_gpu_parity.py (round 6) on these bounds: COLLIDER_TOL plus CG_SLACK x each
# env's sensitivity (oracle_sensitivity), CG_BUDGET envs per output and step within CG_LOOSE x beyond
# it, a budget env with a contact at its activation boundary exempt from the loose limit.


# The cyl variant's cylinder right foot lands flat in the first step (three rim contacts, ncon 3):
# a disk resting on the floor, where MuJoCo's plane-cylinder rule turns the contact triangle with
# the direction of a vanishing tilt. The fp32 and fp64 oracles then disagree by up to 1.7e-5 in
# qpos over the second step in 56 of 64 envs (the limbs variant: 2.4e-7 in none;
# scripts/cyl_flat_probe.py, profiles/r04_cyl_flat_probe.log), so the fp64 slack (MaxErr ref64)
# would cover nearly every env. There the GPU is held to the fp32 oracle without it: every env
# within the same bounds (r04 v17 measured qpos 3.0e-7, qvel 5.3e-6 with Newton; qpos 3.1e-6,
# qvel 2.3e-4 with CG).
NO_FP64_SLACK = {"cyl"}
# The box soles collided by MJX's plane_convex manifold (compile_model(box_rule="mjx")) stand exactly
# flat at reset, where the rule's first-maximum tie-breaks between corners at equal distances decide
# which corners carry the robot: the fp32 and fp64 oracles part in 60-64 of 64 envs over the first
# steps of the rollout below and agree again once the robots have left the flat pose (about 1 env
# from the eleventh step; profiles/r05_mjxbox_oracle_gap.txt). Any fp32 implementation, MJX's
# included, picks its corners from its own rounding there, so that rollout is held to the ensemble
# contract alone; the one-step tests from touching states (no flat face) keep the full contract.
ENSEMBLE_ONLY = {"mjxbox"}


@pytest.mark.parametrize("eulerdamp", [False, True], ids=["explicit", "eulerdamp"])
@pytest.mark.parametrize("solver", ["newton", "cg"])
def test_one_step_matches_oracle(torch_gpu, variant, oracle_mod, solver, eulerdamp):
    """eulerdamp: mj_Euler's implicit damping (the ED instantiations of the general-collider kernels)
    under the same contract as the explicit form, as tests/test_gpu_parity.py holds the two-sole model."""
    torch = torch_gpu
    from test_gpu_parity import (CG_BUDGET, CG_LOOSE, CG_SLACK, MaxErr, boundary_envs, one_step_outputs, oracle_sensitivity,
                                 oracle_steps)

    from zbot_amd.engine import HipEngine

    name, cm = variant
    cfg = default_config(solver=solver, eulerdamp=eulerdamp)
    n = 64
    cg = solver == "cg"
    env = contact_env(oracle_mod, cm, cfg, n, seed=11)
    eng = HipEngine(cm, cfg, n, seed=11)
    kw = dict(budget=CG_BUDGET, loose=CG_LOOSE, max_ill=n, k_slack=CG_SLACK) if cg else {}
    err = MaxErr(f"colliders {name} {solver}{' eulerdamp' if eulerdamp else ''} one-step", exempt_ill=name in ENSEMBLE_ONLY, **kw)
    # the second step starts from the oracle's first, where the lying robots (56 of 64) have been
    # reset onto flat soles: for ENSEMBLE_ONLY variants that is the flat-face tie of their rollouts
    for t in range(1 if name in ENSEMBLE_ONLY else 2):
        st0, rd0 = env.state.copy(), env.rand.copy()
        eng.set_state(torch.from_numpy(st0.copy()))
        eng.set_rand(torch.from_numpy(rd0.copy()))
        a = oracle_mod.synthetic_actions(cm.cmodel, 11, n, 0, t)
        ref, ref64 = oracle_steps(oracle_mod, cm, cfg, env, a, 11)
        ref32 = {k: want for k, _, want in one_step_outputs(env.state, ref, env.state, ref)}
        sens = oracle_sensitivity(oracle_mod, cm, cfg, st0, rd0, a, 11, ref32) if cg else {}
        bnd = boundary_envs(ref64)
        out = eng.step(torch.from_numpy(a).cuda())
        torch.cuda.synchronize()
        gs = eng.get_state().cpu().numpy()
        np.testing.assert_array_equal(out["done"].cpu().numpy(), ref["done"])
        for key, got, want in one_step_outputs(gs, out, env.state, ref):
            # NO_FP64_SLACK: no fp32/fp64 gap (the flat disk's gap covers nearly every env); CG keeps the
            # perturbation sensitivity
            r64 = (want if cg else None) if name in NO_FP64_SLACK else ref64[key]
            err.add(key, got, want, *COLLIDER_TOL[key], ref64=r64, sens=sens.get(key), exempt=bnd)
    err.report()


def test_rollout_launch_equals_steps(torch_gpu, variant, oracle_mod):
    """zb_rollout over T steps is bit-identical to T zb_step launches with the general colliders
    (auto-resets included)."""
    torch = torch_gpu
    from zbot_amd.engine import HipEngine

    _, cm = variant
    cfg = default_config(solver="newton", push=True)
    n, T = 32, 6
    A = torch.from_numpy(np.stack([oracle_mod.synthetic_actions(cm.cmodel, 4, n, 0, t, std=0.5)
                                   for t in range(T)])).cuda()
    env = contact_env(oracle_mod, cm, cfg, n, seed=4)
    a = HipEngine(cm, cfg, n, seed=4)
    b = HipEngine(cm, cfg, n, seed=4)
    for h in (a, b):
        h.set_state(torch.from_numpy(env.state.copy()))
        h.set_rand(torch.from_numpy(env.rand.copy()))
    for t in range(T):
        a.step(A[t])
    b.rollout(A, reward_sum=torch.zeros(n, device="cuda"))
    torch.cuda.synchronize()
    assert np.array_equal(a.get_state().cpu().numpy(), b.get_state().cpu().numpy())


@pytest.mark.parametrize("name", list(DESCS))
def test_rollout_from_reset_matches_oracle(torch_gpu, oracle_mod, name):
    """48 control steps of 64 envs from reset with pushes and wide actions (std 0.5), so robots
    stumble, fall and reset: the general-collider instantiations (levels 1 and 2) over a rollout,
    against the fp32 oracle run alongside. As the golden rollouts (test_gpu_parity.
    test_golden_rollout): the first 8 rewards (cyl: 4) under the one-step contract (the fp64 oracle stepping
    from the fp32 oracle's state gives the slack at a discontinuity; none for the cyl variant,
    NO_FP64_SLACK), done flags exact over the first 16 steps, then the ensemble contract
    (golden_ensemble_check). Prints how often each collider touched the floor in the oracle's
    rollout (every 4th env): the soles (and the cylinder foot) carry the robots; shins, hands and
    head rarely touch before NotUpright ends the episode, so the one-step tests from touching states
    above are the ones that load every collider."""
    torch = torch_gpu
    from test_gpu_parity import GOLDEN_EXACT_STEPS, GOLDEN_TOL, MaxErr, golden_ensemble_check

    from zbot_amd.engine import HipEngine

    cm = compile_model(DESCS[name]())
    cfg = default_config(solver="newton", push=True)
    n, steps, seed = 64, 48, 13
    acts = np.stack([oracle_mod.synthetic_actions(cm.cmodel, seed, n, 0, t, std=0.5) for t in range(steps)])
    e32 = oracle_mod.OracleEnv(cm.cmodel, cfg, n, seed=seed)
    e64 = oracle_mod.OracleEnv(cm.cmodel, cfg, n, seed=seed, precision="f64")
    e32.reset()
    ref_r, ref_d, r64s = [], [], []
    extra = np.zeros(cm.cmodel.ngeom, int)
    for t in range(steps):
        if t < 8:
            e64.state[:] = e32.state
            e64.rand[:] = e32.rand
            r64s.append(e64.step(acts[t])["reward"].copy())
        o = e32.step(acts[t])
        ref_r.append(o["reward"].copy())
        ref_d.append(o["done"].copy())
        for e in range(0, n, 4):
            cons = U.contacts(cm, e32.state[e, :27].astype(np.float64))
            extra += np.array([len(c) > 0 for c in cons])
    names = [gd["name"] for gd in cm.desc["geoms"]]  # U.contacts order (the descriptor's)
    g = {"reward": np.stack(ref_r), "done": np.stack(ref_d), "final_state": e32.state.copy()}
    eng = HipEngine(cm, cfg, n, seed=seed)
    eng.reset()
    rew, done = [], []
    for t in range(steps):
        o = eng.step(torch.from_numpy(acts[t]).cuda())
        rew.append(o["reward"].cpu().numpy().copy())
        done.append(o["done"].cpu().numpy().copy())
    rew, done = np.stack(rew), np.stack(done)
    if name in ENSEMBLE_ONLY:
        print(f"\n[colliders {name} rollout] steps with a contact per collider (every 4th env): "
              + ", ".join(f"{names[k]} {int(extra[k])}" for k in range(len(names))))
        golden_ensemble_check(f"colliders {name}", rew, done, eng.get_state().cpu().numpy(), g)
        return
    np.testing.assert_array_equal(done[:GOLDEN_EXACT_STEPS], g["done"][:GOLDEN_EXACT_STEPS])
    err = MaxErr(f"colliders {name} rollout from reset")
    # the cyl variant's cylinder foot stands exactly upright at reset, the flat-disk discontinuity of
    # NO_FP64_SLACK: each fp32 implementation picks its contact triangle from its own rounding, and
    # on MI355X a few envs part from the fp32 oracle from the fifth step (r04 v21: rewards within
    # 2.4e-6 over steps 0-3, then 1-4 of 64 envs beyond the bound), so its window is 4 steps
    # the mesh variant: MJX's manifold rule reselects all four points when a vertex enters or leaves
    # the penetrating set, so one rounding-level difference at such a crossing moves the whole contact
    # set; on MI355X (r05) rewards held 7.5e-7 over steps 0-3, then 1-2 of 64 envs left the bound per
    # step (the fp32 / fp64 oracles themselves part at 1 env of 64 in 8 steps), so its window is 4 steps
    for t in range(4 if name in NO_FP64_SLACK or name == "mesh" else 8):
        err.add(f"reward[{t}]", rew[t], g["reward"][t], GOLDEN_TOL["reward"],
                ref64=None if name in NO_FP64_SLACK else r64s[t])
    print(f"\n[colliders {name} rollout] steps with a contact per collider (every 4th env): "
          + ", ".join(f"{names[k]} {int(extra[k])}" for k in range(len(names))))
    golden_ensemble_check(f"colliders {name}", rew, done, eng.get_state().cpu().numpy(), g)
    err.report()


@pytest.mark.parametrize("name", list(DESCS))
def test_full_size_properties(torch_gpu, name):
    """Each collider variant at the C2 size (8192 envs, pushes and randomization on, 8 steps from
    reset, two env groups): finite, unit quaternions, no invalid flag, bit-reproducible, and
    shard-invariant (two half-size handles with env_offset give the same bits as one handle, and the
    two-group EnvGroups the same bits again)."""
    torch = torch_gpu
    from zbot_amd.engine import EnvGroups, HipEngine

    cm = compile_model(DESCS[name]())
    cfg = default_config(solver="newton", push=True, randomize=True)
    n = 8192
    g = torch.Generator(device="cuda")
    g.manual_seed(5)
    bias = torch.tensor([cm.cmodel.joint_bias[i] for i in range(20)], device="cuda")
    acts = [bias + 0.2 * torch.randn(n, 20, device="cuda", generator=g) for _ in range(8)]

    def run(h, lo=0, hi=n):
        h.reset()
        for a in acts:
            out = h.step(a[lo:hi].contiguous())
        return h.get_state(), out

    st, out = run(HipEngine(cm, cfg, n, seed=9))
    assert torch.isfinite(st[:, :58]).all() and torch.isfinite(out["obs_critic"]).all()
    assert torch.allclose(st[:, 3:7].norm(dim=1), torch.ones(n, device="cuda"), atol=2e-6)
    assert (st[:, cs.S_NAN].view(torch.int32) == 0).all()
    again, _ = run(HipEngine(cm, cfg, n, seed=9))
    assert torch.equal(again, st)
    halves = [run(HipEngine(cm, cfg, n // 2, env_offset=off, seed=9), off, off + n // 2)[0] for off in (0, n // 2)]
    assert torch.equal(torch.cat(halves), st)
    grouped = EnvGroups(cm, cfg, n, groups=2, seed=9)
    gst, _ = run(grouped)
    grouped.join()
    assert torch.equal(gst, st)


# ---- nine floor colliders (model v9): the second and third banks' per-substep selection ----

# the floor colliders beyond the soles the engine collides per substep: XG 5 (round 6) holds the first
# four within reach in its second and third banks (XG 1 / 2 before: two)
BANK_CAP = 4


def test_many_colliders_match_oracle_within_the_cap(torch_gpu, oracle_mod):
    """Nine floor colliders (collider_util.many_desc): the engine collides the soles and, per substep,
    the first BANK_CAP of the other seven within reach of the floor (zb_engine.hip select_bank2, the
    XG 5 kernels). From touching states: where the selection finds at most BANK_CAP
    (collider_util.bank2_candidates), one forward pass matches the oracle, which collides all nine
    (contact and constraint counts exact, qacc within 1e-3 relative), for both solvers; one step holds
    the collider one-step contract for every env whose step kept within the cap (no overflow flag,
    ZB_S_NAN bit 1); an env that starts with more carries the flag after the step."""
    torch = torch_gpu
    from test_gpu_parity import CG_BUDGET, CG_LOOSE, CG_SLACK, MaxErr, one_step_outputs, oracle_sensitivity, oracle_steps

    from zbot_amd.engine import DBG, HipEngine

    cm = compile_model(U.many_desc())
    n = 64
    for solver, ed in (("newton", False), ("cg", False), ("newton", True), ("cg", True)):
        cfg = default_config(solver=solver, eulerdamp=ed)
        tag = solver + (" eulerdamp" if ed else "")
        env = contact_env(oracle_mod, cm, cfg, n, seed=5)
        st = env.state.copy()
        cand = np.array([len(U.bank2_candidates(cm, st[e, :27].astype(np.float64))) for e in range(n)])
        ctrl = (np.random.default_rng(2).normal(size=(n, 20)) * 0.5).astype(np.float32)
        eng = HipEngine(cm, cfg, n, seed=5)
        g = eng.debug_forward(torch.from_numpy(st), torch.from_numpy(ctrl)).cpu().numpy()
        checked = 0
        for e in range(n):
            if cand[e] > BANK_CAP:
                continue
            ref = oracle_mod.forward_debug(cm.cmodel, cfg, st[e, :27], st[e, 32:58], ctrl[e], precision="f64")
            assert int(g[e, DBG["misc"] + 1]) == ref["ncon"], (tag, e)
            assert int(g[e, DBG["misc"]]) == ref["nefc"], (tag, e)
            qa = g[e, DBG["qacc"]:DBG["qacc"] + 26]
            tol = 1e-3 if solver == "newton" else 5e-2  # CG: 8 unconverged iterations (test_gpu_sole_pair)
            assert np.abs(qa - ref["qacc"]).max() / max(1.0, np.abs(ref["qacc"]).max()) <= tol, (tag, e)
            checked += 1
        print(f"\n[many colliders {tag}] forward pass: {checked} of {n} envs within {BANK_CAP} candidates beyond "
              f"the soles (candidates per env {np.bincount(cand).tolist()}), {int((cand > 2).sum())} of them "
              "beyond round 5's two")
        assert checked >= n // 2
        assert (cand[cand <= BANK_CAP] > 2).any(), "the touching states exercise the third bank"
        # one step
        eng.set_state(torch.from_numpy(env.state.copy()))
        eng.set_rand(torch.from_numpy(env.rand.copy()))
        a = oracle_mod.synthetic_actions(cm.cmodel, 5, n, 0, 0)
        st0, rd0 = env.state.copy(), env.rand.copy()
        ref, ref64 = oracle_steps(oracle_mod, cm, cfg, env, a, 5)
        out = eng.step(torch.from_numpy(a).cuda())
        torch.cuda.synchronize()
        gs = eng.get_state().cpu().numpy()
        flag = (gs[:, cs.S_NAN].view(np.int32) & 2) != 0
        assert np.array_equal(eng.flags()["bank_overflow"].cpu().numpy(), flag)
        assert flag[cand > BANK_CAP].all(), "an env that starts with more than the cap is flagged"
        # bit 2 is the step's own: set with bit 1 by this step
        assert np.array_equal(eng.flags()["bank_overflow_step"].cpu().numpy(), flag)
        keep = ~flag
        cg = solver == "cg"
        kw = dict(budget=CG_BUDGET, loose=CG_LOOSE, max_ill=n, k_slack=CG_SLACK) if cg else {}
        ref32 = {k: want for k, _, want in one_step_outputs(env.state, ref, env.state, ref)}
        sens = oracle_sensitivity(oracle_mod, cm, cfg, st0, rd0, a, 5, ref32) if cg else {}
        err = MaxErr(f"many colliders {tag} one-step (unflagged envs)", **kw)
        for key, got, want in one_step_outputs(gs, out, env.state, ref):
            sk = sens.get(key)
            err.add(key, got[keep], want[keep], *COLLIDER_TOL[key], ref64=ref64[key][keep],
                    sens=None if sk is None else np.asarray(sk)[keep])
        print(f"[many colliders {tag}] one step: {int(keep.sum())} of {n} envs without the overflow flag")
        err.report()


def test_many_colliders_full_size(torch_gpu):
    """The nine-collider model at the C2 size (8192 envs, pushes and randomization, 8 steps from reset):
    finite, no non-finite flag (bit 0), bit-reproducible, and the same bits from two half-size handles
    and from two env groups; prints how many envs ever overflowed the second bank."""
    torch = torch_gpu
    from zbot_amd.engine import EnvGroups, HipEngine

    cm = compile_model(U.many_desc())
    cfg = default_config(solver="newton", push=True, randomize=True)
    n = 8192
    g = torch.Generator(device="cuda")
    g.manual_seed(5)
    bias = torch.tensor([cm.cmodel.joint_bias[i] for i in range(20)], device="cuda")
    acts = [bias + 0.2 * torch.randn(n, 20, device="cuda", generator=g) for _ in range(8)]

    def run(h, lo=0, hi=n):
        h.reset()
        for a in acts:
            out = h.step(a[lo:hi].contiguous())
        return h.get_state(), out

    st, out = run(HipEngine(cm, cfg, n, seed=9))
    assert torch.isfinite(st[:, :58]).all() and torch.isfinite(out["obs_critic"]).all()
    flags = st[:, cs.S_NAN].view(torch.int32)
    assert ((flags & 1) == 0).all()
    print(f"\n[many colliders C2] envs that overflowed the second bank in 8 steps: {int(((flags & 2) != 0).sum())}")
    again, _ = run(HipEngine(cm, cfg, n, seed=9))
    assert torch.equal(again, st)
    halves = [run(HipEngine(cm, cfg, n // 2, env_offset=off, seed=9), off, off + n // 2)[0] for off in (0, n // 2)]
    assert torch.equal(torch.cat(halves), st)
    grouped = EnvGroups(cm, cfg, n, groups=2, seed=9)
    gst, _ = run(grouped)
    grouped.join()
    assert torch.equal(gst, st)


def test_bank2_cap_does_not_bind_on_the_standing_task(torch_gpu):
    """The second bank's two-geom cap (select_bank2) against the task itself: the
    nine-collider model on the standing task with pushes (BASELINE C3's perturbation curriculum) and
    the bench's action noise (JOINT_BIASES + 0.05 N(0,1)), 16384 envs x 128 control steps with automatic
    resets: no env ever has more than two colliders beyond the soles within reach of the floor (the
    sticky flag stays clear). Measured at C3 (32768 envs x 256 steps, tests/diag_bank2_overflow.py): 0.
    Robots that fall (action noise 0.2, ~4 episode ends per env in 256 steps) do overflow: 8.9e-3 of
    env-steps carry the flag, most of them after the episode's fall has begun (the diag prints how many
    end their episode in the overflowing step). Also checks that bit 2 (this step's overflow) clears."""
    torch = torch_gpu
    from zbot_amd.engine import HipEngine

    cm = compile_model(U.many_desc())
    n, T = 16384, 128
    eng = HipEngine(cm, default_config(push=True), n, seed=11)
    bias = torch.tensor([cm.cmodel.joint_bias[i] for i in range(20)], device="cuda")
    g = torch.Generator(device="cuda")
    g.manual_seed(5)
    eng.reset()
    ends = torch.zeros((), dtype=torch.int64, device="cuda")
    for t in range(T):
        out = eng.step(bias + 0.05 * torch.randn(n, 20, device="cuda", generator=g), extras=False)
        ends += out["done"].sum()
    f = eng.flags()
    print(f"\n[bank-2 cap, standing task] {n} envs x {T} steps ({int(ends)} episode ends): envs that ever "
          f"overflowed {int(f['bank_overflow'].sum())}, non-finite {int(f['nonfinite'].sum())}")
    assert int(f["bank_overflow"].sum()) == 0 and int(f["nonfinite"].sum()) == 0
    assert int(f["bank_overflow_step"].sum()) == 0
