"""GPU parity of the GRU actor / critic, through the C
ABI (include/zbot_policy.h) via zbot_amd.policy.

Bar: bit-exact against the CPU oracle (oracle/zb_oracle_policy.c): the matrix
cores compute each product as the k-ordered fp32 fmaf chain the oracle runs,
and both sides share include/zbot_fmath.h for every transcendental and the RNG.
"""

import numpy as np
import pytest
import torch

from zbot_amd.policy import ACTOR, CRITIC, EVAL, MODE, SAMPLE, init_params

pytestmark = pytest.mark.gpu
D, H = 5, 128


@pytest.fixture(scope="module")
def pol():
    from zbot_amd import policy as P

    assert torch.cuda.is_available()
    return P


def _inputs(T, n, I, seed):
    rng = np.random.default_rng(seed)
    obs = rng.normal(size=(T, n, I)).astype(np.float32)
    carry = (0.5 * rng.normal(size=(n, D, H))).astype(np.float32)
    reset = (rng.random((T, n)) < 0.2).astype(np.uint8)
    return obs, carry, reset


@pytest.mark.parametrize("n,T,mode", [(1, 1, SAMPLE), (33, 3, SAMPLE), (256, 2, MODE), (70, 2, EVAL), (2048, 1, SAMPLE)])
def test_actor_bit_exact(pol, oracle_mod, n, T, mode):
    P = init_params(ACTOR, seed=3)
    obs, carry, reset = _inputs(T, n, 50, n + T)
    acts_in = (0.4 * np.random.default_rng(1).normal(size=(T, n, 20))).astype(np.float32) if mode == EVAL else None
    a_ref, lp_ref, c_ref = oracle_mod.policy_actor(P, obs, carry, reset, mode=mode, seed=9, env_offset=5, step0=17,
                                                   actions=acts_in, log_prob=True)
    net = pol.GruPolicy(ACTOR, P)
    c = torch.from_numpy(carry).cuda()
    a, lp = net.actor(torch.from_numpy(obs).cuda(), c, reset=torch.from_numpy(reset).cuda(), mode=mode, seed=9,
                      env_offset=5, step=17, actions=None if acts_in is None else torch.from_numpy(acts_in).cuda(),
                      log_prob=True)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(c.cpu().numpy(), c_ref)
    np.testing.assert_array_equal(a.cpu().numpy(), a_ref)
    np.testing.assert_array_equal(lp.cpu().numpy(), lp_ref)


@pytest.mark.parametrize("n,T", [(5, 2), (64, 3)])
def test_critic_bit_exact(pol, oracle_mod, n, T):
    P = init_params(CRITIC, seed=4)
    obs, carry, reset = _inputs(T, n, 484, 7 * n)
    v_ref, c_ref = oracle_mod.policy_critic(P, obs, carry, reset)
    net = pol.GruPolicy(CRITIC, P)
    c = torch.from_numpy(carry).cuda()
    v = net.critic(torch.from_numpy(obs).cuda(), c, reset=torch.from_numpy(reset).cuda())
    torch.cuda.synchronize()
    np.testing.assert_array_equal(v.cpu().numpy(), v_ref)
    np.testing.assert_array_equal(c.cpu().numpy(), c_ref)


def test_actor_shard_invariant(pol):
    """Envs keep their RNG streams and results whatever batch / offset they run in."""
    net = pol.GruPolicy(ACTOR, init_params(ACTOR, seed=6))
    obs, carry, _ = _inputs(1, 96, 50, 2)
    o = torch.from_numpy(obs[0]).cuda()
    c = torch.from_numpy(carry).cuda()
    full, _ = net.actor(o, c.clone(), seed=1, env_offset=0, step=3)
    part, _ = net.actor(o[40:].contiguous(), c[40:].clone(), seed=1, env_offset=40, step=3)
    assert torch.equal(full[40:], part)


def test_errors(pol):
    net = pol.GruPolicy(ACTOR, init_params(ACTOR))
    with pytest.raises(pol.ZbError):
        net.critic(torch.zeros(2, 484, device="cuda"), net.initial_carry(2))
    with pytest.raises(pol.ZbError):
        net.actor(torch.zeros(2, 50, device="cuda"), net.initial_carry(3))
    with pytest.raises(pol.ZbError):
        pol.GruPolicy(ACTOR, np.zeros(10, np.float32))


def test_policy_in_the_rollout_loop(pol, cmodel):
    """actor -> zb_step per control step, rows straight into [T, n] buffers; reproducible."""
    from zbot_amd import default_config
    from zbot_amd.engine import HipEngine

    runs = []
    for _ in range(2):
        eng = HipEngine(cmodel, default_config(solver="newton"), 64, seed=2)
        ro = pol.PolicyRollout(eng, pol.GruPolicy(ACTOR, init_params(ACTOR, seed=8)), seed=5)
        out = ro.run(6)
        torch.cuda.synchronize()
        runs.append({k: v.cpu().numpy() for k, v in out.items()})
    for k in runs[0]:
        np.testing.assert_array_equal(runs[0][k], runs[1][k])
    r = runs[0]
    assert np.isfinite(r["actions"]).all() and np.isfinite(r["reward"]).all() and np.isfinite(r["log_prob"]).all()
    assert r["obs_actor"].shape == (7, 64, 50)
    assert not np.array_equal(r["actions"][0, 0], r["actions"][0, 1])


def test_kinfer_step_matches_gpu_actor(pol):
    """The exported deployment step (zbot_amd.kinfer.ActorStep) and the GPU actor
    in MODE agree on the same observations and carries (tolerance: fp32 eager vs the matrix-core
    k-ordered chain, 2e-5)."""
    from zbot_amd import kinfer as K

    P = init_params(ACTOR, seed=5)
    rng = np.random.default_rng(4)
    off = K.param_count(ACTOR) - K.JOINTS - K.ACTOR_OUT  # b_out: spread the logits (no near-ties)
    P[off + 200:off + 300] += rng.normal(scale=2.0, size=100).astype(np.float32)
    step = K.ActorStep(P)
    n = 16
    obs, carry = [], []
    for _ in range(n):
        q = rng.normal(size=4)
        xs = (rng.uniform(-1, 1, 20), rng.normal(size=20), q, rng.uniform(-3, 3, 1), rng.uniform(-1, 1, 6))
        obs.append(step.observation(*(torch.tensor(x, dtype=torch.float32) for x in xs)))
        carry.append(torch.tensor(0.5 * rng.normal(size=(D, H)), dtype=torch.float32))
    obs, carry = torch.stack(obs), torch.stack(carry)
    with torch.no_grad():
        ref = [step.act(obs[e], carry[e]) for e in range(n)]
    g = pol.GruPolicy(ACTOR, P)
    c = carry.cuda().contiguous()
    a, _ = g.actor(obs.cuda(), c, mode=MODE)
    torch.cuda.synchronize()
    for e in range(n):
        np.testing.assert_allclose(a[e].cpu().numpy(), ref[e][0].numpy(), rtol=0, atol=2e-5)
        np.testing.assert_allclose(c[e].cpu().numpy(), ref[e][1].numpy(), rtol=0, atol=2e-5)


def test_rollout_step_graph_capture(pol):
    """zb_policy_actor -> zb_step captured in a HIP graph (torch.cuda.CUDAGraph) and replayed
    gives the bits of the same launches run eagerly: neither entry point allocates, copies to the
    host or synchronises (include/zbot.h, include/zbot_policy.h), so a rollout's launch-bound
    inner loop can be a graph."""
    from zbot_amd import compile_model, default_config
    from zbot_amd.engine import HipEngine

    n, T = 64, 3
    cm = compile_model()
    P = init_params(ACTOR, seed=2)
    runs = []
    for mode in ("eager", "graph"):
        eng = HipEngine(cm, default_config(solver="newton"), n, seed=4)
        eng.reset()
        actor = pol.GruPolicy(ACTOR, P)
        carry = actor.initial_carry(n)
        acts = torch.empty(n, 20, device="cuda")

        def body():
            for t in range(T):
                actor.actor(eng.obs_actor, carry, seed=5, step=t, actions=acts)
                eng.step(acts, extras=False)

        if mode == "eager":
            body()
        else:
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            g = torch.cuda.CUDAGraph()
            with torch.cuda.stream(s):
                with torch.cuda.graph(g, stream=s):
                    body()
            torch.cuda.current_stream().wait_stream(s)
            # capture records the launches without running them: the state is still the reset one
            g.replay()
        torch.cuda.synchronize()
        runs.append((eng.get_state().cpu().clone(), carry.cpu().clone(), acts.cpu().clone()))
    for a, b in zip(runs[0], runs[1]):
        assert torch.equal(a, b)


def test_rollout_records_critic_obs_of_acted_states(pol, cmodel):
    """obs_critic[t] is the state the actor acted in at step t (get_ppo_variables evaluates the
    critic there, train.py:1683-1729): row 0 is the reset observation, and a second rollout starts
    from the first one's obs_critic_next."""
    from zbot_amd import default_config
    from zbot_amd.engine import HipEngine, ZbError

    eng = HipEngine(cmodel, default_config(solver="newton"), 32, seed=6)
    ro = pol.PolicyRollout(eng, pol.GruPolicy(ACTOR, init_params(ACTOR, seed=1)), seed=2)
    ro.reset()
    reset_c = eng.obs_critic.clone()
    a = ro.run(3, record_critic=True)
    b = ro.run(2, record_critic=True)
    torch.cuda.synchronize()
    assert a["obs_critic"].shape == (3, 32, 484) and a["obs_critic_next"].shape == (32, 484)
    assert torch.equal(a["obs_critic"][0], reset_c)
    assert torch.equal(b["obs_critic"][0], a["obs_critic_next"])
    assert not torch.equal(a["obs_critic"][1], a["obs_critic"][0])
    ro.run(1)
    with pytest.raises(ZbError):
        ro.run(1, record_critic=True)
