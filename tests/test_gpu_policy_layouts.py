"""The one-wave policy layout (ZB_POL_LAYOUT_WAVE) against the 8-wave block layout: actions, log
probabilities, values and carries bit-identical over several steps, with resets and env counts
that leave partial tiles (the block layout itself is bit-exact against the oracle,
tests/test_gpu_policy.py)."""

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch_gpu():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch


def _bits(t):
    return t.contiguous().view(-1).cpu().numpy().view(np.uint8)


@pytest.mark.parametrize("n", [77, 512])
@pytest.mark.parametrize("mode", [0, 1, 2])
def test_actor_layouts_bit_identical(torch_gpu, n, mode):
    torch = torch_gpu
    from zbot_amd import policy as P

    g = torch.Generator(device="cuda").manual_seed(n + mode)
    T = 3
    obs = torch.randn(T, n, P.ACTOR_IN, device="cuda", generator=g)
    reset = (torch.rand(T, n, device="cuda", generator=g) < 0.2).to(torch.uint8)
    carry0 = 0.5 * torch.randn(n, P.DEPTH, P.HIDDEN, device="cuda", generator=g)
    given = torch.randn(T, n, P.JOINTS, device="cuda", generator=g)
    outs = []
    for layout in (P.LAYOUT_BLOCK, P.LAYOUT_WAVE, P.LAYOUT_WAVE2, P.LAYOUT_WAVE4):
        pol = P.GruPolicy(P.ACTOR, P.init_params(P.ACTOR, seed=4), layout=layout)
        carry = carry0.clone()
        acts = given.clone() if mode == P.EVAL else None
        a, lp = pol.actor(obs, carry, reset=reset, mode=mode, seed=7, env_offset=100, step=5, actions=acts,
                          log_prob=True)
        torch.cuda.synchronize()
        outs.append((a, lp, carry))
    for other in outs[1:]:
        for x, y in zip(outs[0], other):
            np.testing.assert_array_equal(_bits(y), _bits(x))


@pytest.mark.parametrize("n", [45, 300])
def test_critic_layouts_bit_identical(torch_gpu, n):
    torch = torch_gpu
    from zbot_amd import policy as P

    g = torch.Generator(device="cuda").manual_seed(n)
    T = 3
    obs = torch.randn(T, n, P.CRITIC_IN, device="cuda", generator=g)
    reset = (torch.rand(T, n, device="cuda", generator=g) < 0.2).to(torch.uint8)
    carry0 = 0.5 * torch.randn(n, P.DEPTH, P.HIDDEN, device="cuda", generator=g)
    outs = []
    for layout in (P.LAYOUT_BLOCK, P.LAYOUT_WAVE, P.LAYOUT_WAVE2, P.LAYOUT_WAVE4):
        pol = P.GruPolicy(P.CRITIC, P.init_params(P.CRITIC, seed=5), layout=layout)
        carry = carry0.clone()
        v = pol.critic(obs, carry, reset=reset)
        torch.cuda.synchronize()
        outs.append((v, carry))
    for other in outs[1:]:
        for x, y in zip(outs[0], other):
            np.testing.assert_array_equal(_bits(y), _bits(x))


def test_bad_layout_raises(torch_gpu):
    from zbot_amd import policy as P
    from zbot_amd.engine import ZbError

    pol = P.GruPolicy(P.ACTOR)
    with pytest.raises(ZbError):
        pol.set_layout(7)


@pytest.mark.parametrize("kind", ["critic", "actor"])
def test_persistent_launch_bit_identical(torch_gpu, kind):
    """The block layout's persistent launch (one launch over T steps, the carry in registers between
    steps; zb_policy_set_persistent) against one launch per step: values / actions / log
    probabilities and the final carry bit-identical over a 33-step call with episode restarts and a
    partial last tile."""
    torch = torch_gpu
    from zbot_amd import policy as P

    n, T = 300, 33
    spec = P.CRITIC if kind == "critic" else P.ACTOR
    g = torch.Generator(device="cuda").manual_seed(17)
    obs = torch.randn(T, n, P.CRITIC_IN if kind == "critic" else P.ACTOR_IN, device="cuda", generator=g)
    reset = (torch.rand(T, n, device="cuda", generator=g) < 0.05).to(torch.uint8)
    carry0 = 0.5 * torch.randn(n, P.DEPTH, P.HIDDEN, device="cuda", generator=g)
    outs = []
    for persistent in (True, False):
        pol = P.GruPolicy(spec, P.init_params(spec, seed=6), layout=P.LAYOUT_BLOCK)
        pol.set_persistent(persistent)
        carry = carry0.clone()
        if kind == "critic":
            res = [pol.critic(obs, carry, reset=reset)]
        else:
            acts, lp = pol.actor(obs, carry, reset=reset, seed=3, step=5, log_prob=True)
            res = [acts, lp]
        torch.cuda.synchronize()
        outs.append([_bits(r) for r in res] + [_bits(carry)])
    for a, b in zip(*outs):
        np.testing.assert_array_equal(a, b)
