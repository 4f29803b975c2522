"""The ksim-shaped API over env groups: ZbotWalkingEnv(groups=G) gives the bits of
one handle, through a whole training-step cycle — begin_rollout, steps with pushes, randomization
and automatic resets, end_rollout's FeetAirtime row-0 patch and update_curriculum — and StepResult
reads see complete outputs without an explicit join.
"""

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _bits(t):
    return t.contiguous().view(-1).cpu().numpy().view(np.uint8)


def test_default_groups():
    from zbot_amd.task import default_groups

    assert default_groups(512) == 1 and default_groups(4095) == 1
    assert default_groups(4096) == 2 and default_groups(8192) == 2


@pytest.mark.parametrize("n,G", [(300, 2), (517, 3)])
def test_walking_env_groups_bit_identical(cmodel, n, G):
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from zbot_amd.task import ZbotWalkingEnv

    kw = dict(seed=9, model=cmodel, push=True, randomize=True, max_episode_sec=0.2)
    envs = {g: ZbotWalkingEnv(n, groups=g, **kw) for g in (1, G)}
    assert envs[G].groups == G and type(envs[G].engine).__name__ == "EnvGroups"
    gen = torch.Generator(device="cuda").manual_seed(2)
    bias = torch.tensor([cmodel.cmodel.joint_bias[a] for a in range(20)], device="cuda")
    T = 16
    acts = bias + 0.3 * torch.randn(2, T, n, 20, device="cuda", generator=gen)
    rec = {}
    for g, env in envs.items():
        r0 = env.reset()
        rows = {"reward": [], "done": [], "obs": [], "terms": []}
        levels = []
        for rollout in range(2):
            env.begin_rollout()
            rew = torch.empty(T, n, device="cuda")
            terms = torch.empty(T, n, 12, device="cuda")
            for t in range(T):
                r = env.step(acts[rollout, t])
                # reading a field joins the groups: these copies see the finished step
                rew[t].copy_(r.reward)
                terms[t].copy_(torch.stack([r.reward_terms[k] for k in r.reward_terms], 1))
                rows["done"].append(r.done.clone())
                rows["obs"].append(r.critic_inputs.clone())
            env.end_rollout(rew[0], terms[0])
            rows["reward"].append(rew.clone())
            rows["terms"].append(terms.clone())
            levels.append(env.update_curriculum())
        torch.cuda.synchronize()
        rec[g] = (rows, levels, env.engine.get_state(), r0.actor_inputs.clone())
    a, b = rec[1], rec[G]
    assert a[1] == b[1]
    for k in a[0]:
        for x, y in zip(a[0][k], b[0][k]):
            np.testing.assert_array_equal(_bits(y), _bits(x), err_msg=k)
    np.testing.assert_array_equal(_bits(b[2]), _bits(a[2]))
    assert int(torch.stack(a[0]["done"]).sum()) > 0  # resets inside the rollouts


def test_walking_env_open_loop_does_not_join(cmodel):
    """A loop that only steps leaves the groups unjoined between steps (the headline's overlap);
    reading the last result afterwards still gives the one-handle bits."""
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from zbot_amd.task import ZbotWalkingEnv

    n = 256
    acts = torch.from_numpy(np.random.default_rng(0).normal(0, 0.1, (6, n, 20)).astype(np.float32)).cuda()
    out = {}
    for g in (1, 2):
        env = ZbotWalkingEnv(n, groups=g, seed=3, model=cmodel)
        env.reset()
        joins = []
        if g == 2:
            real = env.engine.join
            env.engine.join = lambda: (joins.append(1), real())[1]
        for t in range(6):
            r = env.step(acts[t])
        assert joins == []
        out[g] = r.reward.clone()
        if g == 2:
            assert joins == [1]
        torch.cuda.synchronize()
    np.testing.assert_array_equal(_bits(out[2]), _bits(out[1]))
