"""Repeated zb_policy_actor / zb_policy_critic launches at 8192 envs (profiling driver for
scripts/pmc_policy.sh)."""

import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ksim-gym-zbot_amd"))
from zbot_amd import policy as P  # noqa: E402

n, reps = int(sys.argv[1]), int(sys.argv[2])
for kind, nin in ((P.ACTOR, P.ACTOR_IN), (P.CRITIC, P.CRITIC_IN)):
    pol = P.GruPolicy(kind, np.ascontiguousarray(P.init_params(kind, 0)))
    obs = torch.randn(n, nin, device="cuda")
    carry = pol.initial_carry(n)
    for r in range(reps):
        if kind == P.ACTOR:
            pol.actor(obs, carry, seed=1, step=r)
        else:
            pol.critic(obs, carry)
torch.cuda.synchronize()
print("ok", n, reps)
