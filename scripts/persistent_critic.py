"""The critic over a T-step rollout (bench.py's rollout pipeline shape: [T, n] observations, carry reset
on episode ends) as one persistent launch (zb_policy_set_persistent, the block layout's default) or T
launches: wall time per call by CUDA events, and the values' bits compared. Diagnostic only.

    python scripts/persistent_critic.py [n] [T] [reps]
"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ksim-gym-zbot_amd"))
from zbot_amd import policy as P  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
T = int(sys.argv[2]) if len(sys.argv) > 2 else 32
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 10
crit = P.GruPolicy(P.CRITIC, np.ascontiguousarray(P.init_params(P.CRITIC, 1)))
g = torch.Generator(device="cuda")
g.manual_seed(0)
obs = torch.randn(T, n, P.CRITIC_IN, device="cuda", generator=g)
reset = (torch.rand(T, n, device="cuda", generator=g) < 0.02).to(torch.uint8)
out = {}
for persistent in (True, False, True, False):
    crit.set_persistent(persistent)
    times = []
    for r in range(reps + 1):
        cc = crit.initial_carry(n)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        v = crit.critic(obs, cc, reset=reset)
        e1.record()
        torch.cuda.synchronize()
        if r:
            times.append(e0.elapsed_time(e1))
    out.setdefault(persistent, []).extend(times)
    ref = v.clone() if persistent else ref
    if not persistent:
        assert torch.equal(v, ref), "persistent and per-step values differ"
for persistent, ts in out.items():
    ts = sorted(ts)
    print(f"critic over T={T}, n={n}, {'one persistent launch' if persistent else f'{T} launches'}: "
          f"median {ts[len(ts) // 2]:.3f} ms, min {ts[0]:.3f} ms ({len(ts)} calls)")
print("values bit-identical")
