"""A/B timing of the block-layout (8-wave) actor and critic across builds of the product library
(diagnostic, GPU). Each library runs in its own process: 8192 envs, 3 warm-up and 20 timed launches
per network by HIP events on the launch's stream (and the critic over a 32-step rollout as one
persistent launch), and the outputs of a fixed sequence, which the parent compares bit for bit
against the first library's.

    python scripts/policy_ab.py <lib.so> [<lib.so> ...]
"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(lib: str, out: str) -> None:
    import numpy as np
    import torch

    sys.path.insert(0, os.path.join(ROOT, "ksim-gym-zbot_amd"))
    import zbot_amd.engine as E

    E.LIB_PATH = lib
    from zbot_amd import policy as P

    n = 8192
    res, arrs = {"lib": lib}, {}
    for kind, nin, name in ((P.ACTOR, P.ACTOR_IN, "actor"), (P.CRITIC, P.CRITIC_IN, "critic")):
        pol = P.GruPolicy(kind, np.ascontiguousarray(P.init_params(kind, 0)), layout=P.LAYOUT_BLOCK)
        g = torch.Generator(device="cuda").manual_seed(5)
        obs = torch.randn(4, n, nin, device="cuda", generator=g)
        reset = (torch.rand(4, n, device="cuda", generator=g) < 0.05).to(torch.uint8)
        carry = pol.initial_carry(n)
        for t in range(4):  # the bit-identity sequence (resets, a warm carry)
            if kind == P.ACTOR:
                a, lp = pol.actor(obs[t], carry, reset=reset[t], seed=3, step=t, log_prob=True)
                arrs[f"a{t}"], arrs[f"lp{t}"] = a.cpu().numpy(), lp.cpu().numpy()
            else:
                arrs[f"v{t}"] = pol.critic(obs[t], carry, reset=reset[t]).cpu().numpy()
        arrs[f"{name}_carry"] = carry.cpu().numpy()
        s = torch.cuda.current_stream()
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(20)]
        for r in range(23):
            if r >= 3:
                ev[r - 3][0].record(s)
            if kind == P.ACTOR:
                pol.actor(obs[r % 4], carry, seed=1, step=r)
            else:
                pol.critic(obs[r % 4], carry)
            if r >= 3:
                ev[r - 3][1].record(s)
        torch.cuda.synchronize()
        ms = sorted(a.elapsed_time(b) for a, b in ev)
        res[name] = {"ms_median": ms[len(ms) // 2], "ms_min": ms[0]}
        if kind == P.CRITIC:
            # the rollout pipeline's use: the critic over a 32-step rollout as one persistent launch
            o32 = torch.randn(32, n, nin, device="cuda", generator=g)
            c32 = pol.initial_carry(n)
            arrs["v32"] = pol.critic(o32, c32).cpu().numpy()
            arrs["c32"] = c32.cpu().numpy()
            tt = []
            for r in range(6):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(s)
                pol.critic(o32, c32)
                e1.record(s)
                torch.cuda.synchronize()
                if r:
                    tt.append(e0.elapsed_time(e1))
            res["critic_T32"] = {"ms_median": sorted(tt)[len(tt) // 2]}
    np.savez(out, **arrs)
    print(json.dumps(res), flush=True)


def main() -> None:
    if sys.argv[1] == "--child":
        child(sys.argv[2], sys.argv[3])
        return
    import numpy as np

    base = None
    for i, lib in enumerate(sys.argv[1:]):
        out = f"/tmp/policy_ab_{i}.npz"
        p = subprocess.run([sys.executable, __file__, "--child", os.path.abspath(lib), out], capture_output=True,
                           text=True, timeout=300)
        if p.returncode != 0:
            print(json.dumps({"lib": lib, "error": p.stderr[-2000:]}), flush=True)
            continue
        r = json.loads(p.stdout.strip().splitlines()[-1])
        z = dict(np.load(out))
        if base is None:
            base = z
        r["bit_identical_to_first"] = all(np.array_equal(base[k].view(np.uint32), z[k].view(np.uint32)) for k in base)
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
