"""Chunked step (zb_step's substeps split into work units): timing per chunk count
and bit-exactness against the unchunked step, in ONE process.

    python tests/diag_chunks.py [--sizes 8192,32768] [--chunks 1,2,4,5,10] [--steps 16 --rounds 3]
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ksim-gym-zbot_amd"))
import torch  # noqa: E402
from zbot_amd import compile_model, default_config  # noqa: E402
from zbot_amd.engine import HipEngine  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="8192,32768")
    ap.add_argument("--chunks", default="1,2,4,5,10")
    ap.add_argument("--steps", type=int, default=16)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--push", action="store_true")
    a = ap.parse_args()
    cm = compile_model()
    cfg = default_config(solver="newton", push=a.push, randomize=a.push)
    bias = torch.tensor([cm.cmodel.joint_bias[i] for i in range(20)], device="cuda")
    chunks = [int(k) for k in a.chunks.split(",")]
    for n in [int(x) for x in a.sizes.split(",")]:
        g = torch.Generator(device="cuda")
        g.manual_seed(7)
        acts = [bias + 0.05 * torch.randn(n, 20, device="cuda", generator=g) for _ in range(8)]
        engs = []
        for k in chunks:
            os.environ["ZB_STEP_CHUNKS"] = str(k)
            engs.append(HipEngine(cm, cfg, n, seed=0))
        os.environ.pop("ZB_STEP_CHUNKS")
        outs = []
        for e in engs:
            e.reset()
            o = None
            for t in range(12):
                o = e.step(acts[t % 8])
            outs.append((e.get_state().clone(), e.solver_iters().clone(), {k: v.clone() for k, v in o.items()}))
            torch.cuda.synchronize()
            print(f"n={n} engine done, min iters {outs[-1][1].min().item()}", flush=True)
        torch.cuda.synchronize()
        st0, it0, o0 = outs[0]
        for k, (st, it, o) in zip(chunks[1:], outs[1:]):
            same = torch.equal(st.view(torch.int32), st0.view(torch.int32)) and torch.equal(it, it0)
            same = same and all(torch.equal(o[x], o0[x]) for x in o0)
            print(f"n={n} K={k}: bit-exact vs K={chunks[0]}: {same}", flush=True)
        res = {k: [] for k in chunks}
        for r in range(a.rounds):
            for k, e in zip(chunks, engs):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for t in range(a.steps):
                    e.step(acts[t % 8], extras=False)
                torch.cuda.synchronize()
                res[k].append(n * a.steps / (time.perf_counter() - t0))
        for k in chunks:
            v = sorted(res[k])
            print(f"n={n} K={k:2d} median {v[len(v)//2]:.0f} env-steps/s  all {[round(x) for x in v]}", flush=True)
        del engs


if __name__ == "__main__":
    main()
