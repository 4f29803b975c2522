"""Timing of the chunked step's per-chunk overhead across library variants (diagnostic).

    python tests/diag_chunk_overhead.py lib1.so lib2.so ... [--n 32768 --chunks 1,10 --rounds 3]
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
    ap.add_argument("libs", nargs="+")
    ap.add_argument("--n", type=int, default=32768)
    ap.add_argument("--chunks", default="1,10")
    ap.add_argument("--steps", type=int, default=8)
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args()
    cm = compile_model()
    bias = torch.tensor([cm.cmodel.joint_bias[i] for i in range(20)], device="cuda")
    acts = [bias + 0.05 * torch.randn(a.n, 20, device="cuda") for _ in range(8)]
    engs = []
    for p in a.libs:
        for k in [int(x) for x in a.chunks.split(",")]:
            os.environ["ZB_STEP_CHUNKS"] = str(k)
            e = HipEngine(cm, default_config(solver="newton"), a.n, lib_path=os.path.abspath(p), seed=0)
            e.reset()
            for t in range(3):
                e.step(acts[t])
            engs.append((f"{os.path.basename(p)} K={k}", e))
    torch.cuda.synchronize()
    res = {name: [] for name, _ in engs}
    for r in range(a.rounds):
        for name, e in engs:
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for t in range(a.steps):
                e.step(acts[t % 8], extras=False)
            torch.cuda.synchronize()
            res[name].append((time.perf_counter() - t0) / a.steps * 1e3)
    for name, _ in engs:
        v = sorted(res[name])
        print(f"{name:36s} median {v[len(v)//2]:.3f} ms/step  all {[round(x, 3) for x in v]}", flush=True)


if __name__ == "__main__":
    main()
