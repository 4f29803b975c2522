"""Repeated zb_gae launches over a [T, n] rollout (profiling driver for scripts/pmc_gae.sh)."""

import ctypes as C
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ksim-gym-zbot_amd"))
from zbot_amd import ppo as P  # noqa: E402

T, n, reps = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
dev = torch.device("cuda", 0)
rew = torch.randn(T, n, device=dev)
val = torch.randn(T, n, device=dev)
done = (torch.rand(T, n, device=dev) < 0.01).to(torch.uint8)
gae = torch.empty(T, n, device=dev)
vt = torch.empty(T, n, device=dev)
L = P.load_library()
part = torch.empty(int(L.zb_gae_partials_words(n)), dtype=torch.float64, device=dev)
for _ in range(reps):
    assert L.zb_gae(rew.data_ptr(), val.data_ptr(), done.data_ptr(), None, None, T, n, C.c_float(0.99),
                    C.c_float(0.95), gae.data_ptr(), vt.data_ptr(), part.data_ptr(), None, None) == 0
    flush = torch.empty(512 << 20, dtype=torch.uint8, device=dev).fill_(1)  # evict L2/MALL between launches
torch.cuda.synchronize()
print("ok", T, n, reps)
