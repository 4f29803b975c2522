"""Shape sweep of zb_gae kernel time (HIP events), for the GAE roofline analysis in DESIGN.md."""

import ctypes as C
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ksim-gym-zbot_amd"))
from zbot_amd import ppo as P  # noqa: E402

L = P.load_library()
dev = torch.device("cuda", 0)
res = []
for T, n in [(256, 8192), (256, 4096), (256, 2048), (128, 8192), (512, 8192), (256, 16384), (256, 32768),
             (1024, 8192), (64, 65536)]:
    rew = torch.randn(T, n, device=dev)
    val = torch.randn(T, n, device=dev)
    done = (torch.rand(T, n, device=dev) < 0.01).to(torch.uint8)
    gae = torch.empty(T, n, device=dev)
    vt = torch.empty(T, n, device=dev)
    part = torch.empty(int(L.zb_gae_partials_words(n)), dtype=torch.float64, device=dev)
    flush = torch.empty(512 << 20, dtype=torch.uint8, device=dev)
    ts = []
    for rep in range(8):
        flush.fill_(rep)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        assert L.zb_gae(rew.data_ptr(), val.data_ptr(), done.data_ptr(), None, None, T, n, C.c_float(0.99),
                        C.c_float(0.95), gae.data_ptr(), vt.data_ptr(), part.data_ptr(), None, None) == 0
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b) * 1e3)
    us = sorted(ts[2:])[len(ts[2:]) // 2]
    res.append(dict(T=T, n=n, us=us, GBs=17 * T * n / us / 1e3))
    print(json.dumps(res[-1]), flush=True)
