"""Calibration for the GAE roofline: time zb_gae next to plain streaming kernels that move the
same bytes (torch copy / elementwise), cold (L2/MALL flushed) and back-to-back."""

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
T, n = 256, 8192
rew = torch.randn(T, n, device=dev)
val = torch.randn(T, n, device=dev)
done = (torch.rand(T, n, device=dev) < 0.01).to(torch.uint8)
gae = torch.empty(T, n, device=dev)
vt = torch.empty(T, n, device=dev)
part = torch.empty(2 * n // 32, dtype=torch.float64, device=dev)
big_src = torch.randn(T * n * 17 // 8, device=dev)  # 17.8 MB read + 17.8 MB write = 35.7 MB like one gae
big_dst = torch.empty_like(big_src)
flush = torch.empty(512 << 20, dtype=torch.uint8, device=dev)


def g():
    assert L.zb_gae(rew.data_ptr(), val.data_ptr(), done.data_ptr(), None, None, T, n, C.c_float(0.99),
                    C.c_float(0.95), gae.data_ptr(), vt.data_ptr(), part.data_ptr(), None, None) == 0


ops = {"zb_gae": g, "torch_copy_same_bytes": lambda: big_dst.copy_(big_src),
       "torch_add_3in_2out_like": lambda: (torch.add(rew, val, out=gae), torch.sub(rew, val, out=vt))}
for name, fn in ops.items():
    for cold in (True, False):
        ts = []
        for rep in range(12):
            if cold:
                flush.fill_(rep)
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for _ in range(1 if cold else 10):
                fn()
            b.record()
            torch.cuda.synchronize()
            ts.append(a.elapsed_time(b) * 1e3 / (1 if cold else 10))
        ts = sorted(ts[2:])
        us = ts[len(ts) // 2]
        print(json.dumps(dict(op=name, cold=cold, us=us, GBs=T * n * 17 / us / 1e3)), flush=True)
