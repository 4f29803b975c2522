"""A/B variants of zb::gae_kernel (diagnostic only; the product library is never built this way).

    python scripts/gae_variants.py build   # on the CPU: builds variants/libgae_<name>.so
    python scripts/gae_variants.py run     # on the GPU: times each variant at [256, 8192]

Each variant text-patches csrc/zb_ppo.hip (drop a phase) and links it with the
product's engine and C-ABI objects, so the timed entry point is zb_gae.
"""

import ctypes as C
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "ksim-gym-zbot_amd", "csrc")
OUT = os.path.join(ROOT, "variants")

SCAN = """        g = __builtin_fmaf(dc.y, g, dc.x);"""
PIPELINED_SCAN = """    if (tid < GE) {
      vcarry = sv[0][tid];
      float g = carry;
      constexpr int U = 16;
      float2 buf[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int kk = tl - 1 - u;
        const float2 x = sdc[max(kk, 0)][tid];
        buf[u] = kk >= 0 ? x : make_float2(0.f, 1.f);
      }
      for (int k0 = tl - 1; k0 >= 0; k0 -= U) {
        float2 nb[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int kk = k0 - U - u;
          const float2 x = sdc[max(kk, 0)][tid];
          nb[u] = kk >= 0 ? x : make_float2(0.f, 1.f);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
          g = __builtin_fmaf(buf[u].y, g, buf[u].x);
          if (k0 - u >= 0) sv[k0 - u][tid] = g;
        }
#pragma unroll
        for (int u = 0; u < U; ++u) buf[u] = nb[u];
      }
      carry = g;
    }
    __syncthreads();

    /* 4. stream"""


def _scan_block(src):
    a = src.index("    if (tid < GE) {\n      vcarry = sv[0][tid];")
    b = src.index("    /* 4. stream")
    return src[a:b + len("    /* 4. stream")]


VARIANTS = {
    "base": [],
    "noscan": [(SCAN, "        g = dc.x;")],
    "nostore": [("        st4<VEC>(a.gae, i, nvq, g4);\n        if (a.vtarget) st4<VEC>(a.vtarget, i, nvq, t4);",
                 "        if (g4[0] == 12345.f) st4<VEC>(a.gae, i, nvq, g4);")],
    "pipelinedscan": [("@SCANBLOCK@", PIPELINED_SCAN)],
    "nodelta": [("          sdc[row][4 * q + k] = make_float2((rr[j][k] + gn) - vv[j][k], a.gl * mask);",
                 "          if (gn == 12345.f) sdc[row][4 * q + k] = make_float2(rr[j][k], mask);")],
}


def build():
    os.makedirs(OUT, exist_ok=True)
    subprocess.run(["make", "-C", CSRC, "-s"], check=True)
    src = open(os.path.join(CSRC, "zb_ppo.hip")).read()
    for name, patches in VARIANTS.items():
        s = src
        for a, b in patches:
            if a == "@SCANBLOCK@":
                a = _scan_block(s)
            assert a in s, (name, a)
            s = s.replace(a, b)
        p = os.path.join(OUT, f"gae_{name}.hip")
        open(p, "w").write(s)
        obj = os.path.join(OUT, f"gae_{name}.o")
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC",
                        f"-I{ROOT}/include", f"-I{CSRC}", "-fno-math-errno", "-c", "-o", obj, p], check=True)
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-shared", "-fPIC", "-o",
                        os.path.join(OUT, f"libgae_{name}.so"), os.path.join(CSRC, "build", "zb_engine.o"),
                        os.path.join(CSRC, "build", "zb_capi.o"), obj], check=True)
        print("built", name)


def run():
    import torch

    T, n = 256, 8192
    dev = torch.device("cuda", 0)
    rew = torch.randn(T, n, device=dev)
    val = torch.randn(T, n, device=dev)
    done = (torch.rand(T, n, device=dev) < 0.01).to(torch.uint8)
    gae = torch.empty(T, n, device=dev)
    vt = torch.empty(T, n, device=dev)
    part = torch.empty(2 * n // 32, dtype=torch.float64, device=dev)
    flush = torch.empty(512 << 20, dtype=torch.uint8, device=dev)
    for name, warm in [(v, False) for v in VARIANTS] + [("base", True)]:
        L = C.CDLL(os.path.join(OUT, f"libgae_{name}.so"))
        vp = C.c_void_p
        L.zb_gae.argtypes = [vp, vp, vp, vp, vp, C.c_int, C.c_int, C.c_float, C.c_float, vp, vp, vp, vp, vp]
        for parts in (True, False):
            ts = []
            for rep in range(10):
                if not warm:
                    flush.fill_(rep)
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record()
                assert L.zb_gae(rew.data_ptr(), val.data_ptr(), done.data_ptr(), None, None, T, n, 0.99, 0.95,
                                gae.data_ptr(), vt.data_ptr(), part.data_ptr() if parts else None, None, None) == 0
                b.record()
                torch.cuda.synchronize()
                ts.append(a.elapsed_time(b) * 1e3)
            ts = sorted(ts[2:])
            print(json.dumps(dict(variant=name, warm_cache=warm, moments=parts, us=ts[len(ts) // 2])), flush=True)


if __name__ == "__main__":
    build() if sys.argv[1] == "build" else run()
