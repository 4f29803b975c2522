"""A/B variants of zb::pol::policy_kernel (diagnostic only; the product library is never built this way).

    python scripts/policy_variants.py build   # on the CPU: builds variants/libpol_<name>.so
    python scripts/policy_variants.py run     # on the GPU: times the actor at 8192 envs

Each variant text-patches csrc/zb_policy.hip (drop a phase, or restructure one) and links it with
the product's engine, PPO and C-ABI objects, so the timed entry point is zb_policy_actor.
"""

import ctypes as C
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "ksim-gym-zbot_amd", "csrc")
OUT = os.path.join(ROOT, "variants")

CARRY_LOAD = """      if (ge < a.n && !(a.reset && a.reset[ge]))
        cr[j] = *reinterpret_cast"""
NO_CARRY_LOAD = """      if (ge < 0)
        cr[j] = *reinterpret_cast"""

EPI = """      const float r = zbf_sigmoid((ir[i] + br) + hr[i]);
      const float z = zbf_sigmoid((iz[i] + bz) + hz[i]);
      const float nn = zbf_tanh((in[i] + bni) + r * (hn[i] + bnh));"""
NO_EPI = """      const float r = (ir[i] + br) + hr[i];
      const float z = (iz[i] + bz) + hz[i];
      const float nn = (in[i] + bni) + r * (hn[i] + bnh);"""

HEAD = """    for (int it = tid; it < M * NJ; it += NTHR) {"""
NO_HEAD = """    for (int it = tid; it < (a.n < 0 ? M * NJ : 0); it += NTHR) {"""

# carry of layer l + 1 prefetched into registers while layer l runs
PF_DECL = """  int cur = 0;
  for (int l = 0; l < D; ++l) {"""
PF_DECL_NEW = """  int cur = 0;
  constexpr int CPT = M * (H / 4) / NTHR;
  float4 cr[CPT];
  auto load_carry = [&](int l) {
#pragma unroll
    for (int j = 0; j < CPT; ++j) {
      const int i = tid + j * NTHR;
      const int e = i / (H / 4), q = i - e * (H / 4);
      const int ge = e0 + e;
      cr[j] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (ge < a.n && !(a.reset && a.reset[ge]))
        cr[j] = *reinterpret_cast<const float4*>(a.carry + ((size_t)ge * D + l) * H + 4 * q);
    }
  };
  load_carry(0);
  for (int l = 0; l < D; ++l) {"""
PF_BODY_OLD_START = "    /* carry of layer l -> sh; zero for envs whose episode restarts at this step */"
PF_BODY_OLD_END = "    const float4* wih = wp4 + off_gru + (size_t)l * 2 * MAT + lane;"
PF_BODY_NEW = """    /* carry of layer l (prefetched during layer l - 1) -> sh */
#pragma unroll
    for (int j = 0; j < CPT; ++j) {
      const int i = tid + j * NTHR;
      const int e = i / (H / 4), q = i - e * (H / 4);
      sh[(4 * q) * LDA + e] = cr[j].x;
      sh[(4 * q + 1) * LDA + e] = cr[j].y;
      sh[(4 * q + 2) * LDA + e] = cr[j].z;
      sh[(4 * q + 3) * LDA + e] = cr[j].w;
    }
    __syncthreads();
    if (l + 1 < D) load_carry(l + 1);

"""


def _prefetch(s):
    if "load_carry" in s:  # already in the product source (r01_v17)
        return s
    s = s.replace(PF_DECL, PF_DECL_NEW)
    a = s.index(PF_BODY_OLD_START)
    b = s.index(PF_BODY_OLD_END)
    return s[:a] + PF_BODY_NEW + s[b:]


GLOOP = "    for (int g = 0; g < GH; ++g) {"
TLOOP = "  for (int g = 0; g < G; ++g) {"
TLOAD_END = "    const float4 bn = wp[(size_t)(g + 1 < G ? g + 1 : g) * 64];"
LOOP_OLD = """      const float* xp = xs + (8 * g + h2) * LDA + c32;
      const float* hp = sh + (8 * g + h2) * LDA + c32;
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const float ax = xp[2 * u * LDA], ah = hp[2 * u * LDA];"""
GLOAD_END = "      const float4 n3 = whh[tr + gn], n4 = whh[tz + gn], n5 = whh[tn + gn];"

def _sgb(nvalu):
    return [("        epi_row(g);\n", "        epi_row(g);\n#pragma unroll\n        for (int k = 0; k < 12; ++k) {\n"
             "          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);\n"
             f"          __builtin_amdgcn_sched_group_barrier(0x002, {nvalu}, 0);\n        }}\n")]


VARIANTS = {
    "base": [],
    # an earlier product kernel (e.g. `git show HEAD:.../zb_policy.hip`): ZB_POL_OLD or variants/zb_policy_prev.hip
    "prev": "file:" + os.environ.get("ZB_POL_OLD", os.path.join(OUT, "zb_policy_prev.hip")),
    "base2": [],
    # static priority for the second-dispatched half of the 8 waves (MI355X_MICROARCH.md, two waves
    # per SIMD, item 4): waves 4-7 win VALU / matrix issue arbitration against their SIMD partners
    "prio47": [("  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;\n",
                "  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;\n"
                "  if (__builtin_amdgcn_readfirstlane(w) >= NWAVE / 2) __builtin_amdgcn_s_setprio(1);\n")],
    "prio03": [("  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;\n",
                "  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;\n"
                "  if (__builtin_amdgcn_readfirstlane(w) < NWAVE / 2) __builtin_amdgcn_s_setprio(1);\n")],
}


def build():
    os.makedirs(OUT, exist_ok=True)
    subprocess.run(["make", "-C", CSRC, "-s"], check=True)
    src = open(os.path.join(CSRC, "zb_policy.hip")).read()
    for name, patches in VARIANTS.items():
        if patches == "prefetch":
            s = _prefetch(src)
        elif isinstance(patches, str) and patches.startswith("file:"):
            s = open(patches[5:]).read()
        else:
            s = src
            for a, b in patches:
                assert a in s, (name, a)
                s = s.replace(a, b)
        p = os.path.join(OUT, f"pol_{name}.hip")
        open(p, "w").write(s)
        obj = os.path.join(OUT, f"pol_{name}.o")
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC",
                        f"-I{ROOT}/include", f"-I{CSRC}", "-fno-math-errno", "-c", "-o", obj, p], check=True)
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-shared", "-fPIC", "-o",
                        os.path.join(OUT, f"libpol_{name}.so"), os.path.join(CSRC, "build", "zb_engine.o"),
                        os.path.join(CSRC, "build", "zb_capi.o"), os.path.join(CSRC, "build", "zb_ppo.o"),
                        os.path.join(CSRC, "build", "zb_host.o"), obj],
                       check=True)
        print("built", name)


def run():
    import numpy as np
    import torch

    sys.path.insert(0, os.path.join(ROOT, "ksim-gym-zbot_amd"))
    from zbot_amd.policy import ACTOR, CRITIC, init_params

    n = int(sys.argv[2]) if len(sys.argv) > 2 else 8192
    dev = torch.device("cuda", 0)
    KIND = CRITIC if os.environ.get("ZB_POL_KIND") == "critic" else ACTOR
    P = np.ascontiguousarray(init_params(KIND, 0), dtype=np.float32)
    obs = torch.randn(n, 50 if KIND == ACTOR else 484, device=dev)
    libs = {}
    for name in VARIANTS:
        L = C.CDLL(os.path.join(OUT, f"libpol_{name}.so"))
        vp = C.c_void_p
        L.zb_policy_create.argtypes = [C.c_int, vp, C.c_size_t, C.c_int, C.POINTER(vp)]
        L.zb_policy_actor.argtypes = [vp, vp, C.c_int, C.c_int, vp, vp, C.c_int, C.c_uint64, C.c_int, C.c_uint32,
                                      vp, vp, vp]
        L.zb_policy_critic.argtypes = [vp, vp, C.c_int, C.c_int, vp, vp, vp, vp]
        h = vp()
        assert L.zb_policy_create(KIND, P.ctypes.data, P.size, 0, C.byref(h)) == 0
        libs[name] = (L, h)
    carry = torch.zeros(n, 5, 128, device=dev)
    act = torch.empty(n, 20, device=dev)
    lp = torch.empty(n, 20, device=dev)

    def launch(name, step):
        L, h = libs[name]
        if KIND == ACTOR:
            assert L.zb_policy_actor(h, obs.data_ptr(), 1, n, carry.data_ptr(), None, 0, 7, 0, step,
                                     act.data_ptr(), lp.data_ptr(), None) == 0
        else:
            assert L.zb_policy_critic(h, obs.data_ptr(), 1, n, carry.data_ptr(), None, act.data_ptr(), None) == 0

    # clocks up: ~2 s of back-to-back launches before anything is timed
    for i in range(15000):
        launch("base", i)
    torch.cuda.synchronize()
    times = {name: [] for name in VARIANTS}
    outs = {}
    for rnd in range(4):  # round-robin, so drift hits every variant alike
        for name in VARIANTS:
            carry.zero_()
            ts = []
            for rep in range(25):
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record()
                launch(name, rep)
                b.record()
                torch.cuda.synchronize()
                ts.append(a.elapsed_time(b) * 1e3)
            times[name] += ts[5:]
            if rnd == 0:
                outs[name] = (act.clone(), carry.clone())
    for name in VARIANTS:
        ts = sorted(times[name])
        same = bool(torch.equal(outs[name][0], outs["base"][0]) and torch.equal(outs[name][1], outs["base"][1]))
        print(json.dumps(dict(variant=name, kind="critic" if KIND == CRITIC else "actor", n=n, us=ts[len(ts) // 2], us_min=ts[0], bit_identical_to_base=same)),
              flush=True)


if __name__ == "__main__":
    build() if sys.argv[1] == "build" else run()
