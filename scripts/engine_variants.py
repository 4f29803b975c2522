"""A/B compiler-option variants of the step kernel (diagnostic only; the product library is
never built this way).

    python scripts/engine_variants.py build   # on the CPU: variants/libeng_<name>.so
    python scripts/engine_variants.py run     # on the GPU: C2 (8192 envs) zb_step timing

Each variant compiles csrc/zb_engine.hip with extra flags and links it with the product's C-ABI,
PPO and policy objects, so the timed entry point is zb_step. Timing is round-robin over the
variants after a clock warm-up, so drift hits every variant alike.
"""

import ctypes as C
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "ksim-gym-zbot_amd", "csrc")
OUT = os.path.join(ROOT, "evariants")
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", f"-I{ROOT}/include", f"-I{CSRC}",
         "-fno-signed-zeros", "-freciprocal-math", "-fno-math-errno", "-fapprox-func", "-fno-slp-vectorize"]

VARIANTS = {
    "base": [],
    "waves1": ["-DZB_WAVES_PER_EU=1"],  # 512 registers, no spill, one wave per SIMD
    "base2": [],
}


def build():
    os.makedirs(OUT, exist_ok=True)
    subprocess.run(["make", "-C", CSRC, "-s"], check=True)
    for name, extra in VARIANTS.items():
        obj = os.path.join(OUT, f"eng_{name}.o")
        src = os.path.join(CSRC, "zb_engine.hip")
        if isinstance(extra, str) and extra.startswith("file:"):
            src, extra = extra[5:], []
        subprocess.run(["/opt/rocm/bin/hipcc", *FLAGS, *extra, "-c", "-o", obj, src], check=True)
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-shared", "-fPIC", "-o",
                        os.path.join(OUT, f"libeng_{name}.so"), obj, os.path.join(CSRC, "build", "zb_capi.o"),
                        os.path.join(CSRC, "build", "zb_ppo.o"), os.path.join(CSRC, "build", "zb_policy.o")],
                       check=True)
        print("built", name, flush=True)


def run():
    import torch

    sys.path.insert(0, os.path.join(ROOT, "ksim-gym-zbot_amd"))
    from zbot_amd import compile_model, default_config
    from zbot_amd import engine as E

    n = int(sys.argv[2]) if len(sys.argv) > 2 else 8192
    cm = compile_model()
    cfg = default_config()
    bias = torch.tensor([cm.cmodel.joint_bias[i] for i in range(20)], device="cuda")
    g = torch.Generator(device="cuda")
    g.manual_seed(0)
    acts = [bias + 0.05 * torch.randn(n, 20, device="cuda", generator=g) for _ in range(16)]
    engs = {}
    for name in VARIANTS:
        eng = E.HipEngine(cm, cfg, n, seed=1, lib_path=os.path.join(OUT, f"libeng_{name}.so"))
        eng.reset()
        engs[name] = eng
    for i in range(40):  # clocks up
        engs["base"].step(acts[i % 16], extras=False)
    torch.cuda.synchronize()
    times = {name: [] for name in VARIANTS}
    for rnd in range(4):
        for name, eng in engs.items():
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for t in range(16):
                eng.step(acts[t], extras=False)
            b.record()
            torch.cuda.synchronize()
            times[name].append(a.elapsed_time(b) / 16)
    # bit-identity of every variant with the first, from a fresh reset over 6 steps
    finals = {}
    for name in VARIANTS:
        eng = E.HipEngine(cm, cfg, n, seed=9, lib_path=os.path.join(OUT, f"libeng_{name}.so"))
        eng.reset()
        for t in range(6):
            eng.step(acts[t], extras=False)
        finals[name] = eng.get_state()
    first = next(iter(VARIANTS))
    for name in VARIANTS:
        ts = sorted(times[name])
        print(json.dumps(dict(variant=name, n=n, ms_per_step=ts[len(ts) // 2], ms_min=ts[0],
                              env_steps_per_s=n / ts[0] * 1e3,
                              bit_identical_to_first=bool(torch.equal(finals[name], finals[first])))), flush=True)


if __name__ == "__main__":
    build() if sys.argv[1] == "build" else run()
