"""Build probe variants of the step kernel that add work at one code point (diagnostic only).

    python scripts/probe_variants.py      -> evariants/libeng_<probe>.so

valu<N>: N independent FMAs (8 chains) per line-search evaluation, consumed opaquely: if the
         kernel is VALU-issue bound, time grows by the share those instructions add.
lat<N>:  N dependent LDS round trips (2 instructions each) per line-search evaluation: if the
         kernel is bound by its own dependency chains, time grows by their latency.
Timed against the unmodified kernel with tests/diag_variants.py.
"""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "ksim-gym-zbot_amd", "csrc", "zb_engine.hip")
OUT = os.path.join(ROOT, "evariants")
ANCHOR = "    float gg[2] = {g1, g2};\n    tsum_n<2>(gg);\n"

PROBES = {
    "valu64": """    {
      float p[8];
#pragma unroll
      for (int q = 0; q < 8; q++) p[q] = g1 + (float)q;
#pragma unroll
      for (int it = 0; it < 8; it++)
#pragma unroll
        for (int q = 0; q < 8; q++) p[q] = __builtin_fmaf(p[q], 1.0001f, g2);
      asm volatile("" :: "v"(p[0]), "v"(p[1]), "v"(p[2]), "v"(p[3]), "v"(p[4]), "v"(p[5]), "v"(p[6]), "v"(p[7]));
    }
""",
    "lat8": """    {
      float v = g1;
      volatile float* vp = &c.L->vec[V_TMP2][c.l];
#pragma unroll
      for (int q = 0; q < 8; q++) { *vp = v; v = *vp + 0.f; }
      asm volatile("" :: "v"(v));
    }
""",
}


def main():
    os.makedirs(OUT, exist_ok=True)
    src = open(SRC).read()
    assert src.count(ANCHOR) == 1
    for name, code in PROBES.items():
        p = os.path.join(OUT, f"zb_engine_{name}.hip")
        open(p, "w").write(src.replace(ANCHOR, code + ANCHOR))
        subprocess.run([os.path.join(ROOT, "scripts", "ab_build.sh"), name, "file", p], check=True)


if __name__ == "__main__":
    main()
