"""Build a phase-stamp library with extra stamp points injected at code anchors.

    python scripts/stamp_probe.py OUT.so "anchor text::name[::after]" ...

Each spec inserts `STAMP(S_X_<name>);` before (default) or after the first
occurrence of the anchor text in zb_engine.hip; the new slots extend the S_*
enum and ZB_NSTAMP. Run the result with
    python tests/diag_stamps.py --lib OUT.so --nslots N --names name1,name2,...
Diagnostic only: the product library is never built this way.
"""
import os
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "ksim-gym-zbot_amd", "csrc")


def main():
    out, specs = sys.argv[1], sys.argv[2:]
    src = open(os.path.join(CSRC, "zb_engine.hip")).read()
    hdr = open(os.path.join(CSRC, "zb_internal.h")).read()
    names = []
    for spec in specs:
        parts = spec.split("::")
        anchor, name = parts[0], parts[1]
        after = len(parts) > 2 and parts[2] == "after"
        i = src.index(anchor)
        ins = f"STAMP(S_X_{name});\n"
        if after:
            j = i + len(anchor)
            src = src[:j] + "\n" + ins + src[j:]
        else:
            src = src[:i] + ins + src[i:]
        names.append(name)
    extra = "".join(f"S_X_{n}, " for n in names)
    src = src.replace("S_ENTRY, NSTAMP", "S_ENTRY, " + extra + "NSTAMP")
    n = 20 + len(names)
    hdr = hdr.replace("#define ZB_NSTAMP      20", f"#define ZB_NSTAMP      {n}")
    with tempfile.TemporaryDirectory() as d:
        open(os.path.join(d, "zb_engine.hip"), "w").write(src)
        open(os.path.join(d, "zb_internal.h"), "w").write(hdr)
        # zb_capi.cpp must see the patched header: compiled from a copy beside it
        open(os.path.join(d, "zb_capi.cpp"), "w").write(open(os.path.join(CSRC, "zb_capi.cpp")).read())
        flags = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", f"-I{d}", f"-I{CSRC}", f"-I{ROOT}/include",
                 "-fno-signed-zeros", "-freciprocal-math", "-fno-math-errno", "-fapprox-func", "-fno-slp-vectorize",
                 "-DZB_STAMPS"]
        objs = []
        for f in ("zb_engine.hip", "zb_capi.cpp"):
            objs.append(os.path.join(d, f + ".o"))
            subprocess.run(["hipcc", *flags, "-c", "-o", objs[-1], os.path.join(d, f)], check=True)
        # the PPO / policy kernels and the host half are the product objects
        subprocess.run(["make", "-C", CSRC, "-s", "build/zb_ppo.o", "build/zb_policy.o", "build/zb_host.o"], check=True)
        objs += [os.path.join(CSRC, "build", o) for o in ("zb_ppo.o", "zb_policy.o", "zb_host.o")]
        subprocess.run(["hipcc", "--offload-arch=gfx950", "-shared", "-fPIC", "-o", out, *objs], check=True)
    print(n, ",".join(names))


if __name__ == "__main__":
    main()
