"""Static instruction attribution of the step kernel to source call paths (diagnostic).

    python scripts/isa_attrib.py step_g.s [depth]

Input: the step kernel's device assembly compiled with -gline-tables-only (every instruction
carries a `.loc` with its inline call stack). Each VALU / SALU / LDS instruction is attributed to
the chain of enclosing functions of csrc/zb_engine.hip (outermost first), cut at `depth`
frames below step_kernel. Static counts only: multiply by the phase's calls per substep
(DESIGN.md phase table) for a dynamic estimate.
"""
import collections
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "ksim-gym-zbot_amd", "csrc", "zb_engine.hip")


def func_map():
    """zb_engine.hip line -> enclosing function name (by definition headers)."""
    lines = open(SRC).read().split("\n")
    names = [None] * (len(lines) + 2)
    cur = "?"
    pat = re.compile(r"^(?:template <[^>]*>\s*)?(?:__global__|__device__)[^(]*?\b(\w+)\s*\(")
    for i, l in enumerate(lines, 1):
        m = pat.match(l)
        if m:
            cur = m.group(1)
        names[i] = cur
    return names


def main():
    path = sys.argv[1]
    depth = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    names = func_map()
    loc_re = re.compile(r"zb_engine\.hip:(\d+):\d+")
    stack = ("?",)
    cnt = collections.defaultdict(lambda: collections.Counter())
    for l in open(path):
        if "\t.loc\t" in l:
            frames = [int(x) for x in loc_re.findall(l)]  # innermost first
            if frames:
                fn = [names[f] for f in reversed(frames)]  # outermost first
                # collapse consecutive duplicates (a function's own lines)
                out = []
                for f in fn:
                    if not out or out[-1] != f:
                        out.append(f)
                stack = tuple(out)
            continue
        m = re.match(r"\s+([vsdgb][a-z0-9_]+)", l)
        if not m or l.strip().startswith("."):
            continue
        op = m.group(1)
        kind = "valu" if op.startswith("v_") else "lds" if op.startswith("ds_") else "salu" if op.startswith("s_") else "mem"
        key = " > ".join(stack[1:1 + depth]) if len(stack) > 1 else stack[0]
        cnt[key][kind] += 1
    tot = sum(c["valu"] for c in cnt.values())
    for k, c in sorted(cnt.items(), key=lambda kv: -kv[1]["valu"]):
        print(f"{c['valu']:6d} {100.0 * c['valu'] / tot:5.1f}%  lds {c['lds']:5d} salu {c['salu']:5d}  {k}")


if __name__ == "__main__":
    main()
