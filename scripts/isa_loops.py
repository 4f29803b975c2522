"""Loop-level instruction mix of one kernel in a hipcc --save-temps .s file (static counts per
natural loop: back edges to an earlier label). Diagnostic for register-spill reloads (v_readlane of
spilled SGPRs) and the VALU / LDS mix inside the solver loops.

    python scripts/isa_loops.py <file.s> <kernel symbol>
"""
import re
import sys

s = open(sys.argv[1]).read()
name = sys.argv[2]
i = s.find(name + ":")
j = s.find(".Lfunc_end", i)
labels, ins = {}, []
for raw in s[i:j].split("\n")[1:]:
    l = raw.split(";")[0].strip()
    if not l:
        continue
    if l.endswith(":"):
        labels[l[:-1]] = len(ins)
        continue
    if l.startswith("."):
        continue
    ins.append(l)
loops = []
for k, l in enumerate(ins):
    m = re.match(r"s_(cbranch_\w+|branch)\s+(\S+)", l)
    if m and m.group(2) in labels and labels[m.group(2)] <= k:
        loops.append((labels[m.group(2)], k))
print(f"{name}: {len(ins)} instructions, {len(loops)} loops")
for a, b in sorted(loops):
    seg = ins[a:b + 1]

    def cnt(p):
        return sum(1 for x in seg if x.startswith(p))

    print(f"loop [{a:5d},{b:5d}] len {b - a + 1:5d} readlane {cnt('v_readlane'):3d} writelane {cnt('v_writelane'):3d} "
          f"valu {cnt('v_'):5d} ds {cnt('ds_'):4d} bperm {cnt('ds_bpermute'):3d} waitcnt {cnt('s_waitcnt'):3d} "
          f"salu {cnt('s_') - cnt('s_waitcnt') - cnt('s_nop'):4d} nop {cnt('s_nop'):3d}")
