"""Summarise a phase-duplication run: marginal time and VALU of one more instance of each phase.
    python scripts/dup_report.py gpurun_out/<timing>.log gpurun_out/<pmc>.log [base=cur]"""
import re
import sys

rates, valu = {}, {}
for l in open(sys.argv[1]):
    m = re.match(r"libeng_(\S+)\.so\s+median (\d+)", l)
    if m:
        rates[m.group(1)] = int(m.group(2))
for l in open(sys.argv[2]):
    m = re.match(r"libeng_(\S+)\s+launches.*?VALU\s+(\d+)", l)
    if m:
        valu[m.group(1)] = int(m.group(2))
base = sys.argv[3] if len(sys.argv) > 3 else "cur"
b, bv = rates[base], valu[base]
t0 = 8192 / b * 1e3
print(f"base {b} env-steps/s, {t0:.4f} ms/launch, VALU/wave {bv}")
for k in sorted(rates, key=lambda k: -8192 / rates[k]):
    if k == base:
        continue
    t = 8192 / rates[k] * 1e3
    print(f"{k:14s} dt {100 * (t - t0) / t0:5.1f}%   dVALU {valu.get(k, 0) - bv:6d} ({100 * (valu.get(k, 0) - bv) / bv:4.1f}%)")
