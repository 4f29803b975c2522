"""The solver-event diagnostic (scripts/solver_counts.py) still patches the CPU twin it counts: its text
anchors match oracle/zb_oracle.c and the counting build reports plausible per-substep rates."""
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_solver_counts_runs():
    out = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "solver_counts.py"), "--envs", "8",
                          "--steps", "2", "--warmup", "2"], check=True, capture_output=True, text=True).stdout
    m = re.search(r"Newton solves ([0-9.]+), line searches ([0-9.]+), evaluations ([0-9.]+)", out)
    assert m, out
    newton, ls, ev = map(float, m.groups())
    assert 0.9 <= newton <= 1.0  # one Newton solve per substep (every env has floor contacts)
    assert 1.0 <= ls <= 8.0 and ls <= ev
    assert "warm-start active set" in out
