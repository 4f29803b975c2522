"""Solver event counts per physics substep on the C2 workload (diagnostic only).

    python scripts/solver_counts.py [--envs 64 --steps 40]

Builds a counting copy of the CPU twin (oracle/zb_oracle.c patched in a temporary directory,
never in the tree) and reports per substep: line searches, line-search evaluations (the closed-form
alpha = 0 point excluded, as in the engine), Newton iterations that do not terminate, those whose
active set changed (the engine's refactors), and how often the active set at the warm start equals
the previous substep's final one (the hit rate of a Hessian factored ahead from that guess).
"""
import argparse
import ctypes as C
import os
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "ksim-gym-zbot_amd"))

KEY = ("d->efc_type[r] * 100000 + (d->efc_type[r] == EFC_CONTACT ? d->con_geom[d->efc_id[r]] * 1000 + "
       "(r - d->con_efc[d->efc_id[r]]) + 10 * d->efc_id[r] : d->efc_id[r])")
PATCHES = [
    ("static real update_constraint(const ZbModel* m, ZbData* d, Solver* s) {",
     "long long g_cnt[8];\nvoid zbo_cnt_get(long long* o) { for (int i = 0; i < 8; i++) o[i] = g_cnt[i]; }\n"
     "void zbo_cnt_reset(void) { for (int i = 0; i < 8; i++) g_cnt[i] = 0; }\n"
     "static real update_constraint(const ZbModel* m, ZbData* d, Solver* s) {", 1),
    ("  int solver_iters;\n", "  int solver_iters;\n  int g_n, g_key[MAXEFC], g_act[MAXEFC], g_valid;\n", 1),
    ("    ls_eval(m, d, s, c1, c2, alpha, &d1, &d2);\n    if (FABS(d1) <= gtol) break;",
     "    ls_eval(m, d, s, c1, c2, alpha, &d1, &d2);\n    __atomic_add_fetch(&g_cnt[1], 1, __ATOMIC_RELAXED);\n"
     "    if (FABS(d1) <= gtol) break;", 1),
    ("  s.cost = update_constraint(m, d, &s);\n  hessian_solve(m, d, &s);\n"
     "  for (int i = 0; i < nv; i++) s.search[i] = -s.Mgrad[i];\n  int iter = 0;\n  while (iter < cfg->iterations) {\n"
     "    real alpha = line_search(m, d, &s, cfg);\n",
     "  s.cost = update_constraint(m, d, &s);\n"
     "  if (d->g_valid) {\n    int same = 1, keys[MAXEFC];\n    for (int r = 0; r < d->nefc; r++) keys[r] = KEY;\n"
     "    for (int r = 0; r < d->nefc && same; r++) if (d->efc_active[r]) { int f = 0; for (int q = 0; q < d->g_n; q++) "
     "if (d->g_key[q] == keys[r] && d->g_act[q]) f = 1; if (!f) same = 0; }\n"
     "    for (int q = 0; q < d->g_n && same; q++) if (d->g_act[q]) { int f = 0; for (int r = 0; r < d->nefc; r++) "
     "if (keys[r] == d->g_key[q] && d->efc_active[r]) f = 1; if (!f) same = 0; }\n"
     "    __atomic_add_fetch(&g_cnt[5], 1, __ATOMIC_RELAXED);\n    if (same) __atomic_add_fetch(&g_cnt[6], 1, __ATOMIC_RELAXED);\n  }\n"
     "  hessian_solve(m, d, &s);\n  for (int i = 0; i < nv; i++) s.search[i] = -s.Mgrad[i];\n  int iter = 0;\n"
     "  __atomic_add_fetch(&g_cnt[3], 1, __ATOMIC_RELAXED);\n  while (iter < cfg->iterations) {\n"
     "    real alpha = line_search(m, d, &s, cfg);\n    __atomic_add_fetch(&g_cnt[0], 1, __ATOMIC_RELAXED);\n".replace("KEY", KEY), 1),
    ("    real oldcost = s.cost;\n    s.cost = update_constraint(m, d, &s);\n    hessian_solve(m, d, &s);\n    iter++;\n",
     "    real oldcost = s.cost;\n    int pact[MAXEFC];\n    for (int r = 0; r < d->nefc; r++) pact[r] = d->efc_active[r];\n"
     "    s.cost = update_constraint(m, d, &s);\n    int ch = 0;\n    for (int r = 0; r < d->nefc; r++) ch |= pact[r] != d->efc_active[r];\n"
     "    hessian_solve(m, d, &s);\n    iter++;\n    {\n      real imp_ = scale * (oldcost - s.cost), gn_ = 0;\n"
     "      for (int i = 0; i < nv; i++) gn_ += s.grad[i] * s.grad[i];\n"
     "      int term = imp_ < cfg->tolerance || SQRT(gn_) * scale < cfg->tolerance || iter >= cfg->iterations;\n"
     "      if (!term) __atomic_add_fetch(&g_cnt[4], 1, __ATOMIC_RELAXED);\n"
     "      if (!term && ch) __atomic_add_fetch(&g_cnt[2], 1, __ATOMIC_RELAXED);\n    }\n", 1),
    ("  d->solver_iters += iter;\n}",
     "  d->solver_iters += iter;\n  d->g_n = d->nefc;\n  d->g_valid = 1;\n"
     "  for (int r = 0; r < d->nefc; r++) { d->g_key[r] = KEY; d->g_act[r] = d->efc_active[r]; }\n}".replace("KEY", KEY), 0),
]


def build(tmp):
    src = open(os.path.join(ROOT, "oracle", "zb_oracle.c")).read()
    for old, new, n in PATCHES:
        if n:
            assert src.count(old) == n, old[:60]
        src = src.replace(old, new, 1)  # n == 0: the first occurrence (solve_newton's)
    open(os.path.join(tmp, "zb_oracle.c"), "w").write(src)
    subprocess.run(["gcc", "-O2", "-fPIC", "-std=c11", "-fopenmp", "-ffp-contract=off", "-Wno-unused-function",
                    "-I" + os.path.join(ROOT, "include"), "-shared", "-o", os.path.join(tmp, "liboracle_zbot.so"),
                    os.path.join(tmp, "zb_oracle.c"), "-lm"], check=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=64)
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--warmup", type=int, default=20)
    a = ap.parse_args()
    import oracle  # noqa: PLC0415
    from zbot_amd import compile_model, default_config  # noqa: PLC0415

    with tempfile.TemporaryDirectory() as tmp:
        build(tmp)
        oracle.HERE = tmp
        cm = compile_model()
        env = oracle.OracleEnv(cm.cmodel, default_config(solver="newton"), a.envs)
        env.L.zbo_cnt_get.argtypes = [C.POINTER(C.c_longlong)]
        env.reset()
        for t in range(a.warmup + a.steps):
            if t == a.warmup:
                env.L.zbo_cnt_reset()
            env.step(oracle.synthetic_actions(cm.cmodel, 0, a.envs, 0, t))
        o = (C.c_longlong * 8)()
        env.L.zbo_cnt_get(o)
    sub = a.envs * a.steps * 20
    print(f"C2 workload, {a.envs} envs x {a.steps} env-steps after {a.warmup}: per substep")
    print(f"  Newton solves {o[3] / sub:.3f}, line searches {o[0] / sub:.3f}, evaluations {o[1] / sub:.3f} "
          f"({o[1] / max(o[0], 1):.2f} per line search)")
    print(f"  non-terminating iterations {o[4] / sub:.3f}, of which the active set changed (refactors) {o[2] / sub:.3f}")
    print(f"  warm-start active set == previous substep's final one: {o[6] / max(o[5], 1):.3f} of {o[5]} substeps")


if __name__ == "__main__":
    main()
