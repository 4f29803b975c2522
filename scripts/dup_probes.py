"""Marginal cost of each phase of the step kernel by duplication (diagnostic only).

    python scripts/dup_probes.py                 -> evariants/libeng_d_<phase>.so
    (GPU) python tests/diag_variants.py evariants/libeng_schur.so evariants/libeng_d_*.so

Each probe runs ONE phase a second time at its call site, on opaque copies of its inputs, with
the result discarded: the phase's side effects are idempotent (same LDS values rewritten), so the
outputs stay bit-identical and the time difference against the unmodified kernel is what that
phase costs where it sits (latency the partner wave cannot hide included).
"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "ksim-gym-zbot_amd", "csrc", "zb_engine.hip")
OUT = os.path.join(ROOT, "evariants")
HELPER_AT = "/* Diagnostic phase stamps"
HELPER = """__device__ __forceinline__ float opqf(float x) { asm volatile("" : "+v"(x)); return x; }
#define SINK(x) asm volatile("" :: "v"(x) : "memory")
"""
B = "asm volatile(\"\" ::: \"memory\");"

PROBES = {
    # (anchor, code inserted BEFORE the anchor)
    "mulm_ls": ("  Mv = mul_m_dot(c, r, jr, search, V_TMP, r.Jv, -1, unused_);",
                f"  {{ {B} float d_ = mul_m(c, opqf(search), V_TMP); SINK(d_); }}\n"),
    "rowdot_ls": ("  tsync();\n  /* the quadratic's coefficients",
                  f"  {{ {B} float d_ = r.ex ? row_dot(c, r, V_TMP) : 0.f; SINK(d_); }}\n"),
    "update": ("    red[0] = update_constraint_lane<XG>(c, r, jr, x, qs, fs, Ma, grad);\n    red[1] = c.l < NV ? grad * grad : 0.f;\n    red[2]",
               f"    {{ {B} Rows r2 = r; float g2_; float d_ = update_constraint_lane<XG>(c, r2, jr, opqf(x), qs, fs, Ma, g2_); SINK(d_); SINK(g2_); }}\n"),
    "solve_nw": ("    const float mg = solve_ldl(c, grad, Dinv);",
                 f"    {{ {B} float d_ = solve_ldl(c, opqf(grad), Dinv); SINK(d_); }}\n"),
    "factor_h": ("  return full ? factor_ldl<true>(c, H, Hd, L->Hs) : factor_ldl<false>(c, H, Hd, L->Hs);",
                 f"  {{ {B} float H2[CAP]; for (int e = 0; e < CAP; e++) H2[e] = opqf(H[e]);\n"
                 "    float d_ = full ? factor_ldl<true>(c, H2, opqf(Hd), L->Hs) : factor_ldl<false>(c, H2, opqf(Hd), L->Hs); SINK(d_); }\n"),
    "factor_m": ("  float DinvM = factor_ldl<true>(c, X, Xd, L->M);",
                 f"  {{ {B} float X2[CAP]; for (int e = 0; e < CAP; e++) X2[e] = opqf(X[e]);\n"
                 "    float d_ = factor_ldl<true>(c, X2, opqf(Xd), L->M); SINK(d_); }\n"),
    "kin": ("  kinematics(c, s, ls, B);",
            f"  {{ {B} LaneS l2 = ls; l2.q = opqf(ls.q); BodyK B2; kinematics(c, s, l2, B2); SINK(B2.xp[0]); SINK(B2.xq[0]); }}\n"),
    "crb": ("  com_crb_m(c, s, ls, B, cm);",
            f"  {{ {B} float cm2[3]; BodyK B2 = B; B2.xp[0] = opqf(B2.xp[0]); com_crb_m(c, s, ls, B2, cm2); SINK(cm2[0]); }}\n"),
    "con": ("  make_constraints<XG>(c, s, ls, B, cm, r);",
            f"  {{ {B} Rows r2; float cm2[3] = {{opqf(cm[0]), cm[1], cm[2]}}; make_constraints<XG>(c, s, ls, B, cm2, r2); SINK(r2.D); SINK(r2.aref); }}\n"),
    "rne": ("  float bias = rne_project(c, B, ca, zero6);",
            f"  {{ {B} float ca2[6]; for (int k = 0; k < 6; k++) ca2[k] = opqf(ca[k]); float d_ = rne_project(c, B, ca2, zero6); SINK(d_); }}\n"),
    "solve_sm": ("  float qs = solve_ldl(c, fs, DinvM);",
                 f"  {{ {B} float d_ = solve_ldl(c, opqf(fs), DinvM); SINK(d_); }}\n"),
    "ls": ("    float alpha = line_search<XG>(c, r, jr, search, Ma, fs, grad, Mv);",
           f"    {{ {B} Rows r2 = r; float mv2; float a2 = line_search<XG>(c, r2, jr, opqf(search), Ma, fs, grad, mv2); SINK(a2); SINK(mv2); }}\n"),
    "hess_full": ("  float Dinv = hessian_factor<XG>(c, r, true, 0, 0, 0, 0);",
                  f"  {{ {B} float d_ = hessian_factor<XG>(c, r, true, 0, 0, 0, 0); SINK(d_); }}\n"),
    "warm": ("  STAMP(S_WARM);",
             f"  {{ {B} float Ma2 = mul_m(c, opqf(x), V_TMP); SINK(Ma2); }}\n"),
    "jdj": ("    jdj_mfma<false>();",
            f"    {{ {B} jdj_mfma<false>(); }}\n"),
    "comvel": ("  com_vel(c, B, qv, cdd);\n  float ca[6], zero6",
               f"  {{ {B} BodyK B2 = B; float c2[6]; com_vel(c, B2, opqf(qv), c2); SINK(c2[0]); SINK(B2.cv[0]); }}\n"),
}


def main():
    only = sys.argv[1:]
    os.makedirs(OUT, exist_ok=True)
    src = open(SRC).read()
    assert src.count(HELPER_AT) == 1
    base = src.replace(HELPER_AT, HELPER + HELPER_AT)
    for name, (anchor, code) in PROBES.items():
        if only and name not in only:
            continue
        assert base.count(anchor) == 1, (name, base.count(anchor))
        p = os.path.join(OUT, f"zb_engine_d_{name}.hip")
        open(p, "w").write(base.replace(anchor, code + anchor))
        subprocess.run([os.path.join(ROOT, "scripts", "ab_build.sh"), f"d_{name}", "file", p], check=True)


if __name__ == "__main__":
    main()
