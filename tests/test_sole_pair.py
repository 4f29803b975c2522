"""The sole pair on the CPU (round 5): a model whose two box soles collide with each other compiles to
ZbModel.npair 1 (MuJoCo's contact-parameter mix), zb_create takes it (the XG 3 kernels), any other
self pair is still refused, and the oracle's box-box contacts act as internal forces: their Jacobian
rows have zero root columns (mj_jacDifPair) and they push the interpenetrating soles apart."""

import ctypes as C

import numpy as np

import collider_util as U
from zbot_amd import compile_model, default_config


def test_sole_pair_compiles_to_npair(cmodel):
    cm = compile_model(U.sole_pair_desc())
    m = cm.cmodel
    assert m.npair == 1 and m.nskip_pair == 0
    assert sorted([m.pair_geom[0], m.pair_geom[1]]) == [0, 1]
    assert cm.geom_names[m.pair_geom[0]] == "left_foot_sole"  # geom1 = the pair's first name
    np.testing.assert_allclose([m.pair_friction[k] for k in range(3)], [1.0, 0.005, 0.0001], rtol=1e-6)
    np.testing.assert_allclose([m.pair_solref[k] for k in range(2)], [0.02, 1.0], rtol=1e-6)
    np.testing.assert_allclose([m.pair_solimp[k] for k in range(5)], [0.9, 0.95, 0.001, 0.5, 2.0], rtol=1e-6)
    # MuJoCo's mix: the larger friction, the mean solref / solimp, the larger margin
    d = U.sole_pair_desc()
    for g in d["geoms"]:
        if g["name"] == "left_foot_sole":
            g.update(friction=[0.6, 0.01, 0.001], solref=[0.04, 2.0], margin=0.002)
    m2 = compile_model(d).cmodel
    np.testing.assert_allclose([m2.pair_friction[k] for k in range(3)], [1.0, 0.01, 0.001], rtol=1e-6)
    np.testing.assert_allclose([m2.pair_solref[k] for k in range(2)], [0.03, 1.5], rtol=1e-6)
    assert abs(m2.pair_margin - 0.002) < 1e-9
    # the default robot has no pair; drop_self_contacts compiles it without
    assert cmodel.cmodel.npair == 0
    assert compile_model(U.sole_pair_desc(), drop_self_contacts=True).cmodel.npair == 0


def test_other_self_pairs_are_still_refused():
    from zbot_amd import engine as E

    d = U.sole_pair_desc()
    d["self_pairs"].append(["left_foot_sole", "torso_box"])
    m = compile_model(d).cmodel
    assert m.npair == 1 and m.nskip_pair == 1  # the soles' pair is simulated, the other one is not
    L = E.load_library()
    h = C.c_void_p()
    assert L.zb_create(C.byref(m), C.byref(default_config(solver="newton")), 4, 0, 0, 0, C.byref(h)) == -4
    # the sole pair alone passes the model checks (no GPU here: zb_create stops at the device, not at -4)
    ok = compile_model(U.sole_pair_desc()).cmodel
    rc = L.zb_create(C.byref(ok), C.byref(default_config(solver="newton")), 4, 0, 0, 0, C.byref(h))
    assert rc != -4, L.zb_last_error()
    if rc == 0:
        L.zb_destroy(h)


def test_sole_pair_beside_floor_colliders_compiles(oracle_mod):
    """Round 6: the sole pair beside other floor colliders (the limbs model's shin
    box and hand capsule) compiles to npair 1 with all four colliders and passes zb_create's model
    checks (the XG 4 kernels: the floor bank and a bank of its own for the pair); the oracle collides
    both the pair and every floor collider."""
    from zbot_amd import engine as E

    cm = compile_model(U.limbs_pair_desc())
    m = cm.cmodel
    assert m.npair == 1 and m.nskip_pair == 0 and m.ngeom == 4
    assert sorted([m.pair_geom[0], m.pair_geom[1]]) == [0, 1]
    L = E.load_library()
    h = C.c_void_p()
    rc = L.zb_create(C.byref(m), C.byref(default_config()), 4, 0, 0, 0, C.byref(h))
    assert rc != -4, L.zb_last_error()
    if rc == 0:
        L.zb_destroy(h)
    # the crossing-and-touching states hold pair contacts and floor contacts of the shin / hand
    q = U.crossing_touching_states(cm, 32, 3)
    cfg = default_config()
    npair = nfloor = 0
    for e in range(32):
        p = oracle_mod.constraint_problem(m, cfg, q[e], np.zeros(26), precision="f64")
        npair += int(((p["type"] == 2) & (np.abs(p["J"][:, :6]).max(1) == 0)).any())
        nfloor += int(len(U.contacts(cm, q[e])[2]) + len(U.contacts(cm, q[e])[3]) > 0)
    assert npair >= 8 and nfloor >= 8, (npair, nfloor)


def test_pair_rows_are_internal_and_repulsive(oracle_mod):
    """In the air (no floor contact), legs crossed: every contact row of the pair has exact zero root
    columns (the free joint cannot feel an internal force), the normal forces are non-negative, and a
    few substeps reduce the soles' interpenetration."""
    cm = compile_model(U.sole_pair_desc())
    free = compile_model(U.sole_pair_desc(), drop_self_contacts=True)
    cfg = default_config(solver="newton")
    qs = U.crossing_states(cm, 12, seed=3)
    seen = 0
    for q in qs:
        p = oracle_mod.constraint_problem(cm.cmodel, cfg, q, np.zeros(26), precision="f64")
        rows = p["type"] == 2
        if not rows.any():
            continue
        seen += 1
        assert (p["J"][rows][:, :6] == 0).all()
        assert np.abs(p["J"][rows][:, 6:]).max() > 1e-3
        f = oracle_mod.forward_debug(cm.cmodel, cfg, q, np.zeros(26), precision="f64")
        assert f["ncon"] == rows.sum() // 4 and 1 <= f["ncon"] <= 4
        # both soles' touch sensors see the pair's normal force
        assert f["touch"][0] > 0 and f["touch"][1] > 0 and abs(f["touch"][0] - f["touch"][1]) < 1e-6 * f["touch"][0]

        # 30 substeps with and without the pair: the pair pushes the feet apart
        feet = []
        for model in (cm, free):
            qp, qv, _ = oracle_mod.simulate(model.cmodel, cfg, q, np.zeros(26), 30, precision="f64")
            assert np.isfinite(qp).all() and np.isfinite(qv).all()
            x = oracle_mod.forward_debug(model.cmodel, cfg, qp, qv, precision="f64")["xpos"]
            feet.append(np.linalg.norm(x[cm.cmodel.body_left_foot] - x[cm.cmodel.body_right_foot]))
        assert feet[0] > feet[1] + 1e-4, feet
    assert seen >= 8
