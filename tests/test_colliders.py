"""Floor colliders beyond the two box soles (VERDICT r02 missing item 3): the
oracle's contact sets against an independent numpy restatement of MuJoCo's primitive colliders
(tests/collider_util.py), the models' compilation and their acceptance by zb_create."""

import ctypes as C

import numpy as np
import pytest

import collider_util as U
from zbot_amd import compile_model, default_config
from zbot_amd import cstructs as cs


@pytest.fixture(scope="module", params=["limbs", "round"])
def variant(request):
    return request.param, compile_model(U.limbs_desc() if request.param == "limbs" else U.round_desc())


def test_variant_models_compile(variant):
    name, cm = variant
    m = cm.cmodel
    if name == "limbs":
        # the touch sensors' soles first (the engine's first contact-row bank), then document order
        assert cm.geom_names == ["right_foot_sole", "left_foot_sole", "right_shin", "left_hand"]
        assert list(m.geom_type)[:4] == [cs.GEOM_BOX, cs.GEOM_BOX, cs.GEOM_BOX, cs.GEOM_CAPSULE]
        np.testing.assert_allclose(list(m.geom_size[3])[:2], [0.012, np.hypot(0.01, 0.06) / 2], rtol=1e-6)
    else:
        assert cm.geom_names == ["right_foot_sole", "left_foot_sole", "head_ball"]
        assert list(m.geom_type)[:3] == [cs.GEOM_CAPSULE, cs.GEOM_CAPSULE, cs.GEOM_SPHERE]
        # the touch sensors read the capsule feet
        assert (m.geom_right_foot, m.geom_left_foot) == (0, 1)
    assert m.nskip_geom == 0
    for g in range(m.ngeom):
        assert m.geom_lastdof[g] == cm.bodies[m.geom_body[g]].lastdof


def test_zb_create_accepts_the_variants(variant):
    from zbot_amd import engine as E

    _, cm = variant
    L = E.load_library()
    h = C.c_void_p()
    rc = L.zb_create(C.byref(cm.cmodel), C.byref(default_config()), 4, 0, 0, 0, C.byref(h))
    assert rc != -4, L.zb_last_error()  # validation passes (no device here: -2)
    if rc == 0:
        L.zb_destroy(h)


@pytest.mark.parametrize("precision", ["f64", "f32"])
def test_oracle_contact_sets_match_mujoco_rules(variant, oracle_mod, precision):
    """Over states with every collider type touching the floor, the oracle's contact count equals
    the numpy restatement's (box: the corners below the centre within the margin, at most 4;
    capsule: the end spheres; sphere), and some contacts of every collider occur."""
    name, cm = variant
    cfg = default_config()
    qs = U.touching_states(cm, 96, seed=3).astype(np.float32)
    touched = np.zeros(cm.cmodel.ngeom, int)
    for e in range(len(qs)):
        ref = oracle_mod.forward_debug(cm.cmodel, cfg, qs[e], np.zeros(26, np.float32), precision=precision)
        cons = U.contacts(cm, qs[e].astype(np.float64))
        # a corner within 1e-6 of the floor or of the centre plane may fall either way in fp32
        margin_case = any(abs(d) < 1e-6 for c in cons for _, d in c)
        if not margin_case:
            assert ref["ncon"] == sum(len(c) for c in cons), (name, e)
        assert ref["nefc"] >= 4 * ref["ncon"]
        touched += np.array([len(c) > 0 for c in cons])
    assert (touched > 0).all(), touched


def test_tilted_box_keeps_mujocos_corners():
    """A known answer for the box rule: a 0.02 x 0.02 x 0.02 cube rolled 30 degrees about x, centre
    at height h. A corner's offset along z is y sin30 + z cos30 (y, z = +-0.01): below the centre are
    y- z- (-0.0137) and y+ z- (-0.0037), for both x (indices 0-3); y- z+ is at +0.0037. With
    h = 0.012 the deepest pair (y- z-, at -0.0017) is the only one in contact. (Pins the numpy
    restatement that test_oracle_contact_sets_match_mujoco_rules checks the oracle against.)"""
    c30, s30 = np.cos(np.pi / 6), np.sin(np.pi / 6)
    R = np.array([[1, 0, 0], [0, c30, -s30], [0, s30, c30]])
    got = U.box_corners(np.array([0.0, 0.0, 0.012]), R, [0.01, 0.01, 0.01])
    assert [i for i, _ in got] == [0, 1]  # y- z-: indices 0 (x-) and 1 (x+)
    np.testing.assert_allclose([d for _, d in got], [0.012 - 0.01 * (c30 + s30)] * 2)
    assert [i for i, _ in U.box_corners(np.array([0.0, 0.0, 0.0]), R, [0.01, 0.01, 0.01])] == [0, 1, 2, 3]


def test_limbs_asset_is_the_test_variant():
    """assets/zbot_like_limbs.xml (bench.py --model) is collider_util.limbs_desc written out."""
    import os

    from zbot_amd.mjcf import load_mjcf, to_mjcf
    from zbot_amd.model import DEFAULT_ASSET

    path = os.path.join(os.path.dirname(DEFAULT_ASSET), "zbot_like_limbs.xml")
    with open(path) as f:
        assert f.read() == to_mjcf(U.limbs_desc()) + "\n"
    a, b = compile_model(load_mjcf(path)).cmodel, compile_model(U.limbs_desc()).cmodel
    assert bytes(a) == bytes(b)
