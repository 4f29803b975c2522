"""C-ABI checks that need no GPU: struct layouts, exported symbols, defaults."""

import ctypes as C
import os
import re

import pytest

from zbot_amd import cstructs as cs
from zbot_amd import default_config
from zbot_amd import engine as E

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def hiplib():
    E.build_library()
    return E.load_library()


def test_struct_sizes_match_c(oracle_mod):
    L = oracle_mod.lib()
    assert L.zbo_struct_bytes(0) == C.sizeof(cs.ZbModel)
    assert L.zbo_struct_bytes(1) == C.sizeof(cs.ZbEnvConfig)


@pytest.mark.parametrize("which,cls", [(0, cs.ZbModel), (1, cs.ZbEnvConfig)])
def test_every_field_offset_matches_c(oracle_mod, which, cls):
    L = oracle_mod.lib()
    for name, _ in cls._fields_:
        off = L.zbo_field_offset(which, name.encode())
        assert off >= 0, f"{name} missing from the C offset table"
        assert off == getattr(cls, name).offset, name


def _declared_symbols():
    syms = set()
    for h in ("zbot.h", "zbot_ppo.h", "zbot_policy.h"):
        txt = open(os.path.join(ROOT, "include", h)).read()
        syms |= set(re.findall(r"\b(zb_[a-z_]+)\s*\(", txt))
    return sorted(syms)


def test_library_exports_every_declared_symbol(hiplib):
    syms = _declared_symbols()
    assert len(syms) >= 25
    assert {"zb_policy_create", "zb_policy_actor", "zb_policy_critic", "zb_policy_destroy"} <= set(syms)
    assert {"zb_gae", "zb_moments_combine", "zb_adv_normalize", "zb_gae_partials_words"} <= set(syms)
    for s in syms:
        assert hasattr(hiplib, s), f"libzbot_hip.so does not export {s}"


def test_library_layout_introspection(hiplib):
    assert hiplib.zb_model_struct_bytes() == C.sizeof(cs.ZbModel)
    assert hiplib.zb_config_struct_bytes() == C.sizeof(cs.ZbEnvConfig)
    assert hiplib.zb_state_stride() == cs.STATE_STRIDE
    assert hiplib.zb_rand_stride() == cs.RAND_STRIDE
    assert hiplib.zb_abi_version() >= 1


def test_c_default_config_matches_python(hiplib):
    c = cs.ZbEnvConfig()
    hiplib.zb_default_config(C.byref(c))
    p = default_config()
    assert c.solver == cs.SOLVER_CG and p.solver == cs.SOLVER_CG  # MJX's CG
    for name, _ in cs.ZbEnvConfig._fields_:
        a, b = getattr(c, name), getattr(p, name)
        if hasattr(a, "__len__"):
            assert list(a) == pytest.approx(list(b), rel=1e-6), name
        else:
            assert a == pytest.approx(b, rel=1e-6), name


def test_model_validation_errors(hiplib, cmodel):
    """zb_create rejects a corrupted model before touching any device."""
    bad = type(cmodel.cmodel).from_buffer_copy(cmodel.cmodel)
    bad.magic = 0
    h = C.c_void_p()
    rc = hiplib.zb_create(C.byref(bad), C.byref(default_config(solver="newton")), 4, 0, 0, 0, C.byref(h))
    assert rc == -1
    assert b"magic" in hiplib.zb_last_error()
    bad = type(cmodel.cmodel).from_buffer_copy(cmodel.cmodel)
    bad.nv = 40
    rc = hiplib.zb_create(C.byref(bad), C.byref(default_config(solver="newton")), 4, 0, 0, 0, C.byref(h))
    assert rc == -4


def test_tree_shape_validation(hiplib, cmodel):
    """The engine's kinematics / subtree sums / factorization rely on the tree
    shape (one branching body; root dof chain + unbranched limb chains):
    zb_create must reject models that break it (ZB_EMODEL), not mis-simulate."""
    h = C.c_void_p()
    m = cmodel.cmodel
    # a second branching body: re-parent a hand body onto the first arm link
    bad = type(m).from_buffer_copy(m)
    nb = bad.nbody
    first_leg = [b for b in range(2, nb) if bad.body_parent[b] == 1][0]
    leaf = [b for b in range(2, nb) if all(bad.body_parent[k] != b for k in range(nb))][-1]
    bad.body_parent[leaf] = first_leg + 1  # first_leg + 1 already has a child
    rc = hiplib.zb_create(C.byref(bad), C.byref(default_config(solver="newton")), 4, 0, 0, 0, C.byref(h))
    assert rc == -4 and b"branches" in hiplib.zb_last_error()
    # a branching limb in the dof tree: hang a limb dof off the middle of another limb
    bad = type(m).from_buffer_copy(m)
    heads = [k for k in range(6, bad.nv) if bad.dof_parent[k] == 5]
    k = heads[1]
    bad.dof_parent[k] = heads[0] + 1
    rc = hiplib.zb_create(C.byref(bad), C.byref(default_config(solver="newton")), 4, 0, 0, 0, C.byref(h))
    assert rc == -4 and b"unbranched" in hiplib.zb_last_error()


def test_bad_config_rejected(hiplib, cmodel):
    cfg = default_config(solver="newton")
    cfg.struct_bytes = 4
    h = C.c_void_p()
    rc = hiplib.zb_create(C.byref(cmodel.cmodel), C.byref(cfg), 4, 0, 0, 0, C.byref(h))
    assert rc == -1


def test_engine_fails_loudly_without_gpu(cmodel):
    import torch

    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(E.ZbError):
        E.HipEngine(cmodel, default_config(solver="newton"), 4)


def test_compiled_model_tables(cmodel):
    m = cmodel.cmodel
    assert m.nbody == 26 and m.nv == 26 and m.nq == 27 and m.nu == 20
    # ctrl order == qpos[7:] order == JOINT_BIASES order (train.py:1252-1253, 1358-1359)
    assert [m.act_dof[a] for a in range(20)] == list(range(6, 26))
    assert cmodel.joint_names == [n for n, _, _ in __import__("zbot_amd").JOINT_BIASES]
    # dof_desc consistent with dof_anc
    for d in range(m.nv):
        for k in range(m.nv):
            isdesc = k != d and m.dof_depth[k] > m.dof_depth[d] and m.dof_anc[k][m.dof_depth[d]] == d
            assert bool((m.dof_desc[d] >> k) & 1) == isdesc
    assert m.mrow_size + 8 <= 248
