"""MJCF <-> descriptor converter (reference train.py:1326-1338).

The Z-Bot MJCF itself is network-fetched by the reference and absent here, so the
converter is pinned by round trips through the committed Z-Bot-like descriptor
(assets/zbot_like.json) and by MJCF semantics written out by hand (degree angles,
euler / axis-angle orientations, default classes, inertial frames)."""

import copy
import math
import xml.etree.ElementTree as ET

import numpy as np
import pytest

from zbot_amd import cstructs as cs
from zbot_amd.mjcf import _Defaults, load_mjcf, to_mjcf
from zbot_amd.model import compile_model, load_description, mass_matrix


def _fields(cm):
    m = cm.cmodel
    out = {}
    for name, _ in cs.ZbModel._fields_:
        v = getattr(m, name)
        out[name] = np.ctypeslib.as_array(v).copy() if hasattr(v, "_length_") else v
    return out


def _assert_same_model(a, b, rtol=0.0, atol=0.0):
    fa, fb = _fields(a), _fields(b)
    for k in fa:
        va, vb = np.asarray(fa[k], dtype=np.float64), np.asarray(fb[k], dtype=np.float64)
        if rtol == 0.0 and atol == 0.0:
            assert np.array_equal(va, vb), k
        else:
            np.testing.assert_allclose(va, vb, rtol=rtol, atol=atol, err_msg=k)
    assert a.joint_names == b.joint_names
    assert a.geom_names == b.geom_names
    assert a.site_names == b.site_names


def _tree_order(desc):
    """MJCF numbers sites and geoms in body-tree order (as MuJoCo's compiler does)."""
    d = copy.deepcopy(desc)
    order = {b["name"]: i for i, b in enumerate(d["bodies"])}
    for k in ("sites", "geoms"):
        d[k] = sorted(d[k], key=lambda e: order[e["body"]])
    return d


def test_round_trip_is_exact():
    desc = _tree_order(load_description())
    xml = to_mjcf(desc)
    ET.fromstring(xml)  # well-formed
    back = load_mjcf(xml)
    _assert_same_model(compile_model(desc), compile_model(back))
    # a second trip is a fixed point of the text
    assert to_mjcf(back) == to_mjcf(load_mjcf(to_mjcf(back)))


def test_round_trip_from_file(tmp_path):
    desc = _tree_order(load_description())
    p = tmp_path / "zbot.xml"
    p.write_text(to_mjcf(desc))
    _assert_same_model(compile_model(desc), compile_model(load_mjcf(str(p))))


def _with_degrees(xml: str) -> str:
    root = ET.fromstring(xml)
    root.find("compiler").set("angle", "degree")
    for j in root.iter("joint"):
        if "range" in j.attrib:
            j.set("range", " ".join(repr(math.degrees(float(x))) for x in j.get("range").split()))
    return ET.tostring(root, encoding="unicode")


def test_degree_ranges():
    desc = _tree_order(load_description())
    back = load_mjcf(_with_degrees(to_mjcf(desc)))
    for b0, b1 in zip(desc["bodies"], back["bodies"]):
        if "range" in b0.get("joint", {}):
            np.testing.assert_allclose(b1["joint"]["range"], b0["joint"]["range"], rtol=1e-15, atol=1e-15)
    _assert_same_model(compile_model(desc), compile_model(back), rtol=1e-12, atol=1e-14)


def test_default_angle_unit_is_degree():
    # MJCF's compiler default is degrees: a document without <compiler> reads ranges in degrees
    xml = to_mjcf(load_description())
    root = ET.fromstring(_with_degrees(xml))
    root.remove(root.find("compiler"))
    back = load_mjcf(ET.tostring(root, encoding="unicode"))
    ref = load_description()
    for b0, b1 in zip(ref["bodies"], back["bodies"]):
        if "range" in b0.get("joint", {}):
            np.testing.assert_allclose(b1["joint"]["range"], b0["joint"]["range"], rtol=1e-15, atol=1e-15)


@pytest.mark.parametrize("form", ["quat", "axisangle", "euler_xyz", "euler_zyx_extrinsic"])
def test_body_orientation_forms(form):
    desc = _tree_order(load_description())
    name = "imu"
    ang = 30.0
    q = [math.cos(math.radians(ang) / 2), 0.0, 0.0, math.sin(math.radians(ang) / 2)]
    want = copy.deepcopy(desc)
    next(b for b in want["bodies"] if b["name"] == name)["quat"] = q
    root = ET.fromstring(to_mjcf(want))
    root.find("compiler").set("angle", "degree")
    for j in root.iter("joint"):
        if "range" in j.attrib:
            j.set("range", " ".join(repr(math.degrees(float(x))) for x in j.get("range").split()))
    el = next(b for b in root.iter("body") if b.get("name") == name)
    del el.attrib["quat"]
    if form == "quat":
        el.set("quat", " ".join(repr(2.0 * x) for x in q))  # unnormalized on purpose
    elif form == "axisangle":
        el.set("axisangle", f"0 0 1 {ang}")
    elif form == "euler_xyz":
        el.set("euler", f"0 0 {ang}")
    else:
        root.find("compiler").set("eulerseq", "ZYX")
        el.set("euler", f"{ang} 0 0")
    back = load_mjcf(ET.tostring(root, encoding="unicode"))
    got = next(b for b in back["bodies"] if b["name"] == name)["quat"]
    np.testing.assert_allclose(got, q, rtol=0, atol=1e-15)
    _assert_same_model(compile_model(want), compile_model(back), rtol=1e-12, atol=1e-14)


def test_euler_intrinsic_composition():
    # intrinsic x-then-y: R = Rx(a) @ Ry(b)
    from zbot_amd.model import quat_to_mat

    xml = ('<mujoco><compiler angle="radian"/><worldbody><body name="b" euler="0.3 0.4 0">'
           '<freejoint/><inertial mass="1" diaginertia="1 1 1"/></body></worldbody></mujoco>')
    d = load_mjcf(xml)
    R = quat_to_mat(np.array(d["bodies"][0]["quat"]))
    ca, sa, cb, sb = math.cos(0.3), math.sin(0.3), math.cos(0.4), math.sin(0.4)
    Rx = np.array([[1, 0, 0], [0, ca, -sa], [0, sa, ca]])
    Ry = np.array([[cb, 0, sb], [0, 1, 0], [-sb, 0, cb]])
    np.testing.assert_allclose(R, Rx @ Ry, atol=1e-15)


def test_inertial_frame_quaternion():
    """<inertial quat> rotates the principal axes: a 90° turn about z swaps Ixx and Iyy."""
    desc = load_description()
    name = "right_knee_pitch_link"
    a = copy.deepcopy(desc)
    b = copy.deepcopy(desc)
    ba = next(x for x in a["bodies"] if x["name"] == name)
    bb = next(x for x in b["bodies"] if x["name"] == name)
    ba.pop("box", None)
    bb.pop("box", None)
    ba["inertia"] = [1e-4, 3e-4, 2e-4]
    bb["inertia"] = [3e-4, 1e-4, 2e-4]
    s = math.sqrt(0.5)
    ba["iquat"] = [s, 0.0, 0.0, s]
    ra = load_mjcf(to_mjcf(a))
    assert np.allclose(next(x for x in ra["bodies"] if x["name"] == name)["iquat"], ba["iquat"])
    ca, cb = compile_model(ra), compile_model(b)
    q = ca.reset_qpos()
    q[7:] += 0.2
    Ma = mass_matrix(ca.bodies, q, ca.nv, ca.dof_body, np.zeros(ca.nv))
    Mb = mass_matrix(cb.bodies, q, cb.nv, cb.dof_body, np.zeros(cb.nv))
    np.testing.assert_allclose(Ma, Mb, rtol=1e-12, atol=1e-15)
    # and it matters: without the quaternion the mass matrices differ
    ba.pop("iquat")
    cn = compile_model(a)
    Mn = mass_matrix(cn.bodies, q, cn.nv, cn.dof_body, np.zeros(cn.nv))
    assert not np.allclose(Mn, Mb, rtol=1e-6, atol=1e-12)
    assert list(_fields(ca)["body_iquat"][ca.body_names.index(name)]) != [1.0, 0.0, 0.0, 0.0]


def test_default_classes_nest_and_explicit_wins():
    root = ET.fromstring(
        '<default><joint damping="1" axis="0 1 0"/><geom type="box"/>'
        '<default class="leg"><joint armature="0.01"/>'
        '<default class="knee"><joint damping="2"/></default></default></default>')
    d = _Defaults(root)
    j = ET.fromstring('<joint name="k" class="knee" axis="1 0 0"/>')
    a = d.attrs(j, "main")
    assert a["damping"] == "2" and a["armature"] == "0.01" and a["axis"] == "1 0 0"
    a = d.attrs(ET.fromstring('<joint name="h"/>'), "leg")  # childclass
    assert a["damping"] == "1" and a["armature"] == "0.01" and a["axis"] == "0 1 0"
    assert d.attrs(ET.fromstring('<geom/>'), "main")["type"] == "box"
    with pytest.raises(ValueError):
        d.attrs(ET.fromstring('<joint class="nope"/>'), "main")


def test_joint_dynamics_override_servo_class():
    desc = load_description()
    root = ET.fromstring(to_mjcf(desc))
    j = next(x for x in root.iter("joint") if x.get("name") == "right_knee_pitch")
    j.set("damping", "0.25")
    back = load_mjcf(ET.tostring(root, encoding="unicode"))
    jd = next(b["joint"] for b in back["bodies"] if b.get("joint", {}).get("name") == "right_knee_pitch")
    assert back["servo_classes"][jd["servo"]]["damping"] == 0.25
    base = desc["servo_classes"][next(b["joint"]["servo"] for b in desc["bodies"]
                                      if b.get("joint", {}).get("name") == "right_knee_pitch")]
    assert back["servo_classes"][jd["servo"]]["kp"] == base["kp"]
    cm = compile_model(back)
    d = cm.bodies[cm.body_names.index(next(b["name"] for b in back["bodies"]
                                           if b.get("joint", {}).get("name") == "right_knee_pitch"))].dofadr
    assert _fields(cm)["dof_damping"][d] == 0.25


def test_floor_and_option():
    desc = load_description()
    root = ET.fromstring(to_mjcf(desc))
    root.find("option").set("timestep", "0.004")
    fl = next(g for g in root.iter("geom") if g.get("type") == "plane")
    fl.set("friction", "0.8")
    fl.set("solref", "0.01 1")
    back = load_mjcf(ET.tostring(root, encoding="unicode"))
    assert back["option"]["timestep"] == 0.004
    assert back["floor"]["friction"] == [0.8, 0.005, 0.0001]
    assert back["floor"]["solref"] == [0.01, 1.0]


@pytest.mark.parametrize(
    "xml,err",
    [
        ("<robot/>", "MJCF"),
        ("<mujoco><worldbody><body name='b'><joint name='s' type='slide'/>"
         "<inertial mass='1' diaginertia='1 1 1'/></body></worldbody></mujoco>", "slide"),
        ("<mujoco><worldbody><body name='b'><freejoint/></body></worldbody></mujoco>", "inertial"),
        ("<mujoco><worldbody><body name='b'><joint name='a'/><joint name='c'/>"
         "<inertial mass='1' diaginertia='1 1 1'/></body></worldbody></mujoco>", "one joint"),
    ],
)
def test_rejects_unsupported(xml, err):
    with pytest.raises(ValueError, match=err):
        load_mjcf(xml)


def test_committed_mjcf_asset_matches_descriptor():
    import os

    from zbot_amd.model import ASSET_DIR

    back = load_mjcf(os.path.join(ASSET_DIR, "zbot_like.xml"))
    _assert_same_model(compile_model(_tree_order(load_description())), compile_model(back))


def _one_body(geoms: str, compiler: str = '<compiler angle="radian"/>') -> dict:
    xml = (f"<mujoco>{compiler}<worldbody><body name='b'><freejoint/>{geoms}</body></worldbody></mujoco>")
    return load_mjcf(xml)["bodies"][0]


def _tensor(b):
    from zbot_amd.model import quat_to_mat

    R = quat_to_mat(np.array(b.get("iquat", [1.0, 0, 0, 0])))
    return R @ np.diag(b["inertia"]) @ R.T


def test_inertia_from_box_geom_matches_descriptor_box():
    b = _one_body("<geom type='box' size='0.02 0.03 0.05' mass='0.4' pos='0 0 0.01'/>")
    assert b["mass"] == 0.4 and b["ipos"] == [0.0, 0.0, 0.01] and "iquat" not in b
    from zbot_amd.model import _box_inertia

    np.testing.assert_allclose(b["inertia"], _box_inertia(0.4, [0.04, 0.06, 0.1]), rtol=1e-14)


def test_inertia_from_geoms_density_and_parallel_axes():
    r, d = 0.01, 0.05
    b = _one_body(f"<geom type='sphere' size='{r}' pos='{d} 0 0'/><geom type='sphere' size='{r}' pos='{-d} 0 0'/>")
    m1 = 1000.0 * 4.0 / 3.0 * math.pi * r ** 3
    assert b["mass"] == pytest.approx(2 * m1, rel=1e-14)
    np.testing.assert_allclose(b["ipos"], [0, 0, 0], atol=1e-18)
    i0 = 0.4 * m1 * r * r
    np.testing.assert_allclose(_tensor(b), np.diag([2 * i0, 2 * (i0 + m1 * d * d), 2 * (i0 + m1 * d * d)]),
                               rtol=1e-12, atol=1e-18)


def test_inertia_from_rotated_geom_gives_inertial_frame():
    q = [math.cos(0.3), 0.0, math.sin(0.3) * math.sqrt(0.5), math.sin(0.3) * math.sqrt(0.5)]
    b = _one_body(f"<geom type='box' size='0.01 0.02 0.04' density='500' quat='{' '.join(map(repr, q))}'/>")
    from zbot_amd.model import quat_to_mat

    m = 500.0 * 8 * 0.01 * 0.02 * 0.04
    R = quat_to_mat(np.array(q))
    want = R @ np.diag([m / 3 * (0.02 ** 2 + 0.04 ** 2), m / 3 * (0.01 ** 2 + 0.04 ** 2),
                        m / 3 * (0.01 ** 2 + 0.02 ** 2)]) @ R.T
    assert "iquat" in b
    np.testing.assert_allclose(_tensor(b), want, rtol=1e-10, atol=1e-16)


@pytest.mark.parametrize("gt", ["capsule", "cylinder", "ellipsoid"])
def test_inertia_from_round_geoms_vs_voxels(gt):
    """Closed forms checked against a voxel integration of the same solid (fromto along x)."""
    r, h = 0.02, 0.03
    if gt == "ellipsoid":
        geom = "<geom type='ellipsoid' size='0.02 0.03 0.045'/>"
    else:
        geom = f"<geom type='{gt}' size='{r}' fromto='{-h} 0 0 {h} 0 0'/>"
    b = _one_body(geom)
    n = 160
    ext = 0.05
    g = (np.arange(n) + 0.5) / n * 2 * ext - ext
    X, Y, Z = np.meshgrid(g, g, g, indexing="ij")
    if gt == "capsule":
        xc = np.clip(X, -h, h)
        inside = (X - xc) ** 2 + Y ** 2 + Z ** 2 <= r * r
    elif gt == "cylinder":
        inside = (np.abs(X) <= h) & (Y ** 2 + Z ** 2 <= r * r)
    else:
        inside = (X / 0.02) ** 2 + (Y / 0.03) ** 2 + (Z / 0.045) ** 2 <= 1.0
    dv = (2 * ext / n) ** 3
    m = 1000.0 * dv * inside.sum()
    x, y, z = X[inside], Y[inside], Z[inside]
    rho = 1000.0 * dv
    I = rho * np.array([[np.sum(y * y + z * z), -np.sum(x * y), -np.sum(x * z)],
                        [-np.sum(x * y), np.sum(x * x + z * z), -np.sum(y * z)],
                        [-np.sum(x * z), -np.sum(y * z), np.sum(x * x + y * y)]])
    assert b["mass"] == pytest.approx(m, rel=1e-2)
    np.testing.assert_allclose(_tensor(b), I, rtol=2e-2, atol=1e-3 * np.trace(I))


def test_fullinertia_and_inertiafromgeom_modes():
    b = _one_body("<inertial mass='1' fullinertia='2 3 4 0.1 0.2 0.3'/>")
    np.testing.assert_allclose(_tensor(b), [[2, 0.1, 0.2], [0.1, 3, 0.3], [0.2, 0.3, 4]], rtol=1e-12, atol=1e-14)
    both = "<inertial mass='1' diaginertia='1 1 1'/><geom type='box' size='0.1 0.1 0.1' mass='2'/>"
    assert _one_body(both)["mass"] == 1.0
    assert _one_body(both, '<compiler angle="radian" inertiafromgeom="true"/>')["mass"] == 2.0
    with pytest.raises(ValueError, match="inertiafromgeom"):
        _one_body("<geom type='box' size='0.1 0.1 0.1'/>", '<compiler inertiafromgeom="false"/>')
    with pytest.raises(ValueError, match="mesh"):
        _one_body("<geom type='mesh' mesh='m'/>")
    # geoms outside inertiagrouprange carry no mass
    two = "<geom type='box' size='0.1 0.1 0.1' mass='2'/><geom type='box' size='0.1 0.1 0.1' mass='5' group='3'/>"
    assert _one_body(two)["mass"] == 7.0
    assert _one_body(two, '<compiler inertiagrouprange="0 2"/>')["mass"] == 2.0


def _actuated(mut) -> dict:
    root = ET.fromstring(to_mjcf(load_description()))
    mut(root)
    return load_mjcf(ET.tostring(root, encoding="unicode"))


def _motor(root, joint):
    return next(a for a in root.find("actuator") if a.get("joint") == joint)


def test_actuator_gear_and_ctrlrange():
    def mut(root):
        _motor(root, "right_knee_pitch").set("gear", "2")
        _motor(root, "left_hip_yaw").set("ctrlrange", "-1.5 2.5")
        a = _motor(root, "right_ankle_roll")
        del a.attrib["ctrlrange"]
        a.set("ctrllimited", "false")
        act = root.find("actuator")  # actuator order does not matter
        kids = list(act)
        for k in kids:
            act.remove(k)
        for k in reversed(kids):
            act.append(k)

    d = _actuated(mut)
    cm = compile_model(d)
    f = _fields(cm)
    ia = cm.joint_names.index
    assert f["act_gear"][ia("right_knee_pitch")] == 2.0
    assert list(f["act_ctrlrange"][ia("left_hip_yaw")]) == [-1.5, 2.5]
    assert f["act_ctrlrange"][ia("right_ankle_roll")][1] > 1e29
    base = compile_model(load_description())
    fb = _fields(base)
    for k in range(20):
        if k not in (ia("right_knee_pitch"), ia("left_hip_yaw"), ia("right_ankle_roll")):
            assert f["act_gear"][k] == fb["act_gear"][k] and list(f["act_ctrlrange"][k]) == list(fb["act_ctrlrange"][k])


@pytest.mark.parametrize("what,err", [("drop", "without an actuator"), ("position", "not supported"),
                                      ("twice", "more than one"), ("unknown", "not a hinge")])
def test_actuator_errors(what, err):
    def mut(root):
        act = root.find("actuator")
        a = _motor(root, "right_knee_pitch")
        if what == "drop":
            act.remove(a)
        elif what == "position":
            a.tag = "position"
        elif what == "twice":
            act.append(ET.fromstring('<motor joint="right_knee_pitch"/>'))
        else:
            a.set("joint", "nope")

    with pytest.raises(ValueError, match=err):
        _actuated(mut)


def test_colliders_are_parsed_and_unsupported_ones_reported():
    b = load_mjcf("<mujoco><worldbody><body name='b'><freejoint/><inertial mass='1' diaginertia='1 1 1'/>"
                  "<geom name='shin' type='capsule' size='0.01' fromto='0 0 0 0 0.06 -0.08'/>"
                  "<geom name='hand' type='sphere' size='0.02' pos='0.1 0 0'/>"
                  "<geom name='cyl' type='cylinder' size='0.01 0.05 0.3'/>"
                  "<geom name='ell' type='ellipsoid' size='0.01 0.02 0.03' fromto='0 0 0 0 0 -0.1'/>"
                  "<geom name='foot' type='hfield' hfield='m'/>"
                  "<geom name='vis' type='hfield' hfield='m' contype='0' conaffinity='0'/></body></worldbody></mujoco>")
    assert b["skipped_geoms"] == [{"name": "foot", "body": "b", "type": "hfield"}]
    shin, hand, cyl, ell = b["geoms"]
    # an ellipsoid with fromto: the two semi-axes across, the segment's half-length along
    np.testing.assert_allclose(ell["size"], [0.01, 0.02, 0.05])
    # a cylinder keeps its radius and half-length (MuJoCo's third size is unused)
    assert cyl == {"name": "cyl", "body": "b", "type": "cylinder", "size": [0.01, 0.05]}
    assert shin["type"] == "capsule" and hand == {"name": "hand", "body": "b", "type": "sphere", "size": [0.02],
                                                  "pos": [0.1, 0.0, 0.0]}
    # fromto: centre at the midpoint, half-length 0.05, local +z along the segment
    np.testing.assert_allclose(shin["size"], [0.01, 0.05])
    np.testing.assert_allclose(shin["pos"], [0.0, 0.03, -0.04])
    w, x, y, z = shin["quat"]
    zaxis = [2 * (x * z + w * y), 2 * (y * z - w * x), 1 - 2 * (x * x + y * y)]
    np.testing.assert_allclose(zaxis, [0.0, 0.6, -0.8], atol=1e-12)
    assert "skipped_geoms" not in load_mjcf(to_mjcf(load_description()))


def test_colliders_past_sixteen_are_reported():
    """Up to 16 floor colliders (model v9, ZB_MAX_GEOM); the overflow is listed as skipped."""
    geoms = "".join(f"<geom name='g{i}' type='box' size='0.01 0.01 0.01'/>" for i in range(18))
    b = load_mjcf("<mujoco><worldbody><body name='b'><freejoint/><inertial mass='1' diaginertia='1 1 1'/>"
                  f"{geoms}</body></worldbody></mujoco>")
    assert [g["name"] for g in b["geoms"]] == [f"g{i}" for i in range(16)]
    assert [g["name"] for g in b["skipped_geoms"]] == ["g16", "g17"]


def test_command_line_round_trip(tmp_path):
    import os
    import subprocess
    import sys

    from zbot_amd.model import DEFAULT_ASSET

    pkg_root = os.path.dirname(os.path.dirname(DEFAULT_ASSET))  # ksim-gym-zbot_amd/
    env = dict(os.environ, PYTHONPATH=pkg_root)
    xml, js = tmp_path / "z.xml", tmp_path / "z.json"
    subprocess.run([sys.executable, "-m", "zbot_amd.mjcf", DEFAULT_ASSET, str(xml)], check=True, env=env)
    subprocess.run([sys.executable, "-m", "zbot_amd.mjcf", str(xml), str(js)], check=True, env=env)
    _assert_same_model(compile_model(_tree_order(load_description())), compile_model(str(js)))


def test_missing_file_is_reported():
    with pytest.raises(FileNotFoundError):
        load_mjcf("/nonexistent/zbot.xml")


def test_skipped_colliders_are_rejected_by_zb_create():
    """A collider the engine has no floor contact for (a height field here; or a seventeenth collider) is not
    dropped silently: zb_create rejects the model (ZB_EMODEL, nskip_geom); compile_model(...,
    drop_colliders=True) drops it knowingly (missing item 3). Supported extra colliders
    (a capsule or, since round 4, a cylinder or an ellipsoid shin) pass validation."""
    import ctypes as C
    import xml.etree.ElementTree as ET

    from zbot_amd import compile_model, default_config
    from zbot_amd import engine as E

    def with_shin(gtype):
        root = ET.fromstring(to_mjcf(load_description()))
        for b in root.iter("body"):
            if "knee" in b.get("name"):
                shape = ('size="0.015 0.02 0.04" pos="0 0 -0.04"' if gtype == "ellipsoid"
                         else 'hfield="shin"' if gtype == "hfield" else 'size="0.015" fromto="0 0 0 0 0 -0.08"')
                b.append(ET.fromstring(f'<geom name="shin_col" type="{gtype}" {shape} mass="0" contype="1" '
                                       'conaffinity="0"/>'))
                break
        return load_mjcf(ET.tostring(root, encoding="unicode"))

    L = E.load_library()
    h = C.c_void_p()
    desc = with_shin("hfield")
    assert [g["name"] for g in desc["skipped_geoms"]] == ["shin_col"]
    cm = compile_model(desc)
    assert cm.cmodel.nskip_geom == 1
    rc = L.zb_create(C.byref(cm.cmodel), C.byref(default_config(solver="newton")), 4, 0, 0, 0, C.byref(h))
    assert rc == -4 and b"colliding geoms" in L.zb_last_error()
    for cm in (compile_model(desc, drop_colliders=True), compile_model(with_shin("capsule")),
               compile_model(with_shin("cylinder")), compile_model(with_shin("ellipsoid"))):
        assert cm.cmodel.nskip_geom == 0
        rc = L.zb_create(C.byref(cm.cmodel), C.byref(default_config(solver="newton")), 4, 0, 0, 0, C.byref(h))
        assert rc != -4, L.zb_last_error()  # validation passes (no device here: -2)
        if rc == 0:
            L.zb_destroy(h)
    assert compile_model(with_shin("capsule")).cmodel.ngeom == 3


def test_collider_sizes_beyond_the_type_are_ignored():
    """MuJoCo keeps three sizes per geom and ignores the ones a type does not use (a default class
    often sets all three): a sphere with size='0.05 0 0' is a sphere of radius 0.05; too few sizes
    for the type is an error."""
    b = load_mjcf("<mujoco><worldbody><body name='b'><freejoint/><inertial mass='1' diaginertia='1 1 1'/>"
                  "<geom name='s' type='sphere' size='0.05 0 0'/><geom name='c' type='capsule' size='0.01 0.04 0'/>"
                  "</body></worldbody></mujoco>")
    assert [g["size"] for g in b["geoms"]] == [[0.05], [0.01, 0.04]]
    with pytest.raises(ValueError, match="needs 3 sizes"):
        load_mjcf("<mujoco><worldbody><body name='b'><freejoint/><inertial mass='1' diaginertia='1 1 1'/>"
                  "<geom name='x' type='box' size='0.05 0.02'/></body></worldbody></mujoco>")


def test_touch_sensor_colliders_win_the_cap():
    """With more than sixteen colliders the touch sensors' geoms (the soles) are kept even when
    sixteen other colliders come first in the document; the overflow is listed as skipped."""
    geoms = "".join(f"<geom name='g{i}' type='sphere' size='0.01'/>" for i in range(16))
    b = load_mjcf("<mujoco><worldbody><body name='a'><freejoint/><inertial mass='1' diaginertia='1 1 1'/>"
                  f"{geoms}<body name='foot'><joint name='j' type='hinge'/><inertial mass='1' diaginertia='1 1 1'/>"
                  "<geom name='sole' type='box' size='0.02 0.03 0.005'/><site name='foot_site'/></body></body>"
                  "</worldbody><actuator><motor joint='j'/></actuator>"
                  "<sensor><touch site='foot_site'/></sensor></mujoco>")
    assert [g["name"] for g in b["geoms"]] == [f"g{i}" for i in range(15)] + ["sole"]
    assert [g["name"] for g in b["skipped_geoms"]] == ["g15"]
    assert [s.get("touch_geom") for s in b["sites"]] == ["sole"]


def _pairs_doc(body_geoms, extra="", option=""):
    """A free base with two hinged legs (thigh -> shin) and a jointless foot welded to each shin."""
    g = {k: body_geoms.get(k, "") for k in ("base", "lt", "ls", "lf", "rt", "rs", "rf")}
    inert = "<inertial mass='0.1' diaginertia='1e-4 1e-4 1e-4'/>"
    leg = ("<body name='{s}t' pos='0 {y} -0.05'><joint name='{s}hip' axis='0 1 0'/>" + inert + "{gt}"
           "<body name='{s}s' pos='0 0 -0.1'><joint name='{s}knee' axis='0 1 0'/>" + inert + "{gs}"
           "<body name='{s}f' pos='0 0 -0.1'>" + inert + "{gf}</body></body></body>")
    return ("<mujoco>" + option + "<worldbody><geom name='floor' type='plane' size='0 0 1'/>"
            "<body name='base' pos='0 0 0.3'><freejoint/>" + inert + g["base"]
            + leg.format(s="l", y=0.05, gt=g["lt"], gs=g["ls"], gf=g["lf"])
            + leg.format(s="r", y=-0.05, gt=g["rt"], gs=g["rs"], gf=g["rf"])
            + "</body></worldbody>" + extra + "</mujoco>")


def test_self_contact_pairs_follow_mujocos_filter():
    """The robot's own geom pairs MuJoCo collides (contype / conaffinity, weld bodies, the parent
    filter, <exclude>, <pair>) are listed in desc["self_pairs"]; the engine has floor contacts only."""
    from zbot_amd.mjcf import load_mjcf

    box = "<geom name='{n}' type='box' size='0.01 0.01 0.01'{a}/>"
    feet = {"lf": box.format(n="lfoot", a=""), "rf": box.format(n="rfoot", a="")}
    # default contype = conaffinity = 1: the two feet collide with each other
    d = load_mjcf(_pairs_doc(feet))
    assert d["self_pairs"] == [["lfoot", "rfoot"]]
    assert [g["name"] for g in d["geoms"]] == ["lfoot", "rfoot"]
    # contype 1 / conaffinity 0 on both: each still meets the floor (1 / 1), not each other
    floor_only = {k: box.format(n=n, a=" contype='1' conaffinity='0'") for k, n in (("lf", "lfoot"), ("rf", "rfoot"))}
    d = load_mjcf(_pairs_doc(floor_only))
    assert "self_pairs" not in d and len(d["geoms"]) == 2
    # <exclude> between the feet's bodies removes the pair; between their weld bodies (the shins:
    # the feet have no joint) it does not (the geoms' own bodies are matched)
    d = load_mjcf(_pairs_doc(feet, "<contact><exclude body1='lf' body2='rf'/></contact>"))
    assert "self_pairs" not in d
    d = load_mjcf(_pairs_doc(feet, "<contact><exclude body1='ls' body2='rs'/></contact>"))
    assert d["self_pairs"] == [["lfoot", "rfoot"]]
    # the parent filter: a shin geom and its thigh's geom never collide; the foot is welded to the
    # shin, so the foot and the thigh are a weld body and its parent too
    d = load_mjcf(_pairs_doc({"lt": box.format(n="lthigh", a=""), "lf": box.format(n="lfoot", a="")}))
    assert "self_pairs" not in d
    d = load_mjcf(_pairs_doc({"lt": box.format(n="lthigh", a=""), "lf": box.format(n="lfoot", a="")},
                             option="<option><flag filterparent='disable'/></option>"))
    assert d["self_pairs"] == [["lthigh", "lfoot"]]
    # a base geom and a shin geom (grandparent): a pair
    d = load_mjcf(_pairs_doc({"base": box.format(n="torso", a=""), "ls": box.format(n="lshin", a="")}))
    assert d["self_pairs"] == [["torso", "lshin"]]
    # contype 2 / conaffinity 2: not the floor's (1 / 1), so no floor contact, but each other's
    two = {k: box.format(n=n, a=" contype='2' conaffinity='2'") for k, n in (("lf", "lfoot"), ("rf", "rfoot"))}
    d = load_mjcf(_pairs_doc({**two, "base": box.format(n="torso", a=" contype='1' conaffinity='0'")}))
    assert [g["name"] for g in d["geoms"]] == ["torso"] and d["self_pairs"] == [["lfoot", "rfoot"]]
    # an explicit <pair> counts whatever the bits say
    d = load_mjcf(_pairs_doc(floor_only, "<contact><pair geom1='lfoot' geom2='rfoot'/></contact>"))
    assert d["self_pairs"] == [["lfoot", "rfoot"]]
    # ... even between visual-only geoms (contype = conaffinity = 0): MuJoCo still collides the pair
    vis = {k: box.format(n=n, a=" contype='0' conaffinity='0'") for k, n in (("lf", "lfoot"), ("rf", "rfoot"))}
    d = load_mjcf(_pairs_doc(vis, "<contact><pair geom1='lfoot' geom2='rfoot'/></contact>"))
    assert d["self_pairs"] == [["lfoot", "rfoot"]] and d["geoms"] == []
    d = load_mjcf(_pairs_doc(vis))
    assert "self_pairs" not in d


def test_self_contacts_are_rejected_by_zb_create():
    """A model whose own geoms collide with each other is simulated when the only pair is the two
    box soles (ZbModel.npair, the box-box kernels; round 5) and otherwise refused (ZB_EMODEL,
    nskip_pair) rather than simulated without those contacts; drop_self_contacts=True compiles it
    knowingly."""
    import ctypes as C
    import xml.etree.ElementTree as ET

    from zbot_amd import compile_model, default_config
    from zbot_amd import engine as E

    root = ET.fromstring(to_mjcf(load_description()))
    for g in root.iter("geom"):
        if g.get("name") in ("right_foot_sole", "left_foot_sole"):
            del g.attrib["conaffinity"]  # MuJoCo's default 1: the soles collide with each other
    desc = load_mjcf(ET.tostring(root, encoding="unicode"))
    assert desc["self_pairs"] == [["right_foot_sole", "left_foot_sole"]] or \
        desc["self_pairs"] == [["left_foot_sole", "right_foot_sole"]]
    L = E.load_library()
    h = C.c_void_p()
    cm = compile_model(desc)
    assert cm.cmodel.nskip_pair == 0 and cm.cmodel.npair == 1
    rc = L.zb_create(C.byref(cm.cmodel), C.byref(default_config(solver="newton")), 4, 0, 0, 0, C.byref(h))
    assert rc != -4, L.zb_last_error()
    if rc == 0:
        L.zb_destroy(h)
    # a second pair (a sole against a shin box that also touches the floor) is refused; the soles
    # pair itself stays simulated beside the floor colliders (ZB_XG 4, round 6)
    for b in root.iter("body"):
        if b.get("name") == "right_knee_pitch_link":
            b.append(ET.fromstring('<geom name="right_shin" type="box" size="0.015 0.02 0.05" pos="0 0 -0.05"/>'))
    desc = load_mjcf(ET.tostring(root, encoding="unicode"))
    assert len(desc["self_pairs"]) >= 2
    cm = compile_model(desc)
    assert cm.cmodel.nskip_pair == len(desc["self_pairs"]) - 1 and cm.cmodel.npair == 1
    rc = L.zb_create(C.byref(cm.cmodel), C.byref(default_config(solver="newton")), 4, 0, 0, 0, C.byref(h))
    assert rc == -4 and b"pairs of its own geoms" in L.zb_last_error()
    cm = compile_model(desc, drop_self_contacts=True)
    assert cm.cmodel.nskip_pair == 0 and cm.cmodel.npair == 0
    rc = L.zb_create(C.byref(cm.cmodel), C.byref(default_config(solver="newton")), 4, 0, 0, 0, C.byref(h))
    assert rc != -4, L.zb_last_error()
    if rc == 0:
        L.zb_destroy(h)
