"""Floor colliders for the tests: three model variants with colliders beyond the box soles, an
independent numpy restatement of MuJoCo's plane-box / plane-capsule / plane-cylinder / plane-sphere /
plane-ellipsoid contact sets (engine_collision_primitive.c mjc_PlaneBox, mjc_PlaneCapsule,
mjc_PlaneCylinder, mjc_PlaneSphere, mjc_PlaneEllipsoid), and states whose colliders touch the floor. Test infrastructure only."""

from __future__ import annotations

import xml.etree.ElementTree as ET

import numpy as np


def _variant(edit) -> dict:
    from zbot_amd.mjcf import load_mjcf, to_mjcf
    from zbot_amd.model import load_description

    root = ET.fromstring(to_mjcf(load_description()))
    edit(root)
    return load_mjcf(ET.tostring(root, encoding="unicode"))


def limbs_desc() -> dict:
    """The soles plus a box on the right shin and a capsule on the left hand (4 colliders)."""

    def edit(root):
        for b in root.iter("body"):
            if b.get("name") == "right_knee_pitch_link":
                b.append(ET.fromstring('<geom name="right_shin" type="box" size="0.015 0.02 0.05" pos="0 0 -0.05" '
                                       'euler="0.2 0 0.1" contype="1" conaffinity="0"/>'))
            if b.get("name") == "left_gripper_roll_link":
                b.append(ET.fromstring('<geom name="left_hand" type="capsule" size="0.012" '
                                       'fromto="0 0 0 0.01 0.0 -0.06" contype="1" conaffinity="0"/>'))

    return _variant(edit)


def round_desc() -> dict:
    """Capsule feet (the touch sensors' zones) and a sphere on the head (3 colliders)."""

    def edit(root):
        for g in root.iter("geom"):
            if g.get("name") in ("right_foot_sole", "left_foot_sole"):
                g.set("type", "capsule")
                g.set("size", "0.01 0.035")
                g.set("pos", "0 0 0")
                g.set("quat", "0.7071067811865476 0 0.7071067811865476 0")
        for b in root.iter("body"):
            if b.get("name") == "head":
                b.append(ET.fromstring('<geom name="head_ball" type="sphere" size="0.05" pos="0 0 0.02" contype="1" '
                                       'conaffinity="0"/>'))

    return _variant(edit)


def cyl_desc() -> dict:
    """A cylinder right foot (the touch sensor's zone, axis vertical when the foot is flat), the box
    left sole, a tilted cylinder on the left shin and a tilted ellipsoid on the right hand
    (4 colliders)."""

    def edit(root):
        for g in root.iter("geom"):
            if g.get("name") == "right_foot_sole":
                g.set("type", "cylinder")
                g.set("size", "0.03 0.006")
        for b in root.iter("body"):
            if b.get("name") == "left_knee_pitch_link":
                b.append(ET.fromstring('<geom name="left_shin" type="cylinder" size="0.018" '
                                       'fromto="0 0 -0.02 0.01 0.005 -0.09" contype="1" conaffinity="0"/>'))
            if b.get("name") == "right_gripper_roll_link":
                b.append(ET.fromstring('<geom name="right_hand" type="ellipsoid" size="0.012 0.02 0.035" '
                                       'pos="0 0 -0.03" euler="0.3 -0.2 0.5" contype="1" conaffinity="0"/>'))

    return _variant(edit)


def _jitter(v, seed, amp=0.0004) -> np.ndarray:
    """Every vertex moved by up to amp per axis (a fixed draw): MJX's manifold selection breaks exact
    ties (a flat face's parallel edges, a symmetric solid's equal distances) by the rounding of the
    implementation, which a test against the oracle cannot pin; a generic hull has none."""
    return np.asarray(v, np.float64) + np.random.default_rng(seed).uniform(-amp, amp, size=np.shape(v))


def chamfered_sole(hx=0.045, hy=0.025, hz=0.005) -> np.ndarray:
    """A sole box (the box sole's size) whose bottom corners are cut, 16 hull vertices (top corners,
    the side edges' lower ends 3 mm up, the bottom face an octagon with cuts of 3 / 4.5 mm along x
    and 3.5 / 5 mm along y by side), jittered by up to 0.4 mm."""
    cx, cy = {-1: 0.003, 1: 0.0045}, {-1: 0.0035, 1: 0.005}
    v = []
    for sx in (-1, 1):
        for sy in (-1, 1):
            v.append([sx * hx, sy * hy, hz])
            v.append([sx * hx, sy * hy, -hz + 0.003])
            v.append([sx * (hx - cx[sx]), sy * hy, -hz])
            v.append([sx * hx, sy * (hy - cy[sy]), -hz])
    return _jitter(v, 3)


def icosahedron(r=0.022) -> np.ndarray:
    """The 12 vertices of an icosahedron of circumradius r, flattened 20 % along z."""
    p = (1 + 5 ** 0.5) / 2
    v = []
    for a in (-1, 1):
        for b in (-p, p):
            v += [[0, a, b], [a, b, 0], [b, 0, a]]
    v = np.array(v, np.float64)
    v = v / np.linalg.norm(v[0]) * r
    v[:, 2] *= 0.8
    return _jitter(v, 4)


def mesh_desc() -> dict:
    """Convex mesh colliders (round 5): a chamfered right sole (16 hull vertices, the touch sensor's
    zone) beside the left box sole, a flattened icosahedron on the right shin and a cube mesh on the
    left hand (4 colliders; both contact-row banks hold a mesh)."""

    def fmt(v):
        return " ".join(repr(float(x)) for x in np.asarray(v).ravel())

    def edit(root):
        asset = ET.SubElement(root, "asset")
        ET.SubElement(asset, "mesh", name="sole_mesh", vertex=fmt(chamfered_sole()))
        ET.SubElement(asset, "mesh", name="ico_mesh", vertex=fmt(icosahedron()))
        cube = _jitter(np.array([[sx, sy, sz] for sx in (-1, 1) for sy in (-1, 1) for sz in (-1, 1)])
                       * [0.012, 0.015, 0.02], 5)
        ET.SubElement(asset, "mesh", name="cube_mesh", vertex=fmt(cube))
        root.remove(asset)
        root.insert(1, asset)
        for g in root.iter("geom"):
            if g.get("name") == "right_foot_sole":
                g.set("type", "mesh")
                g.set("mesh", "sole_mesh")
                del g.attrib["size"]
        for b in root.iter("body"):
            if b.get("name") == "right_knee_pitch_link":
                b.append(ET.fromstring('<geom name="right_shin" type="mesh" mesh="ico_mesh" pos="0 0 -0.05" '
                                       'euler="0.2 0 0.1" contype="1" conaffinity="0"/>'))
            if b.get("name") == "left_gripper_roll_link":
                b.append(ET.fromstring('<geom name="left_hand" type="mesh" mesh="cube_mesh" pos="0 0 -0.03" '
                                       'euler="0.3 -0.2 0.5" contype="1" conaffinity="0"/>'))

    return _variant(edit)


def many_desc() -> dict:
    """Nine floor colliders (model v9): the box soles, shin boxes, thigh capsules, a hand capsule, a
    hand cube mesh and a head sphere. The engine's second bank takes, per substep, the first two of
    the seven others within reach of the floor."""

    def fmt(v):
        return " ".join(repr(float(x)) for x in np.asarray(v).ravel())

    def edit(root):
        asset = ET.Element("asset")
        cube = _jitter(np.array([[sx, sy, sz] for sx in (-1, 1) for sy in (-1, 1) for sz in (-1, 1)])
                       * [0.012, 0.015, 0.02], 6)
        ET.SubElement(asset, "mesh", name="hand_mesh", vertex=fmt(cube))
        root.insert(1, asset)
        extra = {
            "right_knee_pitch_link": '<geom name="right_shin" type="box" size="0.015 0.02 0.05" pos="0 0 -0.05" '
                                     'euler="0.2 0 0.1" contype="1" conaffinity="0"/>',
            "left_knee_pitch_link": '<geom name="left_shin" type="box" size="0.015 0.02 0.05" pos="0 0 -0.05" '
                                    'euler="-0.1 0.1 0" contype="1" conaffinity="0"/>',
            "right_hip_yaw_link": '<geom name="right_thigh" type="capsule" size="0.02" fromto="0 0 0 0 0.005 -0.07" '
                                  'contype="1" conaffinity="0"/>',
            "left_hip_yaw_link": '<geom name="left_thigh" type="capsule" size="0.02" fromto="0 0 0 0 -0.005 -0.07" '
                                 'contype="1" conaffinity="0"/>',
            "left_gripper_roll_link": '<geom name="left_hand" type="capsule" size="0.012" '
                                      'fromto="0 0 0 0.01 0.0 -0.06" contype="1" conaffinity="0"/>',
            "right_gripper_roll_link": '<geom name="right_hand" type="mesh" mesh="hand_mesh" pos="0 0 -0.03" '
                                       'contype="1" conaffinity="0"/>',
            "head": '<geom name="head_ball" type="sphere" size="0.05" pos="0 0 0.02" contype="1" conaffinity="0"/>',
        }
        for b in root.iter("body"):
            if b.get("name") in extra:
                b.append(ET.fromstring(extra[b.get("name")]))

    return _variant(edit)


def bank2_candidates(cm, qpos, margin=0.0) -> list[int]:
    """The geoms (index in the compiled model's order, >= 2) that the engine's second-bank selection
    finds within reach of the floor at qpos (zb_engine.hip select_bank2's bound, float64)."""
    from zbot_amd.model import _kinematics

    m = cm.cmodel
    xpos, _ = _kinematics(cm.bodies, np.asarray(qpos, np.float64))
    out = []
    for g in range(2, m.ngeom):
        s = [float(m.geom_size[g][k]) for k in range(3)]
        ty = int(m.geom_type[g])
        from zbot_amd import cstructs as cs

        rb = {cs.GEOM_BOX: np.sqrt(s[0] ** 2 + s[1] ** 2 + s[2] ** 2), cs.GEOM_CAPSULE: s[0] + s[1],
              cs.GEOM_CYLINDER: np.sqrt(s[0] ** 2 + s[1] ** 2), cs.GEOM_ELLIPSOID: max(s)}.get(ty, s[0])
        gp = np.array([float(m.geom_pos[g][k]) for k in range(3)])
        if xpos[m.geom_body[g]][2] - np.linalg.norm(gp) - rb <= margin + 1e-3:
            out.append(g)
    return out


def mjx_box_desc() -> dict:
    """The default robot with its box soles collided as MJX does (compile_model(box_rule="mjx"): each
    box a convex mesh of its 8 corners, MJX's plane_convex manifold), as a descriptor."""
    from zbot_amd.model import load_description, mjx_box_vertices

    d = load_description()
    d["geoms"] = [dict({k: v for k, v in g.items() if k != "size"}, type="mesh", vert=mjx_box_vertices(g["size"]))
                  for g in d["geoms"]]
    return d


def plane_convex(c, R, vert) -> list[tuple[np.ndarray, float]]:
    """MJX's plane_convex with _manifold_points against the floor z = 0 (numpy, float64; the
    oracle's plane_mesh states the rule): the four manifold points (a, b, c, d) as (vertex in the
    world, distance), repeats at distance 1."""
    vert = np.asarray(vert, np.float64)
    n = R.T @ np.array([0.0, 0.0, 1.0])
    p = R.T @ (np.zeros(3) - c)
    support = (p - vert) @ n
    mask = support > max(0.0, support.max() - 1e-3)
    dm = np.where(mask, 0.0, -1e6)
    ia = int(np.argmax(dm))
    a = vert[ia]
    ib = int(np.argmax(((a - vert) ** 2).sum(axis=1) + dm))
    b = vert[ib]
    ab = np.cross(n, a - b)
    ap = a - vert
    ic = int(np.argmax(np.abs(ap @ ab) + dm))
    cc = vert[ic]
    ac, bc = np.cross(n, a - cc), np.cross(n, b - cc)
    dist_bp = np.abs((b - vert) @ bc) + dm
    dist_ap = np.abs(ap @ ac) + dm
    idx = [ia, ib, ic, int(np.argmax(np.concatenate([dist_bp, dist_ap])) % len(vert))]
    out = []
    for q, i in enumerate(idx):
        d = -support[i] if i not in idx[:q] else 1.0
        out.append((c + R @ vert[i], float(d)))
    return out


def _qmat(q) -> np.ndarray:
    w, x, y, z = np.asarray(q, np.float64) / np.linalg.norm(q)
    return np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - w * z), 2 * (x * z + w * y)],
                     [2 * (x * y + w * z), 1 - 2 * (x * x + z * z), 2 * (y * z - w * x)],
                     [2 * (x * z - w * y), 2 * (y * z + w * x), 1 - 2 * (x * x + y * y)]])


def geom_frames(cm, qpos) -> list[tuple[str, np.ndarray, np.ndarray, list[float]]]:
    """(type, world centre, world rotation, size) of each collider at qpos (float64)."""
    from zbot_amd.model import _kinematics

    xpos, xmat = _kinematics(cm.bodies, np.asarray(qpos, np.float64))
    names = cm.body_names
    out = []
    for g in cm.desc["geoms"]:
        b = names.index(g["body"])
        c = xpos[b] + xmat[b] @ np.asarray(g.get("pos", [0.0, 0.0, 0.0]))
        R = xmat[b] @ _qmat(g.get("quat", [1.0, 0.0, 0.0, 0.0]))
        out.append((g.get("type", "box"), c, R, list(g["vert"]) if g.get("type") == "mesh" else list(g["size"])))
    return out


def _corner(sz, i) -> np.ndarray:
    return np.array([sz[0] if i & 1 else -sz[0], sz[1] if i & 2 else -sz[1], sz[2] if i & 4 else -sz[2]])


def box_corners(c, R, sz, margin=0.0) -> list[tuple[int, float]]:
    """mjc_PlaneBox: (corner index, distance) of the corners in index order whose offset along the
    normal is <= 0 and whose distance is within the margin, at most 4."""
    out = []
    for i in range(8):
        w = R @ _corner(sz, i)
        d = c[2] + w[2]
        if d > margin or w[2] > 0:
            continue
        out.append((i, float(d)))
        if len(out) == 4:
            break
    return out


def cylinder_points(c, R, sz, margin=0.0) -> list[tuple[np.ndarray, float]]:
    """mjc_PlaneCylinder against the floor z = 0: the axis turned toward the plane (a, scaled to the
    half-length), the radius vector v in the disk planes pointing down the slope (the geom's x axis
    when the disks are parallel to the plane); the near disk's deepest point c + v + a, which must
    be within the margin for any contact, the far disk's c + v - a, and the near disk's two points
    120 degrees from the first, c + a - v/2 +- sqrt(3)/2 r (v x a)/|v x a|."""
    r, h = sz[0], sz[1]
    a = R[:, 2].copy()
    if a[2] > 0:
        a = -a
    n = np.array([0.0, 0.0, 1.0])
    v = a * a[2] - n
    ln = np.linalg.norm(v)
    v = R[:, 0] * r if ln < 1e-15 else v * (r / ln)
    a = a * h
    pts = [c + v + a]
    if pts[0][2] > margin:
        return []
    out = [(pts[0], float(pts[0][2]))]
    far = c + v - a
    if far[2] <= margin:
        out.append((far, float(far[2])))
    w = np.cross(v, a)
    w = w / np.linalg.norm(w) * r * np.sqrt(3.0) / 2
    for sg in (1.0, -1.0):
        q = c + a - 0.5 * v + sg * w
        if q[2] <= margin:
            out.append((q, float(q[2])))
    return out


def ellipsoid_point(c, R, sz) -> tuple[np.ndarray, float]:
    """mjc_PlaneEllipsoid against the floor z = 0: the support point along -n, R (-s .* sn / |sn|)
    with sn = s .* (R' n)."""
    s = np.asarray(sz[:3], np.float64)
    sn = s * R[2, :]
    p = c + R @ (-s * sn / np.linalg.norm(sn))
    return p, float(p[2])


def contacts(cm, qpos, margin=0.0) -> list[list[tuple[np.ndarray, float]]]:
    """Per collider, its floor contacts (point, distance) by MuJoCo's rules: box corners in index
    order (bit 0 x, 1 y, 2 z) below the centre along the normal and within the margin, at most 4;
    capsule end spheres (+end first); sphere."""
    out = []
    for ty, c, R, sz in geom_frames(cm, qpos):
        cons = []
        if ty == "box":
            cons = [(c + R @ _corner(sz, i), d) for i, d in box_corners(c, R, sz, margin)]
        elif ty == "capsule":
            for sg in (1.0, -1.0):
                e = c + sg * sz[1] * R[:, 2]
                d = e[2] - sz[0]
                if d <= margin:
                    cons.append((e, d))
        elif ty == "cylinder":
            cons = cylinder_points(c, R, sz, margin)
        elif ty == "ellipsoid":
            p, d = ellipsoid_point(c, R, sz)
            if d <= margin:
                cons.append((p, d))
        elif ty == "mesh":
            cons = [(p, d) for p, d in plane_convex(c, R, sz) if d <= margin]
        else:
            d = c[2] - sz[0]
            if d <= margin:
                cons.append((c, d))
        out.append(cons)
    return out


def lowest_point(cm, qpos) -> float:
    """The lowest point of every collider at qpos (box corners, capsule / sphere surfaces)."""
    z = np.inf
    for ty, c, R, sz in geom_frames(cm, qpos):
        if ty == "box":
            for i in range(8):
                loc = np.array([sz[0] if i & 1 else -sz[0], sz[1] if i & 2 else -sz[1], sz[2] if i & 4 else -sz[2]])
                z = min(z, c[2] + (R @ loc)[2])
        elif ty == "capsule":
            z = min(z, c[2] - sz[1] * abs(R[2, 2]) - sz[0])
        elif ty == "cylinder":
            # the lowest rim point: half-length along the axis plus the radius across it
            z = min(z, c[2] - sz[1] * abs(R[2, 2]) - sz[0] * np.sqrt(max(0.0, 1.0 - R[2, 2] ** 2)))
        elif ty == "ellipsoid":
            z = min(z, ellipsoid_point(c, R, sz)[1])
        elif ty == "mesh":
            z = min(z, float((c[2] + np.asarray(sz) @ R[2, :]).min()))
        else:
            z = min(z, c[2] - sz[0])
    return float(z)


def touching_states(cm, n, seed, depth=0.003) -> np.ndarray:
    """[n, 27] qpos: a random base orientation (uniform over rotations, half the envs tipped onto a
    side within 45 degrees of horizontal), the joints at JOINT_BIASES + N(0, 0.3) inside their
    ranges, and the base height that puts the lowest collider point U(0, depth) below the floor."""
    from zbot_amd.constants import JOINT_BIASES

    rng = np.random.default_rng(seed)
    out = np.zeros((n, 27))
    lo, hi = np.full(20, -np.inf), np.full(20, np.inf)
    for b in cm.bodies:
        if b.jnt_type == 3 and b.jrange is not None:
            lo[b.qposadr - 7], hi[b.qposadr - 7] = b.jrange
    for e in range(n):
        q = cm.reset_qpos().astype(np.float64)
        if e % 2:
            # lying: a random heading, pitched or rolled 45..135 degrees
            yaw, tilt, ax = rng.uniform(-np.pi, np.pi), rng.uniform(np.pi / 4, 3 * np.pi / 4), rng.integers(2)
            qy = np.array([np.cos(yaw / 2), 0, 0, np.sin(yaw / 2)])
            qt = np.array([np.cos(tilt / 2), np.sin(tilt / 2) * (ax == 0), np.sin(tilt / 2) * (ax == 1), 0])
            w1, x1, y1, z1 = qy
            w2, x2, y2, z2 = qt
            quat = np.array([w1 * w2 - x1 * x2 - y1 * y2 - z1 * z2, w1 * x2 + x1 * w2 + y1 * z2 - z1 * y2,
                             w1 * y2 - x1 * z2 + y1 * w2 + z1 * x2, w1 * z2 + x1 * y2 - y1 * x2 + z1 * w2])
        else:
            quat = rng.normal(size=4)
        q[3:7] = quat / np.linalg.norm(quat)
        q[7:] = np.clip(np.array([b for _, b, _ in JOINT_BIASES]) + rng.normal(scale=0.3, size=20), lo, hi)
        q[2] = 0.0
        q[2] = -lowest_point(cm, q) - rng.uniform(0.0, depth)
        out[e] = q
    return out


# ---- the sole pair (the two box soles against each other; ZbModel.npair, round 5) ----

def sole_pair_desc() -> dict:
    """The default robot whose two soles collide with each other (MuJoCo's default contype /
    conaffinity 1 on both): desc["self_pairs"] holds the one pair, compile_model makes it npair 1."""
    from zbot_amd.model import load_description

    d = load_description()
    d["self_pairs"] = [["left_foot_sole", "right_foot_sole"]]
    return d


# hip roll offsets (right +, left -) at which the soles cross each other (oracle: 2-4 contacts)
CROSS_ROLL = (0.19, 0.41)


def crossing_states(cm, n: int, seed: int, air: bool = True) -> np.ndarray:
    """qpos [n, 27] with the legs rolled inward until the soles interpenetrate (CROSS_ROLL), small
    joint perturbations; air=True lifts the base to 1 m (no floor contact), else the reset height."""
    rng = np.random.default_rng(seed)
    q0 = cm.reset_qpos().astype(np.float64)
    out = np.repeat(q0[None], n, 0)
    rr = rng.uniform(*CROSS_ROLL, size=n)
    out[:, 7 + 1] += rr  # right_hip_roll
    out[:, 7 + 7] -= rr  # left_hip_roll
    out[:, 7:] += rng.normal(0, 0.01, size=(n, 20))
    if air:
        out[:, 2] = 1.0
    return out


def limbs_pair_desc() -> dict:
    """The limbs model (soles + right shin box + left hand capsule) whose two soles also collide with
    each other (round 6: the sole pair beside other floor colliders, the XG 4 kernels)."""
    d = limbs_desc()
    d["self_pairs"] = [["left_foot_sole", "right_foot_sole"]]
    return d


def many_pair_desc() -> dict:
    """The nine-collider model (many_desc) whose two soles also collide with each other (round 6: the
    XG 4 kernels with the second bank picked per substep)."""
    d = many_desc()
    d["self_pairs"] = [["left_foot_sole", "right_foot_sole"]]
    return d


def crossing_touching_states(cm, n: int, seed: int, depth=0.003) -> np.ndarray:
    """qpos [n, 27] with the legs crossed as in crossing_states (the soles interpenetrate) and the
    robot on the floor: even envs standing at the reset height, odd envs lying (a random heading,
    pitched or rolled 45..135 degrees, as touching_states) with the lowest collider point U(0, depth)
    below the floor, so that the shin or hand colliders touch it while the soles cross."""
    rng = np.random.default_rng(seed + 1000)
    out = crossing_states(cm, n, seed, air=False)
    for e in range(1, n, 2):
        yaw, tilt, ax = rng.uniform(-np.pi, np.pi), rng.uniform(np.pi / 4, 3 * np.pi / 4), rng.integers(2)
        qy = np.array([np.cos(yaw / 2), 0, 0, np.sin(yaw / 2)])
        qt = np.array([np.cos(tilt / 2), np.sin(tilt / 2) * (ax == 0), np.sin(tilt / 2) * (ax == 1), 0])
        w1, x1, y1, z1 = qy
        w2, x2, y2, z2 = qt
        quat = np.array([w1 * w2 - x1 * x2 - y1 * y2 - z1 * z2, w1 * x2 + x1 * w2 + y1 * z2 - z1 * y2,
                         w1 * y2 - x1 * z2 + y1 * w2 + z1 * x2, w1 * z2 + x1 * y2 - y1 * x2 + z1 * w2])
        out[e, 3:7] = quat / np.linalg.norm(quat)
        out[e, 2] = 0.0
        out[e, 2] = -lowest_point(cm, out[e]) - rng.uniform(0.0, depth)
    return out
