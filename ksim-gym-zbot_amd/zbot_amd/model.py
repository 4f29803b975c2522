"""Robot descriptor compiler: JSON robot description -> ZbModel (include/zbot_model.h).

This is the build's stand-in for the part of MuJoCo's MJCF compiler that the
reference relies on (train.py:1326-1331: `mujoco_scenes.mjcf.load_mjmodel` +
`geom_priority[floor] = 2`). It runs once on the host, in float64, and produces:

  * the kinematic tree in the index order MuJoCo would use (bodies in
    definition order, dofs/qpos in body order);
  * inertias of each body from its box dimensions (`box`) and mass;
  * `qpos0` (joint zero) and the free-joint start height: the base is placed so
    the foot soles touch the floor in the JOINT_BIASES pose (the reset pose,
    train.py:1473) — the real MJCF's base height is unknown offline;
  * the constants MuJoCo's `mj_setConst` derives at qpos0 and the constraint
    model uses: `body_invweight0`, `dof_invweight0`, `stat.meaninertia`.

The real Z-Bot MJCF is network-fetched by the reference (train.py:1327) and is
unavailable here, so the default asset `assets/zbot_like.json` is a documented
Z-Bot-like stand-in.
"""

from __future__ import annotations

import json
import math
import os
from dataclasses import dataclass, field

import numpy as np

from . import cstructs as cs
from .constants import JOINT_BIASES

ASSET_DIR = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "assets")
DEFAULT_ASSET = os.path.join(ASSET_DIR, "zbot_like.json")


# --------------------------------------------------------------------------- #
# small float64 rigid-body helpers (host only)
# --------------------------------------------------------------------------- #
def quat_mul(a: np.ndarray, b: np.ndarray) -> np.ndarray:
    w1, x1, y1, z1 = a
    w2, x2, y2, z2 = b
    return np.array(
        [
            w1 * w2 - x1 * x2 - y1 * y2 - z1 * z2,
            w1 * x2 + x1 * w2 + y1 * z2 - z1 * y2,
            w1 * y2 - x1 * z2 + y1 * w2 + z1 * x2,
            w1 * z2 + x1 * y2 - y1 * x2 + z1 * w2,
        ]
    )


def quat_to_mat(q: np.ndarray) -> np.ndarray:
    w, x, y, z = q / np.linalg.norm(q)
    return np.array(
        [
            [1 - 2 * (y * y + z * z), 2 * (x * y - w * z), 2 * (x * z + w * y)],
            [2 * (x * y + w * z), 1 - 2 * (x * x + z * z), 2 * (y * z - w * x)],
            [2 * (x * z - w * y), 2 * (y * z + w * x), 1 - 2 * (x * x + y * y)],
        ]
    )


def axis_angle_quat(axis: np.ndarray, angle: float) -> np.ndarray:
    a = np.asarray(axis, dtype=np.float64)
    a = a / np.linalg.norm(a)
    s = math.sin(0.5 * angle)
    return np.array([math.cos(0.5 * angle), a[0] * s, a[1] * s, a[2] * s])


@dataclass
class Body:
    name: str
    parent: int
    pos: np.ndarray
    quat: np.ndarray
    mass: float
    ipos: np.ndarray
    inertia: np.ndarray
    iquat: np.ndarray = field(default_factory=lambda: np.array([1.0, 0.0, 0.0, 0.0]))  # inertial frame
    jnt_type: int = cs.JNT_NONE
    jnt_name: str = ""
    axis: np.ndarray = field(default_factory=lambda: np.zeros(3))
    jpos: np.ndarray = field(default_factory=lambda: np.zeros(3))
    jrange: tuple[float, float] | None = None
    servo: dict | None = None
    gear: float = 1.0  # actuator on this hinge (MJCF <motor gear ctrlrange>)
    ctrlrange: tuple[float, float] | None = None  # None: +-servo max_torque
    depth: int = 0
    dofadr: int = -1
    dofnum: int = 0
    qposadr: int = -1
    lastdof: int = -1


@dataclass
class CompiledModel:
    """Host-side view of the compiled model (float64) plus the packed ZbModel."""

    desc: dict
    bodies: list[Body]
    nq: int
    nv: int
    nu: int
    qpos0: np.ndarray
    dof_body: np.ndarray
    dof_parent: np.ndarray
    joint_names: list[str]
    geom_names: list[str]
    site_names: list[str]
    cmodel: cs.ZbModel

    @property
    def body_names(self) -> list[str]:
        return [b.name for b in self.bodies]

    def reset_qpos(self) -> np.ndarray:
        """qpos of the reset pose: base at qpos0, joints at JOINT_BIASES (train.py:1473)."""
        q = self.qpos0.copy()
        q[7:] = [b for _, b, _ in JOINT_BIASES]
        return q


# --------------------------------------------------------------------------- #
# kinematics / dynamics in float64 (used only to derive model constants)
# --------------------------------------------------------------------------- #
def _kinematics(bodies: list[Body], qpos: np.ndarray) -> tuple[list[np.ndarray], list[np.ndarray]]:
    xpos = [np.zeros(3) for _ in bodies]
    xmat = [np.eye(3) for _ in bodies]
    xquat = [np.array([1.0, 0, 0, 0]) for _ in bodies]
    for i, b in enumerate(bodies):
        if i == 0:
            continue
        p = b.parent
        if b.jnt_type == cs.JNT_FREE:
            xpos[i] = qpos[b.qposadr : b.qposadr + 3].copy()
            xquat[i] = qpos[b.qposadr + 3 : b.qposadr + 7] / np.linalg.norm(qpos[b.qposadr + 3 : b.qposadr + 7])
        else:
            xpos[i] = xpos[p] + xmat[p] @ b.pos
            xquat[i] = quat_mul(xquat[p], b.quat)
            if b.jnt_type == cs.JNT_HINGE:
                anchor = xpos[i] + quat_to_mat(xquat[i]) @ b.jpos
                xquat[i] = quat_mul(xquat[i], axis_angle_quat(b.axis, qpos[b.qposadr]))
                xpos[i] = anchor - quat_to_mat(xquat[i]) @ b.jpos
        xmat[i] = quat_to_mat(xquat[i])
    return xpos, xmat


def _point_jacobian(bodies: list[Body], xpos, xmat, nv: int, dof_body, body: int, point: np.ndarray):
    """Translational/rotational world Jacobians of a point fixed to `body`."""
    jp = np.zeros((3, nv))
    jr = np.zeros((3, nv))
    b = body
    while b > 0:
        bd = bodies[b]
        if bd.jnt_type == cs.JNT_FREE:
            for k in range(3):
                jp[:, bd.dofadr + k] = np.eye(3)[k]
                axis = xmat[b][:, k]
                jr[:, bd.dofadr + 3 + k] = axis
                jp[:, bd.dofadr + 3 + k] = np.cross(axis, point - xpos[b])
        elif bd.jnt_type == cs.JNT_HINGE:
            axis = xmat[b] @ bd.axis
            anchor = xpos[b] + xmat[b] @ bd.jpos
            jr[:, bd.dofadr] = axis
            jp[:, bd.dofadr] = np.cross(axis, point - anchor)
        b = bd.parent
    return jp, jr


def mass_matrix(bodies: list[Body], qpos: np.ndarray, nv: int, dof_body, armature: np.ndarray) -> np.ndarray:
    xpos, xmat = _kinematics(bodies, qpos)
    M = np.diag(armature.astype(np.float64))
    for i, b in enumerate(bodies):
        if i == 0 or b.mass <= 0:
            continue
        com = xpos[i] + xmat[i] @ b.ipos
        jp, jr = _point_jacobian(bodies, xpos, xmat, nv, dof_body, i, com)
        Ri = xmat[i] @ quat_to_mat(b.iquat)
        Iw = Ri @ np.diag(b.inertia) @ Ri.T
        M += b.mass * jp.T @ jp + jr.T @ Iw @ jr
    return M


# --------------------------------------------------------------------------- #
def _box_inertia(mass: float, box: list[float]) -> np.ndarray:
    lx, ly, lz = box
    return mass / 12.0 * np.array([ly * ly + lz * lz, lx * lx + lz * lz, lx * lx + ly * ly])


def load_description(path: str | None = None) -> dict:
    with open(path or DEFAULT_ASSET) as f:
        return json.load(f)


def mjx_box_vertices(size) -> list[list[float]]:
    """A box as MJX collides it with a plane: a convex mesh of its 8 corners in
    itertools.product((-1, 1), repeat=3) order (x slowest) [U: mjx/_src/mesh.py box()]."""
    return [[sx * size[0], sy * size[1], sz * size[2]] for sx in (-1, 1) for sy in (-1, 1) for sz in (-1, 1)]


def compile_model(desc: dict | str | None = None, drop_colliders: bool = False,
                  drop_self_contacts: bool = False, box_rule: str = "mujoco") -> CompiledModel:
    """Compile a JSON robot description into a ZbModel (+ host float64 view).

    A description from zbot_amd.mjcf.load_mjcf lists the source's colliding geoms the engine does
    not collide with the floor (it collides up to 16 boxes, capsules, cylinders, spheres, ellipsoids and convex meshes) in
    desc["skipped_geoms"]. They are counted into ZbModel.nskip_geom, and zb_create rejects such a
    model (ZB_EMODEL) rather than simulating it without those contacts. drop_colliders=True
    compiles it without them, knowingly (nskip_geom 0). Likewise desc["self_pairs"], the robot's
    own geom pairs the source model collides (the engine has floor contacts only), are counted
    into ZbModel.nskip_pair and refused by zb_create; drop_self_contacts=True compiles the model
    without them (nskip_pair 0).

    box_rule [U: which plane-box rule the reference's MJX uses; DESIGN.md §8]: "mujoco" (default)
    collides boxes by MuJoCo's mjc_PlaneBox (the corners below the centre within the margin);
    "mjx" compiles every box collider as the convex mesh of its 8 corners (mjx_box_vertices), so
    the engine collides it by MJX's plane_convex manifold (the mesh collider, XG 2 kernels). The
    sole pair (box-box) exists only under "mujoco"."""
    if desc is None or isinstance(desc, str):
        desc = load_description(desc)
    if box_rule not in ("mujoco", "mjx"):
        raise ValueError(f"box_rule {box_rule!r}: 'mujoco' or 'mjx'")
    if box_rule == "mjx":
        desc = dict(desc)
        desc["geoms"] = [dict({k: v for k, v in g.items() if k != "size"}, type="mesh", vert=mjx_box_vertices(g["size"]))
                         if g.get("type", "box") == "box" else g for g in desc.get("geoms", [])]

    # ---- bodies -----------------------------------------------------------
    bodies: list[Body] = [Body("world", -1, np.zeros(3), np.array([1.0, 0, 0, 0]), 0.0, np.zeros(3), np.zeros(3))]
    names = {"world": 0}
    servo_classes = desc.get("servo_classes", {})
    auto_z = False
    for bd in desc["bodies"]:
        if bd["parent"] not in names:
            raise ValueError(f"body {bd['name']}: parent {bd['parent']} must be defined before it")
        pos = list(bd["pos"])
        if pos[2] == "auto":
            auto_z = True
            pos[2] = 0.0
        b = Body(
            name=bd["name"],
            parent=names[bd["parent"]],
            pos=np.array(pos, dtype=np.float64),
            quat=np.array(bd.get("quat", [1.0, 0.0, 0.0, 0.0]), dtype=np.float64),
            mass=float(bd["mass"]),
            ipos=np.array(bd.get("ipos", [0.0, 0.0, 0.0]), dtype=np.float64),
            inertia=np.array(bd["inertia"], dtype=np.float64)
            if "inertia" in bd
            else _box_inertia(float(bd["mass"]), bd["box"]),
        )
        if "iquat" in bd:  # principal axes of the inertia (MJCF <inertial quat>)
            iq = np.array(bd["iquat"], dtype=np.float64)
            b.iquat = iq / np.linalg.norm(iq)
        j = bd.get("joint")
        if j is not None:
            b.jnt_name = j["name"]
            if j["type"] == "free":
                if b.parent != 0:
                    raise ValueError("free joint only allowed on a child of the world")
                b.jnt_type = cs.JNT_FREE
            elif j["type"] == "hinge":
                b.jnt_type = cs.JNT_HINGE
                b.axis = np.array(j["axis"], dtype=np.float64)
                b.axis /= np.linalg.norm(b.axis)
                b.jpos = np.array(j.get("pos", [0.0, 0.0, 0.0]), dtype=np.float64)
                b.jrange = tuple(j["range"]) if "range" in j else None
                b.servo = servo_classes[j["servo"]] if "servo" in j else None
                b.gear = float(j.get("gear", 1.0))
                b.ctrlrange = tuple(float(x) for x in j["ctrlrange"]) if "ctrlrange" in j else None
            else:
                raise ValueError(f"unsupported joint type {j['type']}")
        names[b.name] = len(bodies)
        bodies.append(b)

    nbody = len(bodies)
    if nbody > cs.MAX_BODY:
        raise ValueError(f"nbody={nbody} > {cs.MAX_BODY}")

    # ---- dofs / qpos ----------------------------------------------------------
    nq = nv = 0
    dof_body: list[int] = []
    dof_parent: list[int] = []
    for i, b in enumerate(bodies):
        if i == 0:
            continue
        b.depth = bodies[b.parent].depth + 1
        parent_last = bodies[b.parent].lastdof
        if b.jnt_type == cs.JNT_FREE:
            b.dofadr, b.dofnum, b.qposadr = nv, 6, nq
            for k in range(6):
                dof_body.append(i)
                dof_parent.append(parent_last if k == 0 else nv + k - 1)
            nv += 6
            nq += 7
        elif b.jnt_type == cs.JNT_HINGE:
            b.dofadr, b.dofnum, b.qposadr = nv, 1, nq
            dof_body.append(i)
            dof_parent.append(parent_last)
            nv += 1
            nq += 1
        b.lastdof = b.dofadr + b.dofnum - 1 if b.dofnum else parent_last
    if nv > cs.MAX_DOF or nq > cs.MAX_QPOS:
        raise ValueError(f"nv={nv}/nq={nq} exceed limits")

    dof_depth = np.zeros(nv, dtype=np.int64)
    for d in range(nv):
        dof_depth[d] = 0 if dof_parent[d] < 0 else dof_depth[dof_parent[d]] + 1
    max_depth = int(dof_depth.max()) + 1
    if max_depth > cs.MAX_DEPTH:
        raise ValueError(f"dof chain depth {max_depth} > {cs.MAX_DEPTH}")
    dof_anc = -np.ones((nv, cs.MAX_DEPTH), dtype=np.int64)
    for d in range(nv):
        a = d
        while a >= 0:
            dof_anc[d, dof_depth[a]] = a
            a = dof_parent[a]

    hinge_bodies = [b for b in bodies if b.jnt_type == cs.JNT_HINGE]
    joint_names = [b.jnt_name for b in hinge_bodies]
    nu = len(hinge_bodies)
    bias_names = [n for n, _, _ in JOINT_BIASES]
    if joint_names != bias_names:
        raise ValueError(
            "hinge joints must be defined in JOINT_BIASES order (train.py:61-82) so that "
            "ctrl order == qpos[7:] order (train.py:1252-1253, 1358-1359)"
        )

    armature = np.zeros(nv)
    damping = np.zeros(nv)
    frictionloss = np.zeros(nv)
    for b in hinge_bodies:
        s = b.servo or {}
        armature[b.dofadr] = s.get("armature", 0.0)
        damping[b.dofadr] = s.get("damping", 0.0)
        frictionloss[b.dofadr] = s.get("frictionloss", 0.0)

    # ---- qpos0 and base height ---------------------------------------------------
    qpos0 = np.zeros(nq)
    root = bodies[1]
    if root.jnt_type == cs.JNT_FREE:
        qpos0[0:3] = root.pos
        qpos0[3:7] = root.quat / np.linalg.norm(root.quat)

    geoms = desc.get("geoms", [])
    if len(geoms) > cs.MAX_GEOM:
        raise ValueError("too many collision geoms")
    # the touch sensors' geoms (the soles) first, then the others in document order: the engine
    # runs geoms 0-1 in its first contact-row bank and skips the second while it has no contacts
    # (DESIGN.md §4j), so the colliders that touch the floor all the time belong in the first
    touch = [sd["touch_geom"] for sd in desc.get("sites", []) if "touch_geom" in sd]
    geoms = sorted(geoms, key=lambda g: (0 if g["name"] in touch else 1))
    geom_names = [g["name"] for g in geoms]

    if auto_z:
        q = qpos0.copy()
        q[7:] = [v for _, v, _ in JOINT_BIASES]
        xpos, xmat = _kinematics(bodies, q)
        zmin = math.inf
        for g in geoms:
            bi = names[g["body"]]
            size = np.array(g.get("size", [0.0]))
            gpos = xpos[bi] + xmat[bi] @ np.array(g.get("pos", [0, 0, 0]))
            gmat = xmat[bi] @ quat_to_mat(np.array(g.get("quat", [1.0, 0, 0, 0])))
            gt = g.get("type", "box")
            if gt == "box":
                for sx in (-1, 1):
                    for sy in (-1, 1):
                        for sz in (-1, 1):
                            c = gpos + gmat @ (size * np.array([sx, sy, sz]))
                            zmin = min(zmin, c[2])
            elif gt == "capsule":
                for sg in (-1, 1):
                    zmin = min(zmin, gpos[2] + sg * size[1] * gmat[2, 2] - size[0])
            elif gt == "mesh":
                zmin = min(zmin, float((gpos[2] + np.asarray(g["vert"], np.float64) @ gmat[2, :]).min()))
            else:
                zmin = min(zmin, gpos[2] - size[0])
        qpos0[2] = -zmin + float(desc.get("base_clearance", 0.0))
        root.pos[2] = qpos0[2]

    # ---- mj_setConst equivalents at qpos0 ---------------------------------------
    M0 = mass_matrix(bodies, qpos0, nv, dof_body, armature)
    Minv = np.linalg.inv(M0)
    xpos0, xmat0 = _kinematics(bodies, qpos0)
    body_invweight = np.zeros((nbody, 2))
    for i in range(1, nbody):
        com = xpos0[i] + xmat0[i] @ bodies[i].ipos
        jp, jr = _point_jacobian(bodies, xpos0, xmat0, nv, dof_body, i, com)
        J = np.vstack([jp, jr])
        A = J @ Minv @ J.T
        body_invweight[i, 0] = np.trace(A[:3, :3]) / 3.0
        body_invweight[i, 1] = np.trace(A[3:, 3:]) / 3.0
    dof_invweight = np.diag(Minv).copy()
    if root.jnt_type == cs.JNT_FREE:  # MuJoCo averages free-joint dofs (trans / rot)
        dof_invweight[0:3] = dof_invweight[0:3].mean()
        dof_invweight[3:6] = dof_invweight[3:6].mean()
    meaninertia = float(np.trace(M0) / nv)

    # ---- pack ZbModel ------------------------------------------------------------
    m = cs.ZbModel()
    m.magic = cs.MODEL_MAGIC
    m.version = cs.MODEL_VERSION
    m.struct_bytes = C_sizeof(cs.ZbModel)
    m.nbody, m.nq, m.nv, m.nu = nbody, nq, nv, nu
    m.ngeom = len(geoms)
    m.nskip_geom = 0 if drop_colliders else len(desc.get("skipped_geoms", []))
    m.nskip_pair = 0  # set with the sole pair below
    m.max_depth = max_depth
    opt = desc.get("option", {})
    g = opt.get("gravity", [0.0, 0.0, -9.81])
    for k in range(3):
        m.gravity[k] = g[k]
    m.timestep = opt.get("timestep", 0.001)
    m.meaninertia = meaninertia

    for i, b in enumerate(bodies):
        m.body_parent[i] = b.parent
        m.body_depth[i] = b.depth
        m.body_jnttype[i] = b.jnt_type
        m.body_dofadr[i] = b.dofadr
        m.body_dofnum[i] = b.dofnum
        m.body_qposadr[i] = b.qposadr
        m.body_lastdof[i] = b.lastdof
        for k in range(3):
            m.body_pos[i][k] = b.pos[k]
            m.body_ipos[i][k] = b.ipos[k]
            m.body_inertia[i][k] = b.inertia[k]
            m.jnt_axis[i][k] = b.axis[k]
            m.jnt_pos[i][k] = b.jpos[k]
        for k in range(4):
            m.body_quat[i][k] = b.quat[k]
        for k in range(4):
            m.body_iquat[i][k] = b.iquat[k]
        m.body_mass[i][0] = b.mass
        m.body_invweight0[i][0] = body_invweight[i, 0]
        m.body_invweight0[i][1] = body_invweight[i, 1]
    # subtree masses
    sub = np.array([b.mass for b in bodies])
    for i in range(nbody - 1, 0, -1):
        sub[bodies[i].parent] += sub[i]
    for i in range(nbody):
        m.body_mass[i][1] = sub[i]

    for d in range(nv):
        m.dof_body[d] = dof_body[d]
        m.dof_parent[d] = dof_parent[d]
        m.dof_depth[d] = int(dof_depth[d])
        for e in range(cs.MAX_DEPTH):
            m.dof_anc[d][e] = int(dof_anc[d, e])
        m.dof_armature[d] = armature[d]
        m.dof_damping[d] = damping[d]
        m.dof_frictionloss[d] = frictionloss[d]
        m.dof_invweight0[d] = dof_invweight[d]
        m.dof_qposadr[d] = -1
    for d in range(nv, cs.MAX_DOF):
        m.dof_body[d] = -1
        m.dof_parent[d] = -1
        for e in range(cs.MAX_DEPTH):
            m.dof_anc[d][e] = -1
    for b in hinge_bodies:
        m.dof_qposadr[b.dofadr] = b.qposadr
        if b.jrange is not None:
            m.dof_limited[b.dofadr] = 1
            m.dof_range[b.dofadr][0] = b.jrange[0]
            m.dof_range[b.dofadr][1] = b.jrange[1]
    jc = desc.get("joint_constraint", {})
    sr = jc.get("solref", [0.02, 1.0])
    si = jc.get("solimp", [0.9, 0.95, 0.001, 0.5, 2.0])
    for k in range(2):
        m.dof_solref[k] = sr[k]
    for k in range(5):
        m.dof_solimp[k] = si[k]
    for k in range(nq):
        m.qpos0[k] = qpos0[k]

    for a, b in enumerate(hinge_bodies):
        s = b.servo or {}
        m.act_dof[a] = b.dofadr
        m.act_gear[a] = b.gear
        mt = s.get("max_torque", 1e6)
        cr = b.ctrlrange if b.ctrlrange is not None else (-mt, mt)
        m.act_ctrlrange[a][0] = cr[0]
        m.act_ctrlrange[a][1] = cr[1]
        m.fe_kp[a] = s.get("kp", 0.0)
        m.fe_kd[a] = s.get("kd", 0.0)
        m.fe_error_gain[a] = s.get("error_gain", 1.0)
        m.fe_max_pwm[a] = s.get("max_pwm", 1.0)
        m.fe_vin[a] = s.get("vin", 12.0)
        m.fe_kt[a] = s.get("kt", 1.0)
        m.fe_R[a] = s.get("R", 1.0)
        m.fe_vmax[a] = s.get("vmax", 5.0)
        m.fe_amax[a] = s.get("amax", 17.45)
        m.fe_max_torque[a] = mt
        m.fe_max_velocity[a] = s.get("max_velocity", 5.0)
        m.joint_bias[a] = JOINT_BIASES[a][1]
        m.joint_weight[a] = JOINT_BIASES[a][2]

    gtypes = {"box": (cs.GEOM_BOX, 3), "capsule": (cs.GEOM_CAPSULE, 2), "cylinder": (cs.GEOM_CYLINDER, 2),
              "sphere": (cs.GEOM_SPHERE, 1), "ellipsoid": (cs.GEOM_ELLIPSOID, 3), "mesh": (cs.GEOM_MESH, 0)}
    vadr = 0
    for gi, gd in enumerate(geoms):
        gt = gd.get("type", "box")
        if gt not in gtypes:
            raise ValueError(f"geom {gd['name']}: type {gt!r} (box, capsule, cylinder, sphere, ellipsoid and convex "
                             "mesh collide with the floor)")
        code, nsize = gtypes[gt]
        if gt == "mesh":
            # a convex mesh: its hull vertices in the geom frame, in the order MJX's plane_convex scans
            # them; geom_size[0] = the largest vertex distance from the geom origin (the second bank's
            # reach bound, zb_engine.hip contact_rows)
            vert = np.asarray(gd["vert"], dtype=np.float64).reshape(-1, 3)
            if not (1 <= len(vert) <= cs.MAX_MESHV) or not np.isfinite(vert).all():
                raise ValueError(f"geom {gd['name']}: a mesh collider needs 1 to {cs.MAX_MESHV} finite hull vertices "
                                 f"(has {len(vert)}; MJCF <mesh maxhullvert> can cap the hull)")
            if vadr + len(vert) > cs.MAX_MESHVERT:
                raise ValueError(f"geom {gd['name']}: the mesh colliders' hull vertices exceed the model's pool of "
                                 f"{cs.MAX_MESHVERT} (ZB_MAX_MESHVERT: {vadr} used before this geom, {len(vert)} more); "
                                 "cap the hulls with MJCF <mesh maxhullvert> or load_mjcf(maxhullvert=...)")
            m.geom_vertadr[gi] = vadr
            m.geom_vertnum[gi] = len(vert)
            for i, v in enumerate(vert):
                for k in range(3):
                    m.mesh_vert[vadr + i][k] = float(v[k])
            vadr += len(vert)
            m.geom_size[gi][0] = max(float(np.sqrt((np.float32(vert) ** 2).sum(axis=1)).max()), 1e-6) * (1 + 1e-6)
        elif len(gd["size"]) < nsize or any(not (v > 0) for v in gd["size"][:nsize]):
            raise ValueError(f"geom {gd['name']}: a {gt} needs {nsize} positive sizes")
        m.geom_body[gi] = names[gd["body"]]
        m.geom_type[gi] = code
        gp = gd.get("pos", [0, 0, 0])
        gq = gd.get("quat", [1.0, 0, 0, 0])
        for k in range(3):
            m.geom_pos[gi][k] = gp[k]
        for k in range(nsize):
            m.geom_size[gi][k] = gd["size"][k]
        for k in range(4):
            m.geom_quat[gi][k] = gq[k]
    fl = desc.get("floor", {})
    for k, v in enumerate(fl.get("friction", [1.0, 0.005, 0.0001])):
        m.floor_friction[k] = v
    for k, v in enumerate(fl.get("solref", [0.02, 1.0])):
        m.floor_solref[k] = v
    for k, v in enumerate(fl.get("solimp", [0.9, 0.95, 0.001, 0.5, 2.0])):
        m.floor_solimp[k] = v
    m.floor_margin = fl.get("margin", 0.0)

    sites = desc.get("sites", [])
    site_names = [s["name"] for s in sites]
    m.nsite = len(sites)
    for si_, sd in enumerate(sites):
        m.site_body[si_] = names[sd["body"]]
        sp = sd.get("pos", [0, 0, 0])
        sq = sd.get("quat", [1.0, 0, 0, 0])
        for k in range(3):
            m.site_pos[si_][k] = sp[k]
        for k in range(4):
            m.site_quat[si_][k] = sq[k]
    m.site_imu = site_names.index("imu_site")
    m.site_left_foot = site_names.index("left_foot")
    m.site_right_foot = site_names.index("right_foot")
    m.body_base = 1
    m.body_left_foot = names["Left_Foot"]
    m.body_right_foot = names["Right_Foot"]
    m.geom_left_foot = geom_names.index(sites[m.site_left_foot]["touch_geom"])
    m.geom_right_foot = geom_names.index(sites[m.site_right_foot]["touch_geom"])
    _compile_pairs(m, desc, geoms, geom_names, drop_self_contacts)

    _fill_tables(m, bodies, nbody, nv, dof_depth, dof_anc, dof_parent, [m.geom_body[g] for g in range(len(geoms))])

    if nu != cs.NJ or nbody != cs.NBODY_TASK:
        raise ValueError(f"the Z-Bot task layout needs nu=20, nbody=26 (got nu={nu}, nbody={nbody})")

    return CompiledModel(
        desc=desc,
        bodies=bodies,
        nq=nq,
        nv=nv,
        nu=nu,
        qpos0=qpos0,
        dof_body=np.array(dof_body),
        dof_parent=np.array(dof_parent),
        joint_names=joint_names,
        geom_names=geom_names,
        site_names=site_names,
        cmodel=m,
    )


def _fill_tables(m, bodies, nbody, nv, dof_depth, dof_anc, dof_parent, geom_body) -> None:
    """Derived topology tables consumed by the HIP engine (zbot_model.h)."""
    depth = [b.depth for b in bodies]
    m.max_body_depth = max(depth)
    if m.max_body_depth >= 16:
        raise ValueError("body depth must be < 16")
    for b in range(cs.MAX_BODY):
        for k in range(8):
            m.body_child[b][k] = -1
    maxch = [0] * 16
    for b in range(nbody):
        ch = [c for c in range(1, nbody) if bodies[c].parent == b]
        if len(ch) > 8:
            raise ValueError(f"body {bodies[b].name} has more than 8 children")
        m.body_nchild[b] = len(ch)
        for k, c in enumerate(ch):
            m.body_child[b][k] = c
        maxch[depth[b]] = max(maxch[depth[b]], len(ch))
    for d in range(16):
        m.depth_maxchild[d] = maxch[d]
    lastdof = [b.lastdof for b in bodies]
    glast = [lastdof[g] for g in geom_body]
    off = 0
    for d in range(nv):
        desc = 0
        for k in range(nv):
            if k != d and dof_depth[k] > dof_depth[d] and dof_anc[k, dof_depth[d]] == d:
                desc |= 1 << k
        m.dof_desc[d] = desc
        for w in range(4):
            v = 0
            for bb in range(4):
                e = 4 * w + bb
                a = int(dof_anc[d, e]) if e < cs.MAX_DEPTH else -1
                v |= (a if a >= 0 else 0) << (8 * bb)
            m.dof_ancpk[d][w] = v
        rm = 0
        for g, kd in enumerate(glast[:2]):  # geoms 0-1 (the engine's first row bank)
            if kd >= 0 and (kd == d or (desc >> kd) & 1):
                rm |= 0xFFFF << (16 * g)
        m.dof_rowmask[d] = rm
        m.dof_act[d] = -1
        m.dof_rowoff[d] = off
        off += 4 * ((int(dof_depth[d]) + 1 + 3) // 4)
    for d in range(nv, cs.MAX_DOF):
        m.dof_act[d] = -1
        m.dof_rowoff[d] = off
    for a in range(m.nu):
        m.dof_act[m.act_dof[a]] = a
    m.mrow_size = off
    for g, kd in enumerate(glast):
        m.geom_lastdof[g] = kd
    # elimination levels: height of each dof in the dof tree (leaves = 0)
    height = [0] * nv
    for d in range(nv - 1, -1, -1):  # children have larger indices than parents
        p = dof_parent[d]
        if p >= 0:
            height[p] = max(height[p], height[d] + 1)
    m.nlevel = max(height) + 1 if nv else 0
    if m.nlevel > cs.MAX_DEPTH:
        raise ValueError("too many elimination levels")
    for lv in range(cs.MAX_DEPTH):
        mem = [d for d in range(nv) if height[d] == lv]
        if len(mem) > 8:
            raise ValueError(f"elimination level {lv} has {len(mem)} dofs (max 8)")
        m.level_nmem[lv] = len(mem)
        for k in range(8):
            m.level_mem[lv][k] = mem[k] if k < len(mem) else -1


# MuJoCo's geom contact defaults (mjModel geom_friction / solref / solimp / margin)
GEOM_FRICTION = (1.0, 0.005, 0.0001)
GEOM_SOLREF = (0.02, 1.0)
GEOM_SOLIMP = (0.9, 0.95, 0.001, 0.5, 2.0)


def _compile_pairs(m, desc: dict, geoms: list, geom_names: list, drop: bool) -> None:
    """The robot's own colliding pairs (desc["self_pairs"]): the engine simulates the two box soles
    against each other (ZbModel.npair = 1; box-box), beside any other floor colliders (round 6: their
    rows in a bank of their own, the XG 4 kernels); any other pair is counted into nskip_pair, which
    zb_create refuses.
    drop=True: none of them (npair = nskip_pair = 0). The pair's parameters are MuJoCo's mix for two
    geoms of equal priority (mj_contactParam): friction the larger per component, solref / solimp the
    mean (solmix 1 each), margin the larger [U: MuJoCo's mixing rule restated from its documentation]."""
    m.npair = 0
    pairs = [] if drop else [list(p) for p in desc.get("self_pairs", [])]
    soles = {geom_names[m.geom_left_foot], geom_names[m.geom_right_foot]}
    by_name = {g["name"]: g for g in geoms}
    sole = [p for p in pairs if set(p) == soles]
    if sole and all(by_name[n].get("type", "box") == "box" for n in soles):
        g1, g2 = (geom_names.index(n) for n in sole[0])
        m.npair = 1
        m.pair_geom[0], m.pair_geom[1] = g1, g2
        a, b = by_name[sole[0][0]], by_name[sole[0][1]]
        fa, fb = a.get("friction", GEOM_FRICTION), b.get("friction", GEOM_FRICTION)
        for k in range(3):
            m.pair_friction[k] = max(float(fa[k]), float(fb[k]))
        ra, rb = a.get("solref", GEOM_SOLREF), b.get("solref", GEOM_SOLREF)
        for k in range(2):
            m.pair_solref[k] = 0.5 * (float(ra[k]) + float(rb[k]))
        ia, ib = a.get("solimp", GEOM_SOLIMP), b.get("solimp", GEOM_SOLIMP)
        for k in range(5):
            m.pair_solimp[k] = 0.5 * (float(ia[k]) + float(ib[k]))
        m.pair_margin = max(float(a.get("margin", 0.0)), float(b.get("margin", 0.0)))
        pairs = [p for p in pairs if set(p) != soles]
    m.nskip_pair = len(pairs)


def C_sizeof(t: type) -> int:  # noqa: N802
    import ctypes

    return ctypes.sizeof(t)
