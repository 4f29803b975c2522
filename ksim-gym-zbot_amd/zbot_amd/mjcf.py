"""MJCF <-> robot descriptor.

The reference builds its model from the K-Scale Z-Bot MJCF (train.py:1326-1331:
`ksim.get_mujoco_model_path("zbot")` + `mujoco_scenes.mjcf.load_mjmodel`, floor
`geom_priority = 2`) and reads the Feetech servo parameters from the K-Scale
metadata (train.py:1333-1338, 1340-1437). Both are network-fetched and absent
here, so the engine runs on the documented Z-Bot-like descriptor
(assets/zbot_like.json). This module lets an MJCF file take its place offline:

    desc = load_mjcf("zbot.xml", servo_classes=..., joint_servo=...)
    cm = compile_model(desc)               # -> ZbModel for zb_create

It reads the MJCF subset the engine's task topology uses, following MuJoCo's
MJCF semantics (XML reference, MuJoCo 3.3.4 [U]):
  * <compiler angle="degree|radian"> (MuJoCo's default is degree) and
    eulerseq (intrinsic "xyz" by default);
  * <default> classes, nested, applied through `class` / `childclass` with
    explicit attributes winning (joint: axis, range, armature, damping,
    frictionloss, pos; geom: type, size, pos, contype, conaffinity);
  * <body pos quat|euler|axisangle>, one <joint type="hinge"> or a
    <freejoint/> per body;
  * <inertial pos quat mass diaginertia|fullinertia>, or, without one (or with
    inertiafromgeom="true"), the mass and inertia of the body's box / sphere /
    capsule / cylinder / ellipsoid geoms (density or mass, fromto,
    inertiagrouprange), composed about their common centre of mass;
  * <asset><mesh> (inline `vertex`, or an STL / OBJ `file` under <compiler meshdir>,
    `scale`) for mesh <geom>s: a mesh collider is its convex hull (MuJoCo and MJX collide a mesh
    by its hull), its vertices in the geom frame in the file's order [U: MuJoCo re-centres a
    mesh on its centroid and principal axes; the hull is the same solid either way]; at most
    ZB_MAX_MESHV = 64 hull vertices (MJCF's maxhullvert can cap a hull);
  * box / capsule / cylinder / ellipsoid (size or fromto) / sphere / mesh <geom>s whose
    contype / conaffinity pass MuJoCo's test against the floor's
    ((ct1 & ca2) || (ct2 & ca1)) as floor colliders, up to 16 in document order
    (the engine's plane-box / -capsule / -cylinder / -sphere / -ellipsoid contacts;
    other such geoms are listed in desc["skipped_geoms"] and make zb_create refuse
    the model), the <geom type="plane"> of the worldbody as the floor (friction,
    solref, solimp, margin, contype, conaffinity);
  * the robot's own geom pairs MuJoCo would collide (self_pairs below): listed in
    desc["self_pairs"]; the engine has floor contacts only, so zb_create refuses
    such a model unless compiled with drop_self_contacts=True;
  * <motor> / plain <general> actuators (gear, ctrlrange, ctrllimited), one per
    hinge; <site>s and <touch> sensors; <option timestep gravity>.
The servo model (FeetechParams, train.py:1121-1134) is not part of MJCF: it
comes from `servo_classes` + `joint_servo` (joint -> class; by default the
joint's MJCF class when it names a servo class, else the Z-Bot-like
descriptor's assignment for that joint name). `to_mjcf` writes a descriptor
back out, so a descriptor and its MJCF compile to the same ZbModel
(tests/test_mjcf.py).
"""

from __future__ import annotations

import math
import os
import xml.etree.ElementTree as ET

import numpy as np

from .model import load_description

# floor colliders the engine has contacts for (type -> sizes) and how many (ZB_MAX_GEOM)
COLLIDER_TYPES = {"box": 3, "capsule": 2, "cylinder": 2, "sphere": 1, "ellipsoid": 3, "mesh": 0}
MAX_HULL_VERTS = 64  # ZB_MAX_MESHV
MAX_COLLIDERS = 16  # ZB_MAX_GEOM


def _floats(s: str | None, n: int | None = None) -> list[float] | None:
    if s is None:
        return None
    v = [float(x) for x in s.split()]
    if n is not None and len(v) != n:
        raise ValueError(f"expected {n} numbers, got {s!r}")
    return v


def _qmul(a, b):
    w1, x1, y1, z1 = a
    w2, x2, y2, z2 = b
    return [w1 * w2 - x1 * x2 - y1 * y2 - z1 * z2, w1 * x2 + x1 * w2 + y1 * z2 - z1 * y2,
            w1 * y2 - x1 * z2 + y1 * w2 + z1 * x2, w1 * z2 + x1 * y2 - y1 * x2 + z1 * w2]


def _axis_quat(axis, angle):
    a = np.asarray(axis, dtype=np.float64)
    a = a / np.linalg.norm(a)
    s = math.sin(angle / 2)
    return [math.cos(angle / 2), a[0] * s, a[1] * s, a[2] * s]


def _quat_mat(q):
    w, x, y, z = q
    return [[1 - 2 * (y * y + z * z), 2 * (x * y - w * z), 2 * (x * z + w * y)],
            [2 * (x * y + w * z), 1 - 2 * (x * x + z * z), 2 * (y * z - w * x)],
            [2 * (x * z - w * y), 2 * (y * z + w * x), 1 - 2 * (x * x + y * y)]]


def _mat_quat(R: np.ndarray) -> list[float]:
    t = R[0, 0] + R[1, 1] + R[2, 2]
    if t > 0:
        w = math.sqrt(1.0 + t) / 2
        q = [w, (R[2, 1] - R[1, 2]) / (4 * w), (R[0, 2] - R[2, 0]) / (4 * w), (R[1, 0] - R[0, 1]) / (4 * w)]
    else:
        i = int(np.argmax([R[0, 0], R[1, 1], R[2, 2]]))
        j, k = (i + 1) % 3, (i + 2) % 3
        r = math.sqrt(max(0.0, 1.0 + R[i, i] - R[j, j] - R[k, k]))
        v = [0.0, 0.0, 0.0]
        v[i] = r / 2
        v[j] = (R[j, i] + R[i, j]) / (2 * r)
        v[k] = (R[k, i] + R[i, k]) / (2 * r)
        q = [(R[k, j] - R[j, k]) / (2 * r)] + v
    if q[0] < 0:
        q = [-x for x in q]
    n = math.sqrt(sum(x * x for x in q))
    return [x / n for x in q]


def _principal(inertia: np.ndarray) -> tuple[list[float], list[float]]:
    """Principal moments and the frame holding them (MJCF diaginertia + inertial quat)."""
    off = abs(inertia[0, 1]) + abs(inertia[0, 2]) + abs(inertia[1, 2])
    if off <= 1e-14 * max(1e-300, float(np.trace(inertia))):
        return [float(inertia[k, k]) for k in range(3)], [1.0, 0.0, 0.0, 0.0]
    w, V = np.linalg.eigh(inertia)
    if np.linalg.det(V) < 0:
        V[:, 2] = -V[:, 2]
    return [float(x) for x in w], _mat_quat(V)


def _fromto_frame(ft: list[float]) -> tuple[np.ndarray, np.ndarray, float]:
    """Centre, rotation (local z along the segment) and half-length of a geom given by fromto,
    as MuJoCo's compiler sets them (mjuu_frame from the z axis: the shortest rotation of +z)."""
    ft = np.asarray(ft, dtype=np.float64)
    d = ft[3:] - ft[:3]
    L = float(np.linalg.norm(d))
    pos = (ft[:3] + ft[3:]) / 2
    z = d / L
    axis = np.cross([0.0, 0.0, 1.0], z)
    sn, cs_ = float(np.linalg.norm(axis)), float(z[2])
    if sn > 1e-12:
        R = np.array(_quat_mat(_axis_quat(axis, math.atan2(sn, cs_))))
    else:
        R = np.eye(3) if cs_ > 0 else np.diag([1.0, -1.0, -1.0])
    return pos, R, L / 2


def read_mesh_file(path: str) -> np.ndarray:
    """The vertices [n, 3] of an STL (binary or ASCII) or OBJ file, each distinct vertex once in the
    order it first appears (MuJoCo merges an STL's repeated face corners)."""
    with open(path, "rb") as f:
        data = f.read()
    ext = os.path.splitext(path)[1].lower()
    if ext == ".obj":
        pts = [[float(x) for x in ln.split()[1:4]] for ln in data.decode("utf-8", "replace").splitlines()
               if ln.startswith("v ")]
    elif ext == ".stl":
        ntri = int.from_bytes(data[80:84], "little") if len(data) >= 84 else -1
        if len(data) == 84 + 50 * ntri:  # binary: header, count, then normal + 3 corners + attribute per face
            rec = np.frombuffer(data[84:], dtype=np.dtype([("n", "<f4", 3), ("v", "<f4", (3, 3)), ("a", "<u2")]),
                                count=ntri)
            pts = rec["v"].reshape(-1, 3).astype(np.float64).tolist()
        else:
            pts = [[float(x) for x in ln.split()[1:4]] for ln in data.decode("utf-8", "replace").splitlines()
                   if ln.strip().startswith("vertex")]
    else:
        raise ValueError(f"mesh file {path}: STL or OBJ expected")
    if not pts:
        raise ValueError(f"mesh file {path}: no vertices")
    out, seen = [], set()
    for p in pts:
        key = tuple(p)
        if key not in seen:
            seen.add(key)
            out.append(p)
    return np.asarray(out, dtype=np.float64)


def hull_vertices(vert: np.ndarray, maxhullvert: int = -1) -> tuple[np.ndarray, np.ndarray]:
    """The convex hull of a point set: (its vertices in the input order, its triangles as indices into
    them). MuJoCo and MJX collide a mesh geom by this hull [U: MJX's vertex order]. maxhullvert > 3:
    MJCF's <mesh maxhullvert>, qhull stopped after that many vertices (MuJoCo passes qhull "TA" with
    maxhullvert - 4, the vertices added after the initial simplex) [U: the qhull version]."""
    from scipy.spatial import ConvexHull  # noqa: PLC0415

    vert = np.asarray(vert, dtype=np.float64).reshape(-1, 3)
    if len(vert) < 4:
        raise ValueError("a mesh needs at least 4 vertices")
    if maxhullvert != -1 and maxhullvert < 4:
        raise ValueError(f"maxhullvert {maxhullvert}: -1 or more than 3")
    h = ConvexHull(vert, qhull_options="Qt" + (f" TA{maxhullvert - 4}" if maxhullvert > 3 else ""))
    keep = np.sort(h.vertices)
    remap = {int(i): k for k, i in enumerate(keep)}
    tri = np.array([[remap[int(i)] for i in s] for s in h.simplices], dtype=np.int64)
    # orient every face outward (its normal away from the hull's centroid)
    v = vert[keep]
    cen = v.mean(axis=0)
    for t in tri:
        a, b, c = v[t[0]], v[t[1]], v[t[2]]
        if np.dot(np.cross(b - a, c - a), a - cen) < 0:
            t[1], t[2] = t[2], t[1]
    return v, tri


def _mesh_mass_props(v: np.ndarray, tri: np.ndarray):
    """(volume, centroid, inertia tensor per unit density about the centroid) of the closed solid
    with outward triangles tri over vertices v (signed tetrahedra from the origin)."""
    vol, c1, S = 0.0, np.zeros(3), np.zeros((3, 3))
    for t in tri:
        a, b, c = v[t[0]], v[t[1]], v[t[2]]
        dv = float(np.dot(a, np.cross(b, c))) / 6.0
        vol += dv
        c1 += dv * (a + b + c) / 4.0
        # second moments of the tetrahedron (0, a, b, c): dv / 20 (sum_i x_i x_i' + (sum_i x_i)(sum_i x_i)')
        s = a + b + c
        S += dv / 20.0 * (np.outer(a, a) + np.outer(b, b) + np.outer(c, c) + np.outer(s, s))
    if not vol > 0:
        raise ValueError("mesh volume must be positive")
    com = c1 / vol
    S = S - vol * np.outer(com, com)
    return vol, com, np.trace(S) * np.eye(3) - S


def _geom_mass_inertia(ga: dict, quat: list[float]):
    """(mass, centre, rotation, principal moments) of one solid geom, as MuJoCo's compiler
    takes it for inertiafromgeom: uniform density (default 1000) or the geom's explicit mass."""
    gt = ga.get("type", "sphere")
    if gt == "mesh":
        # the hull as a solid [U: MuJoCo's mesh inertia modes; "convex" is the hull's volume]
        hv, tri = hull_vertices(ga["_mesh_vert"], int(ga.get("_maxhullvert", -1)))
        vol, com, I1 = _mesh_mass_props(hv, tri)
        m = float(ga["mass"]) if "mass" in ga else float(ga.get("density", "1000")) * vol
        I = I1 * (m / vol)
        diag, iq = _principal(I)
        Rg = np.array(_quat_mat(quat))
        pos = np.array(_floats(ga.get("pos", "0 0 0"), 3)) + Rg @ com
        return m, pos, Rg @ np.array(_quat_mat(iq)), diag
    size = _floats(ga.get("size", "0 0 0"))
    pos = np.array(_floats(ga.get("pos", "0 0 0"), 3))
    R = np.array(_quat_mat(quat))
    if "fromto" in ga:
        if gt not in ("capsule", "cylinder", "box", "ellipsoid"):
            raise ValueError(f"geom {ga.get('name')}: fromto on a {gt}")
        pos, R, hl = _fromto_frame(_floats(ga["fromto"], 6))
        size = [size[0], hl] if gt in ("capsule", "cylinder") else [size[0], size[1], hl]
    if gt == "sphere":
        r = size[0]
        vol = 4.0 / 3.0 * math.pi * r ** 3

        def f(m):
            return [0.4 * m * r * r] * 3
    elif gt == "box":
        x, y, z = size[:3]
        vol = 8.0 * x * y * z

        def f(m):
            return [m / 3 * (y * y + z * z), m / 3 * (x * x + z * z), m / 3 * (x * x + y * y)]
    elif gt == "ellipsoid":
        a, b_, c = size[:3]
        vol = 4.0 / 3.0 * math.pi * a * b_ * c

        def f(m):
            return [m / 5 * (b_ * b_ + c * c), m / 5 * (a * a + c * c), m / 5 * (a * a + b_ * b_)]
    elif gt == "cylinder":
        r, h = size[0], size[1]
        vol = math.pi * r * r * 2 * h

        def f(m):
            return [m * (3 * r * r + 4 * h * h) / 12] * 2 + [m * r * r / 2]
    elif gt == "capsule":
        r, h = size[0], size[1]
        vcyl, vsph = math.pi * r * r * 2 * h, 4.0 / 3.0 * math.pi * r ** 3
        vol = vcyl + vsph

        def f(m):
            # cylinder about its centre + two solid hemispheres, each with its centroid 3r/8
            # beyond the cylinder's end and a transverse moment (83/320) m_h r^2 about it
            mc, hemi = m * vcyl / vol, m * vsph / vol / 2
            it = mc * (3 * r * r + 4 * h * h) / 12 + 2 * (83.0 / 320.0 * hemi * r * r + hemi * (h + 3 * r / 8) ** 2)
            return [it, it, mc * r * r / 2 + 2 * 0.4 * hemi * r * r]
    else:
        raise ValueError(f"geom {ga.get('name')}: inertia from a {gt} geom is not supported")
    m = float(ga["mass"]) if "mass" in ga else float(ga.get("density", "1000")) * vol
    return m, pos, R, f(m)


def _compose(parts):
    """Sum geom masses and inertias about the common centre of mass (parallel axes)."""
    M = sum(p[0] for p in parts)
    if M <= 0:
        raise ValueError("geom-derived body mass must be positive")
    com = sum(p[0] * p[1] for p in parts) / M
    inertia = np.zeros((3, 3))
    for m, pos, R, diag in parts:
        d = pos - com
        inertia += R @ np.diag(diag) @ R.T + m * (float(d @ d) * np.eye(3) - np.outer(d, d))
    diag, iq = _principal(inertia)
    return float(M), [float(x) for x in com], diag, iq


class _Defaults:
    """MJCF default classes: class name -> {element tag -> attributes}, inherited down the tree."""

    def __init__(self, root: ET.Element | None):
        self.cls: dict[str, dict[str, dict[str, str]]] = {"main": {}}
        if root is not None:
            self._walk(root, "main", {})

    def _walk(self, el: ET.Element, name: str, inherited: dict):
        own = {tag: dict(attrs) for tag, attrs in inherited.items()}
        for child in el:
            if child.tag != "default":
                own.setdefault(child.tag, {}).update(child.attrib)
        self.cls[name] = own
        for child in el:
            if child.tag == "default":
                self._walk(child, child.get("class", name), own)

    def attrs(self, el: ET.Element, cls: str) -> dict[str, str]:
        c = el.get("class", cls)
        if c not in self.cls:
            raise ValueError(f"unknown default class {c!r}")
        out = dict(self.cls[c].get(el.tag, {}))
        out.update(el.attrib)
        return out


def self_pairs(geoms: list[dict], parent: dict[str, str], welded: set[str], excludes: set[frozenset],
               explicit: list[tuple[str, str]] = (), filterparent: bool = True) -> list[list[str]]:
    """Robot geom pairs MuJoCo's collision filter passes (engine_collision_driver.c, as documented in
    the MJCF reference's "Contact" section): geoms g1, g2 with (contype1 & conaffinity2) or
    (contype2 & conaffinity1) nonzero, on different weld bodies (a body without a joint is welded to
    its parent), not a weld body and its weld parent (filterparent, unless the parent is the world),
    not <contact><exclude>-d (matched on the geoms' own bodies [U: MuJoCo's broadphase signature as
    remembered; matching the weld bodies instead would exclude more, so this side reports more
    pairs, never fewer]); plus the explicit <contact><pair>s. geoms: {"name", "body", "contype",
    "conaffinity"}; parent: body -> parent body; welded: bodies without a joint."""

    def weld(b):
        while b != "world" and b in welded:
            b = parent[b]
        return b

    out, seen = [], set()
    for i, g1 in enumerate(geoms):
        for g2 in geoms[i + 1:]:
            if not ((g1["contype"] & g2["conaffinity"]) or (g2["contype"] & g1["conaffinity"])):
                continue
            w1, w2 = weld(g1["body"]), weld(g2["body"])
            if w1 == w2:
                continue
            p1 = weld(parent[w1]) if w1 != "world" else "world"
            p2 = weld(parent[w2]) if w2 != "world" else "world"
            if filterparent and w1 != "world" and w2 != "world" and (w1 == p2 or w2 == p1):
                continue
            if frozenset((g1["body"], g2["body"])) in excludes:
                continue
            out.append([g1["name"], g2["name"]])
            seen.add(frozenset((g1["name"], g2["name"])))
    for a, b in explicit:
        if frozenset((a, b)) not in seen:
            out.append([a, b])
            seen.add(frozenset((a, b)))
    return out


def load_mjcf(src: str, servo_classes: dict | None = None, joint_servo: dict | None = None,
              base_clearance: float | None = None, template: dict | None = None,
              maxhullvert: int | None = None) -> dict:
    """Parse an MJCF file (path or XML text) into the descriptor compile_model() takes.

    template: descriptor supplying what MJCF does not hold (servo classes, the joint -> servo
    map, base clearance, constraint solref/solimp); default assets/zbot_like.json.
    maxhullvert: cap every mesh's hull at this many vertices where the file sets no smaller cap (as
    MJCF's <mesh maxhullvert>; e.g. 64, the engine's limit, to collide meshes whose full hull is
    larger, knowingly with a coarser hull)."""
    tmpl = template or load_description()
    if src.lstrip().startswith("<"):
        text = src
    elif os.path.exists(src):
        with open(src) as f:
            text = f.read()
    else:
        raise FileNotFoundError(f"MJCF file not found: {src}")
    root = ET.fromstring(text)
    if root.tag != "mujoco":
        raise ValueError("not an MJCF document (<mujoco> root expected)")
    comp = root.find("compiler")
    degree = (comp.get("angle", "degree") if comp is not None else "degree") == "degree"
    eulerseq = comp.get("eulerseq", "xyz") if comp is not None else "xyz"
    ang = (lambda v: v * math.pi / 180.0) if degree else (lambda v: v)
    fromgeom = comp.get("inertiafromgeom", "auto") if comp is not None else "auto"
    grp = [int(x) for x in comp.get("inertiagrouprange", "0 5").split()] if comp is not None else [0, 5]
    defaults = _Defaults(root.find("default"))
    meshdir = ""
    if comp is not None:
        meshdir = comp.get("meshdir", comp.get("assetdir", ""))
    base_dir = os.path.dirname(os.path.abspath(src)) if not src.lstrip().startswith("<") else os.getcwd()
    meshes: dict[str, np.ndarray] = {}
    mesh_cap: dict[str, int] = {}  # the hull's vertex cap per mesh (maxhullvert; -1 none)
    for asset in root.findall("asset"):
        for me in asset.findall("mesh"):
            ma = defaults.attrs(me, me.get("class", "main"))
            if "vertex" in ma:
                mv = np.array(_floats(ma["vertex"]), dtype=np.float64).reshape(-1, 3)
            elif "file" in ma:
                fp = ma["file"] if os.path.isabs(ma["file"]) else os.path.join(base_dir, meshdir, ma["file"])
                mv = read_mesh_file(fp)
            else:
                raise ValueError(f"mesh {ma.get('name')}: vertex or file needed")
            mv = mv * np.array(_floats(ma.get("scale", "1 1 1"), 3))
            mname = ma.get("name") or os.path.splitext(os.path.basename(ma["file"]))[0]
            meshes[mname] = mv
            cap = int(ma.get("maxhullvert", "-1"))
            if maxhullvert is not None and (cap == -1 or cap > maxhullvert):
                cap = int(maxhullvert)
            mesh_cap[mname] = cap
    flag = root.find("option/flag")
    filterparent = flag is None or flag.get("filterparent", "enable") != "disable"
    parent_of: dict[str, str] = {}
    welded: set[str] = set()
    colliding: list[dict] = []  # every robot geom with contype or conaffinity, for self_pairs
    robot_geoms: set[str] = set()  # every named robot geom, visual-only ones included (<contact><pair>)

    servo_classes = dict(servo_classes if servo_classes is not None else tmpl.get("servo_classes", {}))
    tmpl_servo = {b["joint"]["name"]: b["joint"].get("servo") for b in tmpl["bodies"] if "joint" in b}

    desc: dict = {
        "name": root.get("model", "mjcf"),
        "description": "imported from MJCF by zbot_amd.mjcf.load_mjcf",
        "option": {"timestep": 0.002, "gravity": [0.0, 0.0, -9.81]},
        "floor": dict(tmpl.get("floor", {})),
        "joint_constraint": dict(tmpl.get("joint_constraint", {})),
        "base_clearance": tmpl.get("base_clearance", 0.0) if base_clearance is None else base_clearance,
        "servo_classes": servo_classes,
        "bodies": [],
        "geoms": [],
        "sites": [],
    }
    opt = root.find("option")
    if opt is not None:
        if opt.get("timestep"):
            desc["option"]["timestep"] = float(opt.get("timestep"))
        if opt.get("gravity"):
            desc["option"]["gravity"] = _floats(opt.get("gravity"), 3)

    def orientation(el, attrs) -> list[float]:
        if "quat" in attrs:
            q = _floats(attrs["quat"], 4)
            n = math.sqrt(sum(x * x for x in q))
            return [x / n for x in q]
        if "axisangle" in attrs:
            v = _floats(attrs["axisangle"], 4)
            return _axis_quat(v[:3], ang(v[3]))
        if "euler" in attrs:
            e = [ang(x) for x in _floats(attrs["euler"], 3)]
            q = [1.0, 0.0, 0.0, 0.0]
            for ch, a in zip(eulerseq, e):
                axis = {"x": [1, 0, 0], "y": [0, 1, 0], "z": [0, 0, 1]}[ch.lower()]
                r = _axis_quat(axis, a)
                q = _qmul(q, r) if ch.islower() else _qmul(r, q)  # intrinsic (moving) vs extrinsic
            return q
        return [1.0, 0.0, 0.0, 0.0]

    def parse_body(el: ET.Element, parent: str, cls: str):
        cls = el.get("childclass", cls)
        name = el.get("name")
        if not name:
            raise ValueError("every body needs a name")
        b: dict = {"name": name, "parent": parent, "pos": _floats(el.get("pos", "0 0 0"), 3)}
        parent_of[name] = parent
        q = orientation(el, el.attrib)
        if q != [1.0, 0.0, 0.0, 0.0]:
            b["quat"] = q
        joints = [c for c in el if c.tag in ("joint", "freejoint")]
        if len(joints) > 1:
            raise ValueError(f"body {name}: one joint per body is supported (got {len(joints)})")
        if not joints:
            welded.add(name)
        for j in joints:
            ja = defaults.attrs(j, cls) if j.tag == "joint" else dict(j.attrib)
            jt = "free" if j.tag == "freejoint" else ja.get("type", "hinge")
            if jt == "free":
                b["joint"] = {"name": ja.get("name", name + "_free"), "type": "free"}
                continue
            if jt != "hinge":
                raise ValueError(f"joint {ja.get('name')}: type {jt} is not supported (hinge / free)")
            jd = {"name": ja["name"], "type": "hinge", "axis": _floats(ja.get("axis", "0 0 1"), 3)}
            if "pos" in ja:
                jd["pos"] = _floats(ja["pos"], 3)
            limited = ja.get("limited", "auto")
            if "range" in ja and limited != "false":
                jd["range"] = [ang(x) for x in _floats(ja["range"], 2)]
            servo = (joint_servo or {}).get(jd["name"])
            if servo is None and j.get("class", cls) in servo_classes:
                servo = j.get("class", cls)
            if servo is None:
                servo = tmpl_servo.get(jd["name"])
            if servo is not None:
                jd["servo"] = servo
            base = servo_classes.get(servo, {}) if servo else {}
            mj = {k: float(ja[k]) for k in ("armature", "damping", "frictionloss")
                  if k in ja and float(ja[k]) != float(base.get(k, 0.0))}
            if mj:  # MJCF joint dynamics that differ from the servo class's own values win
                key = f"{servo or 'mjcf'}@{jd['name']}"
                base = dict(servo_classes.get(servo, {})) if servo else {}
                base.update(mj)
                servo_classes[key] = base
                jd["servo"] = key
            b["joint"] = jd
        inert = el.find("inertial")
        if inert is not None and fromgeom != "true":
            b["mass"] = float(inert.get("mass"))
            b["ipos"] = _floats(inert.get("pos", "0 0 0"), 3)
            if inert.get("diaginertia"):
                b["inertia"] = _floats(inert.get("diaginertia"), 3)
                iq = orientation(inert, inert.attrib)
            elif inert.get("fullinertia"):
                xx, yy, zz, xy, xz, yz = _floats(inert.get("fullinertia"), 6)
                diag, iq = _principal(np.array([[xx, xy, xz], [xy, yy, yz], [xz, yz, zz]]))
                b["inertia"] = diag
            else:
                raise ValueError(f"body {name}: <inertial> needs diaginertia or fullinertia")
        elif fromgeom == "false":
            raise ValueError(f"body {name}: no <inertial> and inertiafromgeom is false")
        else:  # MuJoCo's inertiafromgeom: mass and inertia of the body's geoms at their density
            parts = []
            for c in el:
                if c.tag == "geom":
                    ga = defaults.attrs(c, cls)
                    if grp[0] <= int(ga.get("group", "0")) <= grp[1]:
                        if ga.get("type") == "mesh":
                            if ga.get("mesh") not in meshes:
                                raise ValueError(f"body {name}: geom of unknown mesh {ga.get('mesh')!r}")
                            ga = dict(ga, _mesh_vert=meshes[ga["mesh"]], _maxhullvert=mesh_cap[ga["mesh"]])
                        parts.append(_geom_mass_inertia(ga, orientation(c, ga)))
            if not parts:
                raise ValueError(f"body {name}: no <inertial> element and no geoms to infer it from")
            mass, com, diag, iq = _compose(parts)
            b["mass"], b["ipos"], b["inertia"] = mass, com, diag
        if iq != [1.0, 0.0, 0.0, 0.0]:
            b["iquat"] = iq
        desc["bodies"].append(b)
        for c in el:
            if c.tag == "geom":
                ga = defaults.attrs(c, cls)
                ct, ca = int(ga.get("contype", "1")), int(ga.get("conaffinity", "1"))
                if "name" in ga:
                    robot_geoms.add(ga["name"])
                if ct == 0 and ca == 0:
                    continue  # visual only (an explicit <pair> still collides it, below)
                gt = ga.get("type", "sphere")
                gname = ga.get("name", f"{name}_geom{len(colliding)}")
                colliding.append({"name": gname, "body": name, "type": gt, "contype": ct, "conaffinity": ca})
                if gt not in COLLIDER_TYPES:
                    # the engine collides boxes, capsules, cylinders, spheres and ellipsoids with the floor; other colliding
                    # geoms are listed so a caller can see what the model leaves out (the count cap,
                    # MAX_COLLIDERS, is applied after the touch sensors pick their geoms, below)
                    desc.setdefault("skipped_geoms", []).append({"name": gname, "body": name, "type": gt})
                    continue
                nsz = COLLIDER_TYPES[gt]
                gd = {"name": gname, "body": name, "type": gt}
                if gt == "mesh":
                    if ga.get("mesh") not in meshes:
                        raise ValueError(f"geom {gname}: unknown mesh {ga.get('mesh')!r}")
                    hv, _ = hull_vertices(meshes[ga["mesh"]], mesh_cap[ga["mesh"]])
                    if len(hv) > MAX_HULL_VERTS:
                        # the engine's plane-mesh contact scans at most 64 hull vertices
                        desc.setdefault("skipped_geoms", []).append(
                            {"name": gname, "body": name, "type": gt, "hull_vertices": len(hv)})
                        continue
                    gd["vert"] = [[float(x) for x in p] for p in hv]
                # contact parameters other than MuJoCo's defaults (the sole pair's mix, model.py)
                for key, nk in (("friction", 3), ("solref", 2), ("solimp", 5)):
                    if key in ga:
                        vals = _floats(ga[key])
                        dflt = {"friction": [1.0, 0.005, 0.0001], "solref": [0.02, 1.0],
                                "solimp": [0.9, 0.95, 0.001, 0.5, 2.0]}[key]
                        gd[key] = (vals + dflt[len(vals):])[:nk]
                if "margin" in ga:
                    gd["margin"] = float(ga["margin"])
                gq = orientation(c, ga)
                if gt == "mesh":
                    if "pos" in ga:
                        gd["pos"] = _floats(ga["pos"], 3)
                elif "fromto" in ga:
                    if gt == "sphere":
                        raise ValueError(f"geom {gd['name']}: fromto on a {gt} collider")
                    fpos, fR, hl = _fromto_frame(_floats(ga["fromto"], 6))
                    # the segment's half-length is the last size (capsule / cylinder: the second)
                    sz = _floats(ga["size"])
                    if len(sz) < nsz - 1:
                        raise ValueError(f"geom {gd['name']}: a {gt} with fromto needs {nsz - 1} sizes")
                    gd["size"] = sz[:nsz - 1] + [hl]
                    gd["pos"] = [float(v) for v in fpos]
                    gq = _mat_quat(fR)
                else:
                    # MuJoCo stores three sizes and ignores the ones a type does not use
                    sz = _floats(ga.get("size", ""))
                    if len(sz) < nsz:
                        raise ValueError(f"geom {gd['name']}: a {gt} needs {nsz} sizes, got {ga.get('size')!r}")
                    gd["size"] = sz[:nsz]
                    if "pos" in ga:
                        gd["pos"] = _floats(ga["pos"], 3)
                if gq != [1.0, 0.0, 0.0, 0.0]:
                    gd["quat"] = gq
                desc["geoms"].append(gd)
            elif c.tag == "site":
                sa = defaults.attrs(c, cls)
                sd = {"name": sa["name"], "body": name, "pos": _floats(sa.get("pos", "0 0 0"), 3)}
                sq = orientation(c, sa)
                if sq != [1.0, 0.0, 0.0, 0.0]:
                    sd["quat"] = sq
                desc["sites"].append(sd)
        for c in el:
            if c.tag == "body":
                parse_body(c, name, cls)

    wb = root.find("worldbody")
    if wb is None:
        raise ValueError("no <worldbody>")
    floor_ct = floor_ca = 1
    for c in wb:
        if c.tag == "body":
            parse_body(c, "world", c.get("childclass", "main"))
        elif c.tag == "geom":
            ga = defaults.attrs(c, "main")
            if ga.get("type") == "plane":
                floor_ct, floor_ca = int(ga.get("contype", "1")), int(ga.get("conaffinity", "1"))
                fl = desc["floor"]
                if "friction" in ga:
                    fr = _floats(ga["friction"])
                    fl["friction"] = (fr + [0.005, 0.0001][len(fr) - 1:])[:3] if len(fr) < 3 else fr
                for k in ("solref", "solimp"):
                    if k in ga:
                        fl[k] = _floats(ga[k])
                if "margin" in ga:
                    fl["margin"] = float(ga["margin"])
    # floor colliders are the geoms that pass the contype / conaffinity test against the floor
    touches_floor = {g["name"] for g in colliding
                     if (g["contype"] & floor_ca) or (floor_ct & g["conaffinity"])}
    desc["geoms"] = [g for g in desc["geoms"] if g["name"] in touches_floor]
    if "skipped_geoms" in desc:
        desc["skipped_geoms"] = [g for g in desc["skipped_geoms"] if g["name"] in touches_floor]
        if not desc["skipped_geoms"]:
            del desc["skipped_geoms"]
    # robot-robot pairs (the engine has none): <contact><exclude body1 body2> / <pair geom1 geom2>
    excludes, explicit = set(), []
    for ce in root.findall("contact"):
        for ex in ce.findall("exclude"):
            excludes.add(frozenset((ex.get("body1"), ex.get("body2"))))
        # MuJoCo collides an explicit pair whatever the geoms' contype / conaffinity
        for pr in ce.findall("pair"):
            if pr.get("geom1") in robot_geoms and pr.get("geom2") in robot_geoms:
                explicit.append((pr.get("geom1"), pr.get("geom2")))
    sp = self_pairs(colliding, parent_of, welded, excludes, explicit, filterparent)
    if sp:
        desc["self_pairs"] = sp
    # actuators: a motor (or gain-1 general actuator) per hinge; ctrl order is the joint order
    # the engine requires (JOINT_BIASES, train.py:61-82), whatever the actuator order here
    act = root.find("actuator")
    if act is not None:
        hinges = {b["joint"]["name"]: b["joint"] for b in desc["bodies"]
                  if b.get("joint", {}).get("type") == "hinge"}
        seen = set()
        for a in act:
            aa = defaults.attrs(a, "main")
            if a.tag not in ("motor", "general"):
                raise ValueError(f"actuator {aa.get('name')}: <{a.tag}> is not supported (motor / general)")
            if a.tag == "general" and (aa.get("biastype", "none") != "none"
                                       or _floats(aa.get("gainprm", "1"))[0] != 1.0):
                raise ValueError(f"actuator {aa.get('name')}: only a plain-gain general actuator is supported")
            jn = aa.get("joint")
            if jn not in hinges:
                raise ValueError(f"actuator {aa.get('name')}: joint {jn!r} is not a hinge of the model")
            if jn in seen:
                raise ValueError(f"joint {jn}: more than one actuator")
            seen.add(jn)
            jd = hinges[jn]
            gear = _floats(aa.get("gear", "1"))[0]
            if gear != 1.0:
                jd["gear"] = gear
            limited = aa.get("ctrllimited", "auto")
            mt = servo_classes.get(jd.get("servo"), {}).get("max_torque")
            if "ctrlrange" in aa and limited != "false":
                cr = _floats(aa["ctrlrange"], 2)
                if mt is None or cr != [-mt, mt]:
                    jd["ctrlrange"] = cr
            else:
                jd["ctrlrange"] = [-1e30, 1e30]  # unlimited: the servo's torque is not clamped
        missing = set(hinges) - seen
        if missing:
            raise ValueError(f"hinge joints without an actuator: {sorted(missing)}")
    # touch sensors (the TouchSensor foot zones, train.py:1511-1516) read the collision box on
    # the site's body; without a <sensor> section every site on a body with a box is a zone
    sens = root.find("sensor")
    touched = {t.get("site") for t in sens.iter("touch")} if sens is not None else None
    for sd in desc["sites"]:
        if touched is not None and sd["name"] not in touched:
            continue
        geom = next((g["name"] for g in desc["geoms"] if g["body"] == sd["body"]), None)
        if geom is not None:
            sd["touch_geom"] = geom
        elif touched is not None:
            raise ValueError(f"touch sensor on site {sd['name']}: no collider on body {sd['body']}")
    # at most MAX_COLLIDERS floor colliders: the touch sensors' geoms (the soles) first, then the
    # others in document order; the rest are listed as skipped (zb_create refuses such a model)
    touch = {sd["touch_geom"] for sd in desc["sites"] if "touch_geom" in sd}
    if len(touch) > MAX_COLLIDERS:
        raise ValueError(f"{len(touch)} touch-sensor colliders, the engine has contacts for {MAX_COLLIDERS}")
    room = MAX_COLLIDERS - len(touch)
    keep = []
    for g in desc["geoms"]:
        if g["name"] in touch:
            keep.append(g)
        elif room > 0:
            keep.append(g)
            room -= 1
        else:
            desc.setdefault("skipped_geoms", []).append({"name": g["name"], "body": g["body"], "type": g["type"]})
    desc["geoms"] = keep
    return desc


def _fmt(v) -> str:
    return " ".join(repr(float(x)) for x in v)


def to_mjcf(desc: dict) -> str:
    """Write a descriptor as MJCF (radians, one default class per servo class)."""
    lines = [f'<mujoco model="{desc.get("name", "zbot")}">', '  <compiler angle="radian"/>']
    opt = desc.get("option", {})
    lines.append(f'  <option timestep="{opt.get("timestep", 0.001)!r}" gravity="{_fmt(opt.get("gravity", [0, 0, -9.81]))}"/>')
    lines.append("  <default>")
    for cname, sc in desc.get("servo_classes", {}).items():
        attrs = " ".join(f'{k}="{float(sc[k])!r}"' for k in ("armature", "damping", "frictionloss") if k in sc)
        lines.append(f'    <default class="{cname}"><joint {attrs}/></default>')
    lines.append("  </default>")
    mesh_geoms = [g for g in desc.get("geoms", []) if g.get("type") == "mesh"]
    if mesh_geoms:
        lines.append("  <asset>")
        for g in mesh_geoms:  # the hull's vertices inline, one mesh asset per collider
            lines.append(f'    <mesh name="{g["name"]}_mesh" vertex="{_fmt(np.asarray(g["vert"]).ravel())}"/>')
        lines.append("  </asset>")
    lines.append("  <worldbody>")
    fl = desc.get("floor", {})
    fattr = " ".join(f'{k}="{_fmt(fl[k])}"' for k in ("friction", "solref", "solimp") if k in fl)
    lines.append(f'    <geom name="floor" type="plane" size="0 0 0.05" {fattr} margin="{float(fl.get("margin", 0.0))!r}"/>')
    root_z = None
    if any(b["pos"][2] == "auto" for b in desc["bodies"]):
        from .model import compile_model  # "auto" start height -> the compiled value

        root_z = float(compile_model(desc).qpos0[2])
    children: dict[str, list[dict]] = {}
    for b in desc["bodies"]:
        children.setdefault(b["parent"], []).append(b)
    geoms: dict[str, list[dict]] = {}
    for g in desc.get("geoms", []):
        geoms.setdefault(g["body"], []).append(g)
    sites: dict[str, list[dict]] = {}
    for s in desc.get("sites", []):
        sites.setdefault(s["body"], []).append(s)

    def body(b: dict, ind: str):
        pos = list(b["pos"])
        if pos[2] == "auto":
            pos[2] = root_z
        q = f' quat="{_fmt(b["quat"])}"' if "quat" in b else ""
        lines.append(f'{ind}<body name="{b["name"]}" pos="{_fmt(pos)}"{q}>')
        j = b.get("joint")
        if j is not None:
            if j["type"] == "free":
                lines.append(f'{ind}  <freejoint name="{j["name"]}"/>')
            else:
                cls = f' class="{j["servo"]}"' if "servo" in j else ""
                rng = f' range="{_fmt(j["range"])}"' if "range" in j else ""
                jp = f' pos="{_fmt(j["pos"])}"' if "pos" in j else ""
                lines.append(f'{ind}  <joint name="{j["name"]}" type="hinge"{cls} axis="{_fmt(j["axis"])}"{rng}{jp}/>')
        if "inertia" in b:
            di = b["inertia"]
        else:
            lx, ly, lz = b["box"]
            m = float(b["mass"])
            di = [m / 12 * (ly * ly + lz * lz), m / 12 * (lx * lx + lz * lz), m / 12 * (lx * lx + ly * ly)]
        iq = f' quat="{_fmt(b["iquat"])}"' if "iquat" in b else ""
        lines.append(f'{ind}  <inertial pos="{_fmt(b.get("ipos", [0, 0, 0]))}"{iq} mass="{float(b["mass"])!r}" '
                     f'diaginertia="{_fmt(di)}"/>')
        for g in geoms.get(b["name"], []):
            gp = f' pos="{_fmt(g["pos"])}"' if "pos" in g else ""
            gq = f' quat="{_fmt(g["quat"])}"' if "quat" in g else ""
            # contype 1 / conaffinity 0: the floor (1 / 1) collides with every collider and no two
            # colliders collide with each other, which is what the engine simulates
            shape = (f'mesh="{g["name"]}_mesh"' if g.get("type") == "mesh" else f'size="{_fmt(g["size"])}"')
            lines.append(f'{ind}  <geom name="{g["name"]}" type="{g.get("type", "box")}" {shape}{gp}{gq} '
                         f'contype="1" conaffinity="0"/>')
        for s in sites.get(b["name"], []):
            sq = f' quat="{_fmt(s["quat"])}"' if "quat" in s else ""
            lines.append(f'{ind}  <site name="{s["name"]}" pos="{_fmt(s.get("pos", [0, 0, 0]))}"{sq}/>')
        for c in children.get(b["name"], []):
            body(c, ind + "  ")
        lines.append(f"{ind}</body>")

    for b in children.get("world", []):
        body(b, "    ")
    lines.append("  </worldbody>")
    touch = [sd for sd in desc.get("sites", []) if "touch_geom" in sd]
    if touch:
        lines.append("  <sensor>")
        for sd in touch:
            lines.append(f'    <touch name="{sd["name"]}_touch" site="{sd["name"]}"/>')
        lines.append("  </sensor>")
    lines.append("  <actuator>")
    for b in desc["bodies"]:
        j = b.get("joint")
        if j is not None and j["type"] == "hinge":
            mt = desc.get("servo_classes", {}).get(j.get("servo"), {}).get("max_torque", 1e6)
            cr = j.get("ctrlrange", [-mt, mt])
            lines.append(f'    <motor name="{j["name"]}_ctrl" joint="{j["name"]}" gear="{float(j.get("gear", 1.0))!r}" '
                         f'ctrllimited="true" ctrlrange="{_fmt(cr)}"/>')
    lines.append("  </actuator>")
    lines.append("</mujoco>")
    return "\n".join(lines) + "\n"


if __name__ == "__main__":
    import argparse
    import json

    ap = argparse.ArgumentParser(description="convert between MJCF and the zbot_amd robot descriptor")
    ap.add_argument("src", help="an .xml (MJCF -> descriptor JSON) or .json (descriptor -> MJCF)")
    ap.add_argument("dst")
    a = ap.parse_args()
    if a.src.endswith(".json"):
        out = to_mjcf(load_description(a.src))
    else:
        out = json.dumps(load_mjcf(a.src), indent=1) + "\n"
    with open(a.dst, "w") as f:
        f.write(out)
