"""ctypes wrapper of the CPU oracle (TEST INFRASTRUCTURE ONLY).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import
this module; the product path (zbot_amd.engine) never does.
"""

from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
_LIBS: dict[str, C.CDLL] = {}


def build(force: bool = False) -> None:
    """Compile the oracle libraries with the committed Makefile."""
    targets = [os.path.join(HERE, n) for n in ("liboracle_zbot.so", "liboracle_zbot_f64.so", "liboracle_ppo.so",
                                               "liboracle_policy.so")]
    if force or not all(os.path.exists(t) for t in targets):
        subprocess.run(["make", "-C", HERE, "-s"], check=True)


def lib(precision: str = "f32") -> C.CDLL:
    """precision: "f32" (the twin), "f64" (accuracy reference) or "flops" (the fp32 twin with
    counted arithmetic, zbo_flops_get / zbo_flops_reset; scripts/count_flops.py)."""
    name = {"f32": "liboracle_zbot.so", "f64": "liboracle_zbot_f64.so", "flops": "liboracle_flops.so"}[precision]
    if name in _LIBS:
        return _LIBS[name]
    path = os.path.join(HERE, name)
    if precision == "flops":
        subprocess.run(["make", "-C", HERE, "-s", name], check=True)
    elif not os.path.exists(path):
        build()
    L = C.CDLL(path)
    fp = C.POINTER(C.c_float)
    u8p = C.POINTER(C.c_uint8)
    i32p = C.POINTER(C.c_int32)
    L.zbo_threefry2x32.argtypes = [C.c_uint32] * 4 + [C.POINTER(C.c_uint32)]
    L.zbo_reset.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_uint64, fp, fp, u8p, fp, fp, fp]
    L.zbo_step.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_uint64, fp, fp, fp, fp, fp, fp, fp, fp,
                           u8p, u8p, C.c_float, fp, i32p]
    L.zbo_forward_debug.argtypes = [C.c_void_p, C.c_void_p, fp, fp, fp, fp, fp, fp, fp, fp, fp, fp,
                                    C.POINTER(C.c_int), fp]
    L.zbo_simulate.argtypes = [C.c_void_p, C.c_void_p, fp, fp, fp, fp, C.c_int]
    L.zbo_constraint_debug.argtypes = [C.c_void_p, C.c_void_p, fp, fp, fp, fp, fp, fp, fp, fp, fp, fp, fp, fp,
                                       C.POINTER(C.c_int)]
    L.zbo_constraint_debug.restype = C.c_int
    L.zbo_trapezoidal_step.argtypes = [fp, fp, fp, C.c_float, fp, fp, C.c_int, fp, fp]
    L.zbo_rotate_quat_by_quat.argtypes = [fp, fp, C.c_int, fp]
    L.zbo_feetech.argtypes = [C.c_void_p, C.c_float, fp, fp, fp, fp, fp, fp, fp, fp]
    L.zbo_synthetic_actions.argtypes = [C.c_void_p, C.c_uint64, C.c_int, C.c_int, C.c_uint32, C.c_float, fp]
    L.zbo_field_offset.argtypes = [C.c_int, C.c_char_p]
    L.zbo_field_offset.restype = C.c_long
    L.zbo_struct_bytes.argtypes = [C.c_int]
    L.zbo_box_box.argtypes = [fp, fp, fp, fp, fp, fp, C.c_float, fp, fp, fp]
    L.zbo_box_box.restype = C.c_int
    L.zbo_plane_mesh.argtypes = [fp, C.c_int, fp, fp, C.c_float, C.POINTER(C.c_int32), fp, fp]
    L.zbo_plane_mesh.restype = C.c_int
    L.zbo_struct_bytes.restype = C.c_size_t
    L.zbo_set_clearance_out.argtypes = [fp]
    L.zbo_contact_count.argtypes = [C.c_void_p, C.c_void_p, fp, fp]
    L.zbo_contact_count.restype = C.c_int
    if precision == "flops":
        L.zbo_flops_get.argtypes = [C.POINTER(C.c_uint64)]
        L.zbo_flops_reset.argtypes = []
    _LIBS[name] = L
    return L


def _p(a: np.ndarray | None, t=C.c_float):
    if a is None:
        return None
    assert a.flags["C_CONTIGUOUS"]
    return a.ctypes.data_as(C.POINTER(t))


def threefry2x32(k0: int, k1: int, c0: int, c1: int) -> tuple[int, int]:
    out = (C.c_uint32 * 2)()
    lib().zbo_threefry2x32(k0 & 0xFFFFFFFF, k1 & 0xFFFFFFFF, c0 & 0xFFFFFFFF, c1 & 0xFFFFFFFF, out)
    return out[0], out[1]


def trapezoidal_step(pos, vel, target, dt, vmax, amax):
    pos, vel, target, vmax, amax = (np.ascontiguousarray(x, dtype=np.float32) for x in (pos, vel, target, vmax, amax))
    n = pos.shape[0]
    npos = np.zeros(n, np.float32)
    nvel = np.zeros(n, np.float32)
    lib().zbo_trapezoidal_step(_p(pos), _p(vel), _p(target), dt, _p(vmax), _p(amax), n, _p(npos), _p(nvel))
    return npos, nvel


def feetech(cmodel, dt, plan_pos, plan_vel, action, q, qd):
    arrs = [np.ascontiguousarray(x, dtype=np.float32) for x in (plan_pos, plan_vel, action, q, qd)]
    n = cmodel.nu
    npos, nvel, tau = np.zeros(n, np.float32), np.zeros(n, np.float32), np.zeros(n, np.float32)
    lib().zbo_feetech(C.byref(cmodel), dt, *[_p(a) for a in arrs], _p(npos), _p(nvel), _p(tau))
    return npos, nvel, tau


def rotate_quat_by_quat(q, r, inverse=False):
    q = np.ascontiguousarray(q, dtype=np.float32)
    r = np.ascontiguousarray(r, dtype=np.float32)
    out = np.zeros(4, np.float32)
    lib().zbo_rotate_quat_by_quat(_p(q), _p(r), int(inverse), _p(out))
    return out


def synthetic_actions(cmodel, seed: int, n: int, env_offset: int, t: int, std: float = 0.05) -> np.ndarray:
    a = np.zeros((n, 20), dtype=np.float32)
    lib().zbo_synthetic_actions(C.byref(cmodel), seed, n, env_offset, t, std, _p(a))
    return a


def feet_airtime_traj(contact, done, carry, ctrl_dt: float = 0.02, touchdown_penalty: float = 0.3):
    """FeetAirtimeReward.get_reward_stateful over one trajectory, as ksim evaluates it after the
    rollout (train.py:503-546; stand_still_threshold=None as registered at train.py:1559-1564).

    contact [T, n, 2] bool (touch > 0.1, train.py:516-517), done [T, n] bool, carry [n, 2] float32
    (the airtime carry, initial_carry zeros, train.py:499-501) -> (reward [T, n], carry' [n, 2]).
    float32 throughout, the operations in the reference's order:
      _airtime_sequence (:503-513): scan new = where(contact | done, 0, air + ctrl_dt)
      touchdown (:526-528): c & ~concatenate([False], c[:-1])   -- prev = False at t = 0
      (:533-539): (roll(air, 1) - penalty) * touchdown, left + right -- row 0 reads air[T-1]
    """
    f32 = np.float32
    contact = np.asarray(contact, dtype=bool)
    done = np.asarray(done, dtype=bool)
    T, n = done.shape
    a = np.asarray(carry, dtype=f32).copy()
    air = np.empty((T, n, 2), dtype=f32)
    for t in range(T):
        a = np.where(contact[t] | done[t][:, None], f32(0.0), a + f32(ctrl_dt)).astype(f32)
        air[t] = a
    prev = np.concatenate([np.zeros((1, n, 2), dtype=bool), contact[:-1]], axis=0)
    td = contact & ~prev
    shifted = np.roll(air, 1, axis=0)
    r = ((shifted - f32(touchdown_penalty)) * td.astype(f32)).astype(f32)
    return (r[..., 0] + r[..., 1]).astype(f32), a


class OracleEnv:
    """N environments simulated by the CPU oracle, same state layout as the engine."""

    def __init__(self, cmodel, cfg, n_envs: int, env_offset: int = 0, seed: int = 0, precision: str = "f32"):
        from zbot_amd import cstructs as cs  # noqa: PLC0415

        self.cs = cs
        self.L = lib(precision)
        self.model = cmodel
        self.cfg = cfg
        self.n = n_envs
        self.env_offset = env_offset
        self.seed = seed
        self.state = np.zeros((n_envs, cs.STATE_STRIDE), dtype=np.float32)
        self.rand = np.zeros((n_envs, cs.RAND_STRIDE), dtype=np.float32)
        self.stats = np.zeros((n_envs, cs.NUM_STATS), dtype=np.float32)
        self.iters = np.zeros(n_envs, dtype=np.int32)

    def reset(self, mask: np.ndarray | None = None):
        cs = self.cs
        oa = np.zeros((self.n, cs.OBS_ACTOR), dtype=np.float32)
        oc = np.zeros((self.n, cs.OBS_CRITIC), dtype=np.float32)
        ox = np.zeros((self.n, cs.OBS_EXTRA), dtype=np.float32)
        m = None if mask is None else np.ascontiguousarray(mask, dtype=np.uint8)
        rc = self.L.zbo_reset(C.byref(self.model), C.byref(self.cfg), self.n, self.env_offset, self.seed,
                              _p(self.state), _p(self.rand), _p(m, C.c_uint8), _p(oa), _p(oc), _p(ox))
        assert rc == 0
        return oa, oc, ox

    def step(self, action: np.ndarray, curriculum: float = 1.0):
        cs = self.cs
        action = np.ascontiguousarray(action, dtype=np.float32)
        assert action.shape == (self.n, cs.NJ)
        oa = np.zeros((self.n, cs.OBS_ACTOR), dtype=np.float32)
        oc = np.zeros((self.n, cs.OBS_CRITIC), dtype=np.float32)
        ox = np.zeros((self.n, cs.OBS_EXTRA), dtype=np.float32)
        terms = np.zeros((self.n, cs.NUM_TERMS), dtype=np.float32)
        rew = np.zeros(self.n, dtype=np.float32)
        done = np.zeros(self.n, dtype=np.uint8)
        success = np.zeros(self.n, dtype=np.uint8)
        rc = self.L.zbo_step(C.byref(self.model), C.byref(self.cfg), self.n, self.env_offset, self.seed,
                             _p(self.state), _p(self.rand), _p(action), _p(oa), _p(oc), _p(ox), _p(terms), _p(rew),
                             _p(done, C.c_uint8), _p(success, C.c_uint8), curriculum, _p(self.stats),
                             _p(self.iters, C.c_int32))
        assert rc == 0
        return dict(obs_actor=oa, obs_critic=oc, obs_extra=ox, reward_terms=terms, reward=rew, done=done,
                    success=success)


def box_box(c1, R1, s1, c2, R2, s2, margin: float = 0.0, precision: str = "f64"):
    """The oracle's box-box collider (zb_oracle.c box_box, the sole pair): (positions [k, 3],
    distances [k], normal from box 1 to box 2). R: 3x3 rotations (columns = the box axes)."""
    f = lambda a, n: np.ascontiguousarray(np.asarray(a, np.float32).reshape(n))  # noqa: E731
    pos, dist, nrm = np.zeros(12, np.float32), np.zeros(4, np.float32), np.zeros(3, np.float32)
    k = lib(precision).zbo_box_box(_p(f(c1, 3)), _p(f(R1, 9)), _p(f(s1, 3)), _p(f(c2, 3)), _p(f(R2, 9)), _p(f(s2, 3)),
                                   float(margin), _p(pos), _p(dist), _p(nrm))
    return pos.reshape(4, 3)[:k], dist[:k], nrm


def plane_mesh(verts, R, c, margin: float = 0.0, precision: str = "f64"):
    """The oracle's plane - convex mesh collider (zb_oracle.c plane_mesh, MJX's plane_convex): the four
    candidates' vertex indices [4], distances [4] (1 for a repeat) and world positions [4, 3] (the
    vertices, before the half-distance shift), and how many pass the margin. verts: [nv, 3] hull
    vertices in the geom frame; R: the geom's 3x3 world rotation; c: its centre."""
    v = np.zeros((len(verts), 4), np.float32)
    v[:, :3] = np.asarray(verts, np.float32)
    f = lambda a, n: np.ascontiguousarray(np.asarray(a, np.float32).reshape(n))  # noqa: E731
    idx, dist, pos = np.zeros(4, np.int32), np.zeros(4, np.float32), np.zeros(12, np.float32)
    k = lib(precision).zbo_plane_mesh(_p(v), len(verts), _p(f(R, 9)), _p(f(c, 3)), float(margin),
                                      idx.ctypes.data_as(C.POINTER(C.c_int32)), _p(dist), _p(pos))
    assert k >= 0
    return idx, dist, pos.reshape(4, 3), k


def forward_debug(cmodel, cfg, qpos, qvel, ctrl=None, precision: str = "f32") -> dict:
    nv, nb = cmodel.nv, cmodel.nbody
    qpos = np.ascontiguousarray(qpos, dtype=np.float32)
    qvel = np.ascontiguousarray(qvel, dtype=np.float32)
    ctrl = None if ctrl is None else np.ascontiguousarray(ctrl, dtype=np.float32)
    out = dict(
        qM=np.zeros((nv, nv), np.float32), qfrc_bias=np.zeros(nv, np.float32), qacc_smooth=np.zeros(nv, np.float32),
        qacc=np.zeros(nv, np.float32), xpos=np.zeros((nb, 3), np.float32), cinert=np.zeros((nb, 10), np.float32),
        cvel=np.zeros((nb, 6), np.float32), touch=np.zeros(2, np.float32),
    )
    nn = (C.c_int * 2)()
    lib(precision).zbo_forward_debug(C.byref(cmodel), C.byref(cfg), _p(qpos), _p(qvel), _p(ctrl), _p(out["qM"]),
                                     _p(out["qfrc_bias"]), _p(out["qacc_smooth"]), _p(out["qacc"]), _p(out["xpos"]),
                                     _p(out["cinert"]), _p(out["cvel"]), nn, _p(out["touch"]))
    out["nefc"], out["ncon"] = nn[0], nn[1]
    return out


def step_clearance(env, action, curriculum: float = 1.0):
    """env.step(action) that also returns each env's smallest floor-contact clearance over the step's
    substeps, min |distance - margin| of a contact candidate (zbo_set_clearance_out): (outputs, [n])."""
    out = np.full(env.n, np.inf, np.float32)
    env.L.zbo_set_clearance_out(_p(out))
    try:
        res = env.step(action, curriculum)
    finally:
        env.L.zbo_set_clearance_out(None)
    return res, out


def contact_count(cmodel, cfg, qpos, rnd=None, precision: str = "f64") -> int:
    """Contacts of the collision stage at qpos (the env's randomization row rnd applied)."""
    q = np.ascontiguousarray(qpos, dtype=np.float32)
    r = None if rnd is None else np.ascontiguousarray(rnd, dtype=np.float32)
    return int(lib(precision).zbo_contact_count(C.byref(cmodel), C.byref(cfg), _p(q), _p(r)))


def constraint_problem(cmodel, cfg, qpos, qvel, ctrl=None, qaccw=None, precision: str = "f32") -> dict:
    """The constrained-acceleration problem of one forward pass and the oracle's Newton solution:
    qM [nv, nv], qacc_smooth, qacc, and the rows J [nefc, nv], D, R, aref, floss, type
    (0 frictionloss, 1 joint limit, 2 contact pyramid edge)."""
    nv = cmodel.nv
    maxefc = 2 * 32 + 4 * 32
    qpos = np.ascontiguousarray(qpos, dtype=np.float32)
    qvel = np.ascontiguousarray(qvel, dtype=np.float32)
    ctrl = None if ctrl is None else np.ascontiguousarray(ctrl, dtype=np.float32)
    qaccw = None if qaccw is None else np.ascontiguousarray(qaccw, dtype=np.float32)
    qM = np.zeros((nv, nv), np.float32)
    qs, qa = np.zeros(nv, np.float32), np.zeros(nv, np.float32)
    J = np.zeros((maxefc, nv), np.float32)
    D, R, aref, floss = (np.zeros(maxefc, np.float32) for _ in range(4))
    typ = np.zeros(maxefc, np.int32)
    ne = lib(precision).zbo_constraint_debug(C.byref(cmodel), C.byref(cfg), _p(qpos), _p(qvel), _p(ctrl), _p(qaccw),
                                             _p(qM), _p(qs), _p(qa), _p(J), _p(D), _p(R), _p(aref), _p(floss),
                                             typ.ctypes.data_as(C.POINTER(C.c_int)))
    return dict(qM=qM, qacc_smooth=qs, qacc=qa, J=J[:ne], D=D[:ne], R=R[:ne], aref=aref[:ne], floss=floss[:ne],
                type=typ[:ne])


def simulate(cmodel, cfg, qpos, qvel, nsteps: int, ctrl=None, qaccw=None, precision: str = "f32"):
    qpos = np.array(qpos, dtype=np.float32)
    qvel = np.array(qvel, dtype=np.float32)
    qaccw = np.zeros(cmodel.nv, np.float32) if qaccw is None else np.array(qaccw, dtype=np.float32)
    ctrl = None if ctrl is None else np.ascontiguousarray(ctrl, dtype=np.float32)
    lib(precision).zbo_simulate(C.byref(cmodel), C.byref(cfg), _p(qpos), _p(qvel), _p(qaccw), _p(ctrl), nsteps)
    return qpos, qvel, qaccw


# ---- post-rollout PPO inputs (zb_oracle_ppo.c) ----

def ppo_lib() -> C.CDLL:
    if "ppo" in _LIBS:
        return _LIBS["ppo"]
    path = os.path.join(HERE, "liboracle_ppo.so")
    if not os.path.exists(path):
        build()
    L = C.CDLL(path)
    fp, u8p, dp = C.POINTER(C.c_float), C.POINTER(C.c_uint8), C.POINTER(C.c_double)
    L.zbo_gae.argtypes = [fp, fp, u8p, u8p, fp, C.c_int, C.c_int, C.c_float, C.c_float, fp, fp, dp]
    L.zbo_moments_tree.argtypes = [dp, C.c_int, dp]
    L.zbo_adv_normalize.argtypes = [fp, fp, C.c_longlong, dp, C.c_double, C.c_float]
    _LIBS["ppo"] = L
    return L


def gae(reward, values, done, gamma: float, lam: float, success=None, bootstrap=None):
    """Serial reverse-scan GAE over [T, n] arrays -> (gae, value_targets, per-env moments [n, 2])."""
    f32 = lambda x: None if x is None else np.ascontiguousarray(x, dtype=np.float32)  # noqa: E731
    u8 = lambda x: None if x is None else np.ascontiguousarray(x, dtype=np.uint8)  # noqa: E731
    reward, values, bootstrap = f32(reward), f32(values), f32(bootstrap)
    done, success = u8(done), u8(success)
    T, n = reward.shape
    g = np.zeros((T, n), np.float32)
    vt = np.zeros((T, n), np.float32)
    mom = np.zeros((n, 2), np.float64)
    ppo_lib().zbo_gae(_p(reward), _p(values), _p(done, C.c_uint8), _p(success, C.c_uint8), _p(bootstrap), T, n,
                      gamma, lam, _p(g), _p(vt), _p(mom, C.c_double))
    return g, vt, mom


def moments_tree(pairs) -> np.ndarray:
    """Pairwise tree over [k, 2] (sum, sum^2) rows, zero-padded to a power of two."""
    p = np.ascontiguousarray(pairs, dtype=np.float64).reshape(-1, 2)
    out = np.zeros(2, np.float64)
    ppo_lib().zbo_moments_tree(_p(p, C.c_double), p.shape[0], _p(out, C.c_double))
    return out


def adv_normalize(g, moments, total: float, eps: float = 1e-6) -> np.ndarray:
    g = np.ascontiguousarray(g, dtype=np.float32)
    out = np.zeros_like(g)
    m = np.ascontiguousarray(moments, dtype=np.float64)
    ppo_lib().zbo_adv_normalize(_p(g), _p(out), g.size, _p(m, C.c_double), float(total), eps)
    return out


# ---- GRU actor / critic + mixture head (zb_oracle_policy.c) ----

def policy_lib() -> C.CDLL:
    if "policy" in _LIBS:
        return _LIBS["policy"]
    path = os.path.join(HERE, "liboracle_policy.so")
    if not os.path.exists(path):
        build()
    L = C.CDLL(path)
    fp, u8p, u32p = C.POINTER(C.c_float), C.POINTER(C.c_uint8), C.POINTER(C.c_uint32)
    L.zbo_policy_param_count.argtypes = [C.c_int]
    L.zbo_policy_param_count.restype = C.c_size_t
    L.zbo_policy_actor.argtypes = [fp, fp, C.c_int, C.c_int, fp, u8p, C.c_int, C.c_uint64, C.c_int, C.c_uint32, fp, fp]
    L.zbo_policy_critic.argtypes = [fp, fp, C.c_int, C.c_int, fp, u8p, fp]
    for name in ("exp", "log", "tanh", "sigmoid", "softplus"):
        f = getattr(L, "zbo_fm_" + name)
        f.argtypes = [C.c_float]
        f.restype = C.c_float
    L.zbo_fm_sincos_turns.argtypes = [C.c_float, fp, fp]
    L.zbo_fm_threefry.argtypes = [C.c_uint32] * 4 + [u32p]
    L.zbo_fm_normal.argtypes = [C.c_uint64, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32]
    L.zbo_fm_normal.restype = C.c_float
    L.zbo_fm_mix_log_prob.argtypes = [fp, fp, fp, C.c_float]
    L.zbo_fm_mix_log_prob.restype = C.c_float
    L.zbo_fm_mix_sample_batch.argtypes = [fp, fp, fp, C.c_int, C.c_uint64, C.c_int, C.c_uint32, C.c_int, fp]
    L.zbo_fm_normal_batch.argtypes = [C.c_uint64, C.c_uint32, C.c_int, fp]
    _LIBS["policy"] = L
    return L


def policy_param_count(kind: int) -> int:
    return int(policy_lib().zbo_policy_param_count(kind))


def policy_actor(params, obs, carry, reset=None, mode: int = 0, seed: int = 0, env_offset: int = 0, step0: int = 0,
                 actions=None, log_prob: bool = False):
    """obs [T, n, 50], carry [n, 5, 128] (a copy is updated and returned).
    Returns (actions [T, n, 20], log_prob [T, n, 20] or None, carry)."""
    P = np.ascontiguousarray(params, dtype=np.float32)
    obs = np.ascontiguousarray(obs, dtype=np.float32)
    T, n, _ = obs.shape
    c = np.array(carry, dtype=np.float32, copy=True, order="C")
    r = None if reset is None else np.ascontiguousarray(np.asarray(reset).reshape(T, n), dtype=np.uint8)
    a = (np.zeros((T, n, 20), np.float32) if actions is None
         else np.array(actions, dtype=np.float32, copy=True, order="C").reshape(T, n, 20))
    lp = np.zeros((T, n, 20), np.float32) if log_prob else None
    policy_lib().zbo_policy_actor(_p(P), _p(obs), T, n, _p(c), _p(r, C.c_uint8), mode, seed, env_offset, step0, _p(a),
                                  _p(lp))
    return a, lp, c


def policy_critic(params, obs, carry, reset=None):
    """obs [T, n, 484], carry [n, 5, 128] -> (value [T, n], carry)."""
    P = np.ascontiguousarray(params, dtype=np.float32)
    obs = np.ascontiguousarray(obs, dtype=np.float32)
    T, n, _ = obs.shape
    c = np.array(carry, dtype=np.float32, copy=True, order="C")
    r = None if reset is None else np.ascontiguousarray(np.asarray(reset).reshape(T, n), dtype=np.uint8)
    v = np.zeros((T, n), np.float32)
    policy_lib().zbo_policy_critic(_p(P), _p(obs), T, n, _p(c), _p(r, C.c_uint8), _p(v))
    return v, c


def fm(name: str, x) -> np.ndarray:
    f = getattr(policy_lib(), "zbo_fm_" + name)
    return np.array([f(float(v)) for v in np.asarray(x, dtype=np.float32).ravel()], dtype=np.float32)


def fm_sincos(t):
    L = policy_lib()
    s, c = C.c_float(), C.c_float()
    out = []
    for v in np.asarray(t, dtype=np.float32).ravel():
        L.zbo_fm_sincos_turns(float(v), C.byref(s), C.byref(c))
        out.append((s.value, c.value))
    return np.array(out, dtype=np.float32).T


def fm_threefry(k0, k1, c0, c1):
    o = (C.c_uint32 * 2)()
    policy_lib().zbo_fm_threefry(k0 & 0xFFFFFFFF, k1 & 0xFFFFFFFF, c0 & 0xFFFFFFFF, c1 & 0xFFFFFFFF, o)
    return o[0], o[1]


def fm_normals(seed: int, purpose: int, n: int) -> np.ndarray:
    out = np.zeros(n, np.float32)
    policy_lib().zbo_fm_normal_batch(seed, purpose, n, _p(out))
    return out


def mix_sample_batch(mu, sd, lg, seed: int, n: int, step: int = 0, j: int = 0, argmax: bool = False):
    mu, sd, lg = (np.ascontiguousarray(x, dtype=np.float32) for x in (mu, sd, lg))
    out = np.zeros(n, np.float32)
    policy_lib().zbo_fm_mix_sample_batch(_p(mu), _p(sd), _p(lg), int(argmax), seed, n, step, j, _p(out))
    return out


def mix_log_prob(mu, sd, lg, a: float) -> float:
    mu, sd, lg = (np.ascontiguousarray(x, dtype=np.float32) for x in (mu, sd, lg))
    return float(policy_lib().zbo_fm_mix_log_prob(_p(mu), _p(sd), _p(lg), float(a)))
