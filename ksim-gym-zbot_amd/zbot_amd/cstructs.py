"""ctypes mirrors of include/zbot_model.h and include/zbot_layout.h.

Field order and types must match the C headers exactly; tests/test_abi.py checks
every field offset against the offsets the compiled C code reports.
"""

import ctypes as C

MAX_BODY = 32
MAX_DOF = 32
MAX_QPOS = 40
MAX_DEPTH = 12
MAX_GEOM = 16
MAX_MESHV = 64
MAX_MESHVERT = 512
MAX_SITE = 8
MAX_ACT = 32
CON_PER_GEOM = 4
CON_PER_PAIR = 4  # box-box: the sole pair

MODEL_MAGIC = 0x5A424F54
MODEL_VERSION = 9

JNT_NONE = -1
JNT_FREE = 0
JNT_HINGE = 3
GEOM_SPHERE, GEOM_CAPSULE, GEOM_ELLIPSOID, GEOM_CYLINDER, GEOM_BOX, GEOM_MESH = 2, 3, 4, 5, 6, 7

# zbot_layout.h
NJ = 20
NBODY_TASK = 26
OBS_ACTOR = 50
OBS_CRITIC = 484
OBS_EXTRA = 96
NUM_TERMS = 12
NUM_CMD = 7
NUM_STATS = 4

STATE_STRIDE = 192
S_QPOS = 0
S_QVEL = 32
S_QACCW = 64
S_PLAN_POS = 96
S_PLAN_VEL = 116
S_PLAN_TAU = 136
S_IMU_EMA = 156
S_IMU_LAG = 160
S_AIRTIME = 161
S_PUSH_TIMER = 163
S_TOUCH = 164
S_FEET_DIST = 166
S_EP_RETURN = 167
S_EP_STEPS = 168
S_RNG_STEP = 169
S_PREV_CONT = 170
S_EPISODE = 172
S_NAN = 173
# S_NAN's sticky flag bits (include/zbot_layout.h)
NAN_NONFINITE = 1
NAN_BANK_OVERFLOW = 2
NAN_BANK_OVERFLOW_STEP = 4  # the same, in the last control step only
S_AIR0_CONT = 174
S_AIR0_TERM = 175
S_END = 176

RAND_STRIDE = 160
R_MASS = 0
R_ARMATURE = 32
R_DAMPING = 64
R_FRICTION = 96
R_QPOS0 = 128
R_FLOOR_MU = 148
R_IMU_QUAT = 149
R_IMU_POS = 153

X_BASE_LINVEL = 0
X_BASE_ANGVEL = 3
X_BASE_LINACC = 6
X_BASE_ANGACC = 9
X_BASE_HEIGHT = 12
X_TOUCH = 13
X_FORCE = 15
X_FEET_POS = 21
X_FEETECH_TAU = 27
X_ACT_ACC = 47

TERM_NAMES = (
    "stay_alive",
    "upright",
    "naive_forward",
    "naive_forward_orientation",
    "linear_velocity_penalty_y",
    "simple_single_foot_contact",
    "feet_airtime",
    "feet_orientation",
    "feet_too_close",
    "straight_leg_penalty",
    "ankle_knee_penalty",
    "arm_pose_penalty",
)

ST_RETURN = 0
ST_LENGTH = 1
ST_DONE = 2
ST_REWARD = 3

SOLVER_NEWTON = 0  # ZB_SOLVER_NEWTON
SOLVER_CG = 1  # ZB_SOLVER_CG
F_OBS_NOISE = 1
F_PUSH = 2
F_RANDOMIZE = 4
F_AUTORESET = 8
F_EULERDAMP = 16  # ZB_F_EULERDAMP: mj_Euler's implicit joint damping


def _f(n: int, m: int = 0) -> type:
    t = C.c_float * n
    return (C.c_float * m) * n if m else t


def _i(n: int, m: int = 0) -> type:
    return (C.c_int32 * m) * n if m else C.c_int32 * n


class ZbModel(C.Structure):
    _fields_ = [
        ("magic", C.c_uint32),
        ("version", C.c_int32),
        ("struct_bytes", C.c_int32),
        ("nbody", C.c_int32),
        ("nq", C.c_int32),
        ("nv", C.c_int32),
        ("nu", C.c_int32),
        ("ngeom", C.c_int32),
        ("nsite", C.c_int32),
        ("max_depth", C.c_int32),
        ("gravity", _f(4)),
        ("timestep", C.c_float),
        ("meaninertia", C.c_float),
        ("pad_opt", _f(2)),
        ("body_parent", _i(MAX_BODY)),
        ("body_depth", _i(MAX_BODY)),
        ("body_jnttype", _i(MAX_BODY)),
        ("body_dofadr", _i(MAX_BODY)),
        ("body_dofnum", _i(MAX_BODY)),
        ("body_qposadr", _i(MAX_BODY)),
        ("body_lastdof", _i(MAX_BODY)),
        ("body_pos", _f(MAX_BODY, 4)),
        ("body_quat", _f(MAX_BODY, 4)),
        ("body_ipos", _f(MAX_BODY, 4)),
        ("body_iquat", _f(MAX_BODY, 4)),
        ("body_mass", _f(MAX_BODY, 4)),
        ("body_inertia", _f(MAX_BODY, 4)),
        ("body_invweight0", _f(MAX_BODY, 4)),
        ("jnt_axis", _f(MAX_BODY, 4)),
        ("jnt_pos", _f(MAX_BODY, 4)),
        ("dof_body", _i(MAX_DOF)),
        ("dof_parent", _i(MAX_DOF)),
        ("dof_depth", _i(MAX_DOF)),
        ("dof_anc", _i(MAX_DOF, MAX_DEPTH)),
        ("dof_limited", _i(MAX_DOF)),
        ("dof_qposadr", _i(MAX_DOF)),
        ("dof_armature", _f(MAX_DOF)),
        ("dof_damping", _f(MAX_DOF)),
        ("dof_frictionloss", _f(MAX_DOF)),
        ("dof_invweight0", _f(MAX_DOF)),
        ("dof_range", _f(MAX_DOF, 2)),
        ("dof_solref", _f(4)),
        ("dof_solimp", _f(8)),
        ("qpos0", _f(MAX_QPOS)),
        ("pad_q", _f(4)),
        ("act_dof", _i(MAX_ACT)),
        ("act_gear", _f(MAX_ACT)),
        ("act_ctrlrange", _f(MAX_ACT, 2)),
        ("fe_kp", _f(MAX_ACT)),
        ("fe_kd", _f(MAX_ACT)),
        ("fe_error_gain", _f(MAX_ACT)),
        ("fe_max_pwm", _f(MAX_ACT)),
        ("fe_vin", _f(MAX_ACT)),
        ("fe_kt", _f(MAX_ACT)),
        ("fe_R", _f(MAX_ACT)),
        ("fe_vmax", _f(MAX_ACT)),
        ("fe_amax", _f(MAX_ACT)),
        ("fe_max_torque", _f(MAX_ACT)),
        ("fe_max_velocity", _f(MAX_ACT)),
        ("geom_body", _i(MAX_GEOM)),
        ("geom_type", _i(MAX_GEOM)),
        ("geom_pos", _f(MAX_GEOM, 4)),
        ("geom_quat", _f(MAX_GEOM, 4)),
        ("geom_size", _f(MAX_GEOM, 4)),
        ("floor_friction", _f(4)),
        ("floor_solref", _f(4)),
        ("floor_solimp", _f(8)),
        ("floor_margin", C.c_float),
        ("pad_floor", _f(3)),
        ("npair", C.c_int32),
        ("pair_geom", _i(2)),
        ("pair_margin", C.c_float),
        ("pair_friction", _f(4)),
        ("pair_solref", _f(4)),
        ("pair_solimp", _f(8)),
        ("site_body", _i(MAX_SITE)),
        ("site_pos", _f(MAX_SITE, 4)),
        ("site_quat", _f(MAX_SITE, 4)),
        ("site_imu", C.c_int32),
        ("site_left_foot", C.c_int32),
        ("site_right_foot", C.c_int32),
        ("body_base", C.c_int32),
        ("body_left_foot", C.c_int32),
        ("body_right_foot", C.c_int32),
        ("geom_left_foot", C.c_int32),
        ("geom_right_foot", C.c_int32),
        ("max_body_depth", C.c_int32),
        ("mrow_size", C.c_int32),
        ("nskip_geom", C.c_int32),
        ("nskip_pair", C.c_int32),
        ("body_nchild", _i(MAX_BODY)),
        ("body_child", _i(MAX_BODY, 8)),
        ("depth_maxchild", _i(16)),
        ("dof_desc", C.c_uint32 * MAX_DOF),
        ("dof_ancpk", (C.c_uint32 * 4) * MAX_DOF),
        ("dof_rowmask", C.c_uint32 * MAX_DOF),
        ("dof_act", _i(MAX_DOF)),
        ("dof_rowoff", _i(MAX_DOF)),
        ("geom_lastdof", _i(MAX_GEOM)),
        ("nlevel", C.c_int32),
        ("pad_lvl", _i(3)),
        ("level_nmem", _i(MAX_DEPTH)),
        ("level_mem", _i(MAX_DEPTH, 8)),
        ("joint_bias", _f(MAX_ACT)),
        ("joint_weight", _f(MAX_ACT)),
        ("geom_vertadr", _i(MAX_GEOM)),
        ("geom_vertnum", _i(MAX_GEOM)),
        ("mesh_vert", _f(MAX_MESHVERT, 4)),
        ("pad_end", _f(4)),
    ]


class ZbEnvConfig(C.Structure):
    _fields_ = [
        ("struct_bytes", C.c_int32),
        ("flags", C.c_uint32),
        ("n_substeps", C.c_int32),
        ("iterations", C.c_int32),
        ("ls_iterations", C.c_int32),
        ("dt", C.c_float),
        ("ctrl_dt", C.c_float),
        ("tolerance", C.c_float),
        ("ls_tolerance", C.c_float),
        ("imu_noise_std", C.c_float),
        ("acc_noise_std", C.c_float),
        ("reset_qvel_scale", C.c_float),
        ("max_episode_sec", C.c_float),
        ("lag_range", _f(2)),
        ("bad_z", _f(2)),
        ("max_tilt_rad", C.c_float),
        ("push_linvel", _f(4)),
        ("push_interval", _f(2)),
        ("push_vel_range", _f(2)),
        ("reward_scale", _f(NUM_TERMS)),
        ("reward_by_curriculum", _i(NUM_TERMS)),
        ("feet_airtime_touchdown_penalty", C.c_float),
        ("naive_forward_clip_max", C.c_float),
        ("feet_orient_error_scale", C.c_float),
        ("feet_too_close_threshold", C.c_float),
        ("touch_threshold", C.c_float),
        ("stay_alive_balance", C.c_float),
        ("rand_mass", _f(2)),
        ("rand_armature", _f(2)),
        ("rand_damping", _f(2)),
        ("rand_friction", _f(2)),
        ("rand_qpos0", _f(2)),
        ("rand_floor_mu", _f(2)),
        ("rand_imu_tilt_std", C.c_float),
        ("rand_imu_yaw_std", C.c_float),
        ("rand_imu_pos_std", C.c_float),
        ("solver", C.c_int32),
        ("pad", _f(2)),
    ]


def struct_field_names(cls: type) -> list[str]:
    return [name for name, _ in cls._fields_]
