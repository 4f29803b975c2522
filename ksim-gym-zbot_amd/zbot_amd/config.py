"""Environment configuration (ZbEnvConfig) with the reference's values.

Sources: train.py:1766-1788 (simulation parameters), train.py:1439-1476
(randomizers, push event, resets), train.py:1478-1537 (observation noise),
train.py:1546-1593 (reward scales, terminations). Values marked [U] belong to
un-vendored ksim 0.1.99 defaults that cannot be read in this container.
"""

from __future__ import annotations

import ctypes
import math

from . import cstructs as cs
from .constants import CTRL_DT, DT, ITERATIONS, LS_ITERATIONS, REWARDS


def default_config(
    *,
    obs_noise: bool = True,
    push: bool = False,
    randomize: bool = False,
    autoreset: bool = True,
    iterations: int = ITERATIONS,
    ls_iterations: int = LS_ITERATIONS,
    dt: float = DT,
    ctrl_dt: float = CTRL_DT,
    max_episode_sec: float = 80.0,
    solver: str = "cg",
    eulerdamp: bool = False,
) -> cs.ZbEnvConfig:
    """solver: "cg" (default: mj_solCG / MJX SolverType.CG, the solver ksim's MJX model setup selects
    as DESIGN.md §8 records it [U: ksim 0.1.99 is not on disk]) or "newton" (MuJoCo's own default,
    mj_solNewton). SURVEY §8a a11 reads "likely CG".

    eulerdamp: mj_Euler's implicit joint damping (MuJoCo's default, mjDSBL_EULERDAMP clear): qvel
    advances with (M + dt diag(damping))^-1 (qfrc_smooth + qfrc_constraint). Off by default: ksim
    sets the disable bit on its MJX model [U], so the damping is explicit."""
    if solver not in ("newton", "cg"):
        raise ValueError(f"solver must be 'newton' or 'cg', got {solver!r}")
    c = cs.ZbEnvConfig()
    c.struct_bytes = ctypes.sizeof(cs.ZbEnvConfig)
    flags = 0
    if obs_noise:
        flags |= cs.F_OBS_NOISE
    if push:
        flags |= cs.F_PUSH
    if randomize:
        flags |= cs.F_RANDOMIZE
    if autoreset:
        flags |= cs.F_AUTORESET
    if eulerdamp:
        flags |= cs.F_EULERDAMP
    c.flags = flags
    c.n_substeps = int(round(ctrl_dt / dt))  # ksim: round(ctrl_dt / dt) physics steps per control step
    c.iterations = iterations  # train.py:1779
    c.ls_iterations = ls_iterations  # train.py:1780
    c.dt = dt  # train.py:1777
    c.ctrl_dt = ctrl_dt  # train.py:1778
    c.tolerance = 1e-8  # MuJoCo opt.tolerance default
    c.ls_tolerance = 0.01  # MuJoCo opt.ls_tolerance default
    c.imu_noise_std = math.radians(1)  # train.py:1497
    c.acc_noise_std = 0.5  # train.py:1503
    c.reset_qvel_scale = 0.01  # ksim RandomJointVelocityReset default scale [U]
    c.max_episode_sec = max_episode_sec  # train.py:1592 (80 s)
    c.lag_range[0], c.lag_range[1] = 0.0, 0.1  # train.py:1496
    c.bad_z[0], c.bad_z[1] = 0.05, 0.5  # train.py:1590
    c.max_tilt_rad = math.radians(60)  # train.py:1591
    c.push_linvel[0], c.push_linvel[1], c.push_linvel[2] = 0.1, 0.1, 0.05  # train.py:1460-1462
    c.push_interval[0], c.push_interval[1] = 2.0, 4.0  # train.py:1467
    c.push_vel_range[0], c.push_vel_range[1] = 0.05, 0.15  # train.py:1466
    for i, (_, scale, by_curr) in enumerate(REWARDS):
        c.reward_scale[i] = scale
        c.reward_by_curriculum[i] = 1 if by_curr else 0
    c.feet_airtime_touchdown_penalty = 0.3  # train.py:1562
    c.naive_forward_clip_max = 0.2  # train.py:1550
    c.feet_orient_error_scale = 0.25  # train.py:1568
    c.feet_too_close_threshold = 0.12  # train.py:1573
    c.touch_threshold = 0.1  # train.py:516, 702
    c.stay_alive_balance = 10.0  # ksim StayAliveReward balance [U]
    c.rand_mass[0], c.rand_mass[1] = 0.95, 1.15  # train.py:1443
    c.rand_armature[0], c.rand_armature[1] = 1.0, 1.05  # ksim ArmatureRandomizer [U]
    c.rand_damping[0], c.rand_damping[1] = 0.95, 1.05  # ksim JointDampingRandomizer [U]
    c.rand_friction[0], c.rand_friction[1] = 0.5, 1.5  # ksim StaticFrictionRandomizer [U]
    c.rand_qpos0[0], c.rand_qpos0[1] = math.radians(-2), math.radians(2)  # train.py:1445
    c.rand_floor_mu[0], c.rand_floor_mu[1] = 0.3, 1.5  # train.py:1447
    c.rand_imu_tilt_std = math.radians(5)  # train.py:1453
    c.rand_imu_yaw_std = math.radians(1.0)
    c.rand_imu_pos_std = 0.005
    c.solver = cs.SOLVER_CG if solver == "cg" else cs.SOLVER_NEWTON
    return c


def config_flags(c: cs.ZbEnvConfig) -> dict:
    return {
        "obs_noise": bool(c.flags & cs.F_OBS_NOISE),
        "push": bool(c.flags & cs.F_PUSH),
        "randomize": bool(c.flags & cs.F_RANDOMIZE),
        "autoreset": bool(c.flags & cs.F_AUTORESET),
        "eulerdamp": bool(c.flags & cs.F_EULERDAMP),
    }
