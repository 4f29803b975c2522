"""Known-answer tests of the oracle's restatement of the reference's pure functions.

Expected values are derived by hand from the train.py text (cited per test),
from the reference's own docstring example (train.py:798) and from Random123's
published threefry2x32-20 vectors.
"""

import math

import numpy as np
import pytest


# ---- threefry2x32-20 known-answer vectors (Random123) ----
@pytest.mark.parametrize(
    "key,ctr,expect",
    [
        ((0, 0), (0, 0), (0x6B200159, 0x99BA4EFE)),
        ((0xFFFFFFFF, 0xFFFFFFFF), (0xFFFFFFFF, 0xFFFFFFFF), (0x1CB996FC, 0xBB002BE7)),
        ((0x13198A2E, 0x03707344), (0x243F6A88, 0x85A308D3), (0xC4923A9C, 0x483DF7A0)),
    ],
)
def test_threefry_kat(oracle_mod, key, ctr, expect):
    assert oracle_mod.threefry2x32(key[0], key[1], ctr[0], ctr[1]) == expect


# ---- trapezoidal_step, train.py:1137-1196 ----
DT = 0.001
VMAX = 5.0  # train.py:1345
AMAX = 17.45  # train.py:1346
DEADBAND = 2 * 0.087 * math.pi / 180  # train.py:1113-1116


def _trap(O, pos, vel, target):
    n = len(pos)
    return O.trapezoidal_step(np.array(pos), np.array(vel), np.array(target), DT, np.full(n, VMAX), np.full(n, AMAX))


def test_deadband_decay(oracle_mod):
    # |error| <= deadband -> velocity * 0.8, position integrates it (train.py:1151-1156)
    p, v = _trap(oracle_mod, [0.0], [1.0], [0.5 * DEADBAND])
    assert v[0] == pytest.approx(0.8, rel=1e-6)
    assert p[0] == pytest.approx(0.8 * DT, rel=1e-6)


def test_accelerate_from_rest(oracle_mod):
    # |vel| < 1e-6 -> accelerate towards target (train.py:1178-1182)
    p, v = _trap(oracle_mod, [0.0], [0.0], [1.0])
    assert v[0] == pytest.approx(AMAX * DT, rel=1e-6)
    assert p[0] == pytest.approx(AMAX * DT * DT, rel=1e-5)


def test_velocity_clip(oracle_mod):
    # moving towards a far target at vmax: accelerate then clip to vmax (train.py:1185)
    p, v = _trap(oracle_mod, [0.0], [VMAX], [10.0])
    assert v[0] == pytest.approx(VMAX, rel=1e-7)
    assert p[0] == pytest.approx(VMAX * DT, rel=1e-6)


def test_decelerate_inside_stopping_distance(oracle_mod):
    # stopping distance v^2/(2 a_max) = 0.1146 > error 0.05 -> decelerate (train.py:1162-1175)
    p, v = _trap(oracle_mod, [0.0], [2.0], [0.05])
    assert v[0] == pytest.approx(2.0 - AMAX * DT, rel=1e-6)
    assert p[0] == pytest.approx((2.0 - AMAX * DT) * DT, rel=1e-6)


def test_moving_away_decelerates(oracle_mod):
    # velocity opposite to the target direction -> acceleration = -sign(v) * a_max
    p, v = _trap(oracle_mod, [0.0], [-1.0], [1.0])
    assert v[0] == pytest.approx(-1.0 + AMAX * DT, rel=1e-6)


def test_negative_direction(oracle_mod):
    p, v = _trap(oracle_mod, [0.0], [0.0], [-1.0])
    assert v[0] == pytest.approx(-AMAX * DT, rel=1e-6)


def test_vectorised_mixed(oracle_mod):
    pos = [0.0, 0.0, 0.0, 0.0]
    vel = [1.0, 0.0, VMAX, 2.0]
    tgt = [0.5 * DEADBAND, 1.0, 10.0, 0.05]
    p, v = _trap(oracle_mod, pos, vel, tgt)
    np.testing.assert_allclose(v, [0.8, AMAX * DT, VMAX, 2.0 - AMAX * DT], rtol=1e-6)


# ---- Feetech duty -> torque, train.py:1260-1269 ----
def test_feetech_torque(oracle_mod, cmodel):
    m = cmodel.cmodel
    nu = m.nu
    q = np.array([m.joint_bias[a] for a in range(nu)], np.float32)
    plan_pos = q.copy()
    plan_vel = np.zeros(nu, np.float32)
    action = q + 0.2  # outside the deadband -> planner accelerates from rest
    qd = np.zeros(nu, np.float32)
    npos, nvel, tau = oracle_mod.feetech(m, DT, plan_pos, plan_vel, action, q, qd)
    for a in range(nu):
        amax = m.fe_amax[a]
        v_des = amax * DT
        p_des = q[a] + v_des * DT
        duty = m.fe_kp[a] * m.fe_error_gain[a] * (p_des - q[a]) + m.fe_kd[a] * v_des
        duty = max(-m.fe_max_pwm[a], min(m.fe_max_pwm[a], duty))
        expect = duty * m.fe_vin[a] * m.fe_kt[a] / m.fe_R[a]
        assert tau[a] == pytest.approx(expect, rel=1e-5, abs=1e-7)
        assert nvel[a] == pytest.approx(v_des, rel=1e-6)


def test_feetech_duty_clip(oracle_mod, cmodel):
    m = cmodel.cmodel
    nu = m.nu
    q = np.zeros(nu, np.float32)
    # huge tracking error -> duty clipped at +/- max_pwm
    npos, nvel, tau = oracle_mod.feetech(m, DT, q + 2.0, np.zeros(nu), q + 3.0, q, np.zeros(nu))
    for a in range(nu):
        assert tau[a] == pytest.approx(m.fe_max_pwm[a] * m.fe_vin[a] * m.fe_kt[a] / m.fe_R[a], rel=1e-6)


# ---- rotate_quat_by_quat, train.py:751-787 ----
def test_rotate_quat_docstring_example(oracle_mod):
    # train.py:798: yaw cmd = 3.14, IMU [0,0,0,1] -> back-spun obs [1,0,0,0]
    yaw = math.pi
    heading = np.array([math.cos(yaw / 2), 0.0, 0.0, math.sin(yaw / 2)])
    out = oracle_mod.rotate_quat_by_quat([0.0, 0.0, 0.0, 1.0], heading, inverse=True)
    np.testing.assert_allclose(np.abs(out), [1.0, 0.0, 0.0, 0.0], atol=1e-5)


def test_rotate_quat_identity_normalises(oracle_mod):
    q = np.array([2.0, 0.0, 0.0, 0.0])
    out = oracle_mod.rotate_quat_by_quat(q, [1.0, 0.0, 0.0, 0.0], inverse=True)
    # q/(|q|+eps) * ... / (|r|+eps): slightly below 1 because of the eps terms
    assert out[0] == pytest.approx(1.0, abs=2e-6)
    assert out[0] < 1.0


def test_rotate_quat_composition(oracle_mod):
    rng = np.random.default_rng(0)
    for _ in range(10):
        a = rng.normal(size=4)
        b = rng.normal(size=4)
        a /= np.linalg.norm(a)
        b /= np.linalg.norm(b)
        out = oracle_mod.rotate_quat_by_quat(a, b, inverse=False)
        w1, x1, y1, z1 = b
        w2, x2, y2, z2 = a
        ref = np.array([w1 * w2 - x1 * x2 - y1 * y2 - z1 * z2, w1 * x2 + x1 * w2 + y1 * z2 - z1 * y2,
                        w1 * y2 - x1 * z2 + y1 * w2 + z1 * x2, w1 * z2 + x1 * y2 - y1 * x2 + z1 * w2])
        np.testing.assert_allclose(out, ref / np.linalg.norm(ref), atol=1e-5)


def test_servo_deadband_value():
    from zbot_amd.constants import SERVO_DEADBAND

    assert SERVO_DEADBAND[0] == pytest.approx(0.0030368728984701336)
    assert SERVO_DEADBAND == (SERVO_DEADBAND[0], SERVO_DEADBAND[0])


def test_observation_dims():
    from zbot_amd.constants import NUM_ACTOR_INPUTS, NUM_CRITIC_INPUTS

    assert NUM_ACTOR_INPUTS == 50  # train.py:53
    assert NUM_CRITIC_INPUTS == 484  # train.py:54


# ---- FeetAirtimeReward over a trajectory, train.py:503-546 ----
def test_feet_airtime_traj_hand_case(oracle_mod):
    """Hand-derived: left contact [1,0,0,1,1], right always down, carry (0.1, 0), no dones.
    air_l = [0, .02, .04, 0, 0]; touchdowns (prev = False at t = 0): left t0, t3; right t0.
    Row 0 reads roll(air)[0] = air[T-1] = 0 for both feet: -0.3 - 0.3; row 3: .04 - .3."""
    c = np.zeros((5, 1, 2), bool)
    c[:, 0, 0] = [1, 0, 0, 1, 1]
    c[:, 0, 1] = True
    r, carry = oracle_mod.feet_airtime_traj(c, np.zeros((5, 1), bool), np.array([[0.1, 0.0]], np.float32))
    np.testing.assert_allclose(r[:, 0], [-0.6, 0, 0, np.float32(0.04) - np.float32(0.3), 0], rtol=0, atol=1e-7)
    assert carry.tolist() == [[0.0, 0.0]]


def test_feet_airtime_traj_roll_wrap_and_done(oracle_mod):
    """A touchdown at t = 0 only: row 0 is air[T-1] - 0.3 (jnp.roll wrap, train.py:533-534); a done
    zeroes the airtime like a contact (contact_or_done, train.py:511)."""
    c = np.zeros((5, 1, 2), bool)
    c[0, 0, 0] = True
    d = np.zeros((5, 1), bool)
    r, carry = oracle_mod.feet_airtime_traj(c, d, np.zeros((1, 2), np.float32))
    f = np.float32
    air4 = f(f(f(f(0.02) + f(0.02)) + f(0.02)) + f(0.02))
    assert r[0, 0] == f(air4 - f(0.3)) and (r[1:] == 0).all()
    assert carry[0, 0] == air4 and carry[0, 1] == f(f(f(f(f(0.02) + f(0.02)) + f(0.02)) + f(0.02)) + f(0.02))
    d[2, 0] = True
    r, _ = oracle_mod.feet_airtime_traj(c, d, np.zeros((1, 2), np.float32))
    assert r[0, 0] == f(f(f(0.02) + f(0.02)) - f(0.3))


def test_feet_airtime_causal_form_equals_ksim_after_row0(oracle_mod):
    """The fused step's causal per-step form (zb_engine.hip rewards(): touchdown against the
    previous step's contact, airtime of the previous step) gives ksim's rows t >= 1 bit for bit on
    random contact / done sequences; only row 0 differs (include/zbot.h zb_feet_airtime_exact)."""
    f = np.float32
    rng = np.random.default_rng(0)
    T, n = 40, 64
    c = rng.random((T, n, 2)) < 0.6
    d = rng.random((T, n)) < 0.05
    carry = rng.uniform(0, 0.3, (n, 2)).astype(f)
    prev0 = rng.random((n, 2)) < 0.5
    ref, _ = oracle_mod.feet_airtime_traj(c, d, carry)
    air, prev = carry.copy(), prev0.copy()
    causal = np.zeros((T, n), f)
    for t in range(T):
        rr = np.zeros(n, f)
        for sd in range(2):
            td = c[t, :, sd] & ~prev[:, sd]
            rr = (rr + (air[:, sd] - f(0.3)) * td.astype(f)).astype(f)
            air[:, sd] = np.where(c[t, :, sd] | d[t], f(0), air[:, sd] + f(0.02))
            prev[:, sd] = c[t, :, sd]
        causal[t] = rr
    np.testing.assert_array_equal(causal[1:], ref[1:])
    assert not np.array_equal(causal[0], ref[0])
