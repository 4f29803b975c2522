""".kinfer export of the actor (reference convert.py:46-112).

kinfer 0.5.4, onnx and onnxruntime are absent, so:
  * the step function's arithmetic is pinned to the oracle's GRU actor (mode), on observations
    built by a float64 numpy restatement of convert.py:69-97 (quaternion spin, obs layout);
  * the exported ONNX graphs are read and evaluated by tests/onnx_mini.py (an independent
    protobuf reader + numpy interpreter) and must reproduce the torch module;
  * the archive layout (gzip'd tar of init_fn.onnx, step_fn.onnx, metadata.json) and tensor
    names are [U]: kinfer's own pack/runtime cannot be run here.
"""

import math

import numpy as np
import pytest
import torch

import onnx_mini
from zbot_amd import kinfer as K
from zbot_amd.policy import ACTOR, MODE, init_params


@pytest.fixture(scope="module")
def params():
    p = init_params(ACTOR, seed=11)
    rng = np.random.default_rng(3)
    # spread the mixture logits so the mode's argmax is well separated from ties
    off = K.param_count(ACTOR) - K.JOINTS - K.ACTOR_OUT
    p[off + 2 * K.JOINTS * K.MIX:off + K.ACTOR_OUT] += rng.normal(scale=2.0, size=K.JOINTS * K.MIX).astype(np.float32)
    return p


@pytest.fixture(scope="module")
def exported(params):
    return K.unpack(K.export_kinfer(params))


def _np_qmul(r, q):
    w1, x1, y1, z1 = r
    w2, x2, y2, z2 = q
    return np.array([w1 * w2 - x1 * x2 - y1 * y2 - z1 * z2, w1 * x2 + x1 * w2 + y1 * z2 - z1 * y2,
                     w1 * y2 - x1 * z2 + y1 * w2 + z1 * x2, w1 * z2 + x1 * y2 - y1 * x2 + z1 * w2])


def _np_rotate(q, r, inverse, eps=1e-6):
    """convert.py:18-40 in float64."""
    q = q / (np.linalg.norm(q) + eps)
    r = r / (np.linalg.norm(r) + eps)
    if inverse:
        r = np.concatenate([r[:1], -r[1:]])
    out = _np_qmul(r, q)
    return out / (np.linalg.norm(out) + eps)


def _np_obs(ja, jv, quat, heading, cmd):
    hq = np.array([math.cos(cmd[2] / 2), 0, 0, math.sin(cmd[2] / 2)])
    iq = np.array([math.cos(heading[0] / 2), 0, 0, math.sin(heading[0] / 2)])
    spun = _np_rotate(_np_rotate(quat, iq, True), hq, True)
    if spun[0] < 0:
        spun = -spun
    return np.concatenate([ja, jv, spun, cmd[:2], cmd[2:3], cmd[3:]])


def _inputs(rng):
    q = rng.normal(size=4)
    return (rng.uniform(-1, 1, 20), rng.normal(scale=2.0, size=20), q / np.linalg.norm(q) * rng.uniform(0.9, 1.1),
            rng.uniform(-math.pi, math.pi, 1), rng.uniform(-1, 1, 6))


def _t(xs):
    return tuple(torch.tensor(np.asarray(x), dtype=torch.float32) for x in xs)


def test_archive_layout(exported):
    init, step, meta = exported
    from zbot_amd.model import JOINT_BIASES

    assert meta == {"joint_names": [n for n, _, _ in JOINT_BIASES], "num_commands": 6, "carry_size": [5, 128]}
    gi, gs = onnx_mini.Model(init), onnx_mini.Model(step)
    assert gi.inputs == [] and gi.outputs == [("carry", [5, 128])]
    assert gs.inputs == [("joint_angles", [20]), ("joint_angular_velocities", [20]), ("quaternion", [4]),
                         ("initial_heading", [1]), ("command", [6]), ("carry", [5, 128])]
    assert gs.outputs == [("action", [20]), ("carry_out", [5, 128])]
    assert gs.opset[""] == K.OPSET
    out = gi.run({})[0]
    assert out.shape == (5, 128) and not out.any()


def test_observation_restates_convert(params):
    m = K.ActorStep(params)
    rng = np.random.default_rng(0)
    for _ in range(20):
        ja, jv, q, h, cmd = _inputs(rng)
        got = m.observation(*_t((ja, jv, q, h, cmd))).numpy()
        want = _np_obs(ja, jv, q, h, cmd)
        np.testing.assert_allclose(got, want, rtol=0, atol=2e-6)
        assert got[40] >= 0.0  # spun quaternion on the w >= 0 hemisphere (convert.py:82)


def test_step_matches_oracle_actor_mode(params, oracle_mod):
    """ActorStep == the oracle's GRU actor + mixture mode (SURVEY §8f f1 oracle) on the same
    observation, over a few steps with the carry fed back."""
    m = K.ActorStep(params)
    rng = np.random.default_rng(1)
    carry_t = torch.zeros(5, 128)
    carry_o = np.zeros((1, 5, 128), np.float32)
    for _ in range(4):
        xs = _inputs(rng)
        obs = _np_obs(*xs).astype(np.float32)
        a_o, _, carry_o = oracle_mod.policy_actor(params, obs[None, None], carry_o, mode=MODE)
        with torch.no_grad():
            a_t, carry_t = m(*_t(xs), carry_t)
        np.testing.assert_allclose(a_t.numpy(), a_o[0, 0], rtol=0, atol=2e-5)
        np.testing.assert_allclose(carry_t.numpy(), carry_o[0], rtol=0, atol=2e-5)


def test_onnx_step_evaluates_like_torch(params, exported):
    _, step, _ = exported
    g = onnx_mini.Model(step)
    m = K.ActorStep(params)
    rng = np.random.default_rng(2)
    carry = np.zeros((5, 128), np.float32)
    for _ in range(3):
        xs = _inputs(rng)
        feeds = dict(zip(K.STEP_INPUTS, [np.asarray(x, np.float32) for x in xs] + [carry]))
        a_g, c_g = g.run(feeds)
        with torch.no_grad():
            a_t, c_t = m(*_t(xs), torch.from_numpy(carry))
        np.testing.assert_allclose(a_g, a_t.numpy(), rtol=0, atol=2e-5)
        np.testing.assert_allclose(c_g, c_t.numpy(), rtol=0, atol=2e-5)
        carry = c_g.astype(np.float32)


def test_export_file_and_errors(params, tmp_path):
    p = tmp_path / "zbot.kinfer"
    blob = K.export_kinfer(params, str(p))
    assert p.read_bytes() == blob
    with pytest.raises(ValueError):
        K.export_kinfer(params[:-1])
    with pytest.raises(ValueError):
        K.metadata(["a", "b"])


def test_command_line_export(tmp_path):
    import os
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, PYTHONPATH=os.path.join(root, "ksim-gym-zbot_amd"))
    out = tmp_path / "r.kinfer"
    subprocess.run([sys.executable, "-m", "zbot_amd.kinfer", "random", str(out)], check=True, env=env,
                   capture_output=True, timeout=300)
    init, step, meta = K.unpack(out.read_bytes())
    assert meta["carry_size"] == [5, 128] and onnx_mini.Model(step).outputs[0] == ("action", [20])
