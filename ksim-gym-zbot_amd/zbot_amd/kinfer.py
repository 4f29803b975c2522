"""`.kinfer` export of the GRU actor (reference convert.py:46-112).

The reference converts a checkpoint into a deployable `.kinfer` file:
  * `init_fn()` returns the zero carry [depth, hidden] (convert.py:63-67);
  * `step_fn(joint_angles, joint_angular_velocities, quaternion, initial_heading, command, carry)`
    spins the IMU quaternion by the initial heading and the commanded heading, builds the 50-float
    actor observation, runs `Actor.forward` and returns `dist.mode()` plus the new carry
    (convert.py:69-97);
  * both go through kinfer's JAX -> ONNX exporter and `pack(init, step, metadata)` with
    `PyModelMetadata(joint_names, num_commands=6, carry_size)` (convert.py:99-111).

kinfer 0.5.4 (`uv.lock:1737-1750`: a Rust-backed wheel over jax2onnx / tf2onnx) and jax are absent
here. This module re-states the two functions as torch modules over the same natural-layout
parameters that `zb_policy_create` takes (include/zbot_policy.h), exports them with torch's
TorchScript ONNX exporter, and packs them as a gzip'd tar of `init_fn.onnx`, `step_fn.onnx` and
`metadata.json`. kinfer's runtime and its exact archive layout / tensor names are not available
to check against: the layout here is [U] and is documented in DESIGN.md. The arithmetic is
pinned by tests/test_kinfer.py: the exported graph, evaluated by an independent ONNX reader, and
the torch module both reproduce the oracle's actor (mode) on the same observation.
"""

from __future__ import annotations

import contextlib
import io
import json
import tarfile
import time
import warnings

import numpy as np
import torch

from .policy import ACTOR, param_count

HIDDEN, DEPTH, MIX, JOINTS, ACTOR_IN, ACTOR_OUT = 128, 5, 5, 20, 50, 300
NUM_COMMANDS = 6  # vx, vy, heading, base height, rx, ry (convert.py:43)
OPSET = 17
STEP_INPUTS = ["joint_angles", "joint_angular_velocities", "quaternion", "initial_heading", "command", "carry"]
STEP_OUTPUTS = ["action", "carry_out"]
INIT_OUTPUTS = ["carry"]


def _split_actor(params: np.ndarray) -> dict[str, torch.Tensor]:
    p = np.ascontiguousarray(params, dtype=np.float32).ravel()
    if p.size != param_count(ACTOR):
        raise ValueError(f"actor parameters: expected {param_count(ACTOR)} floats, got {p.size}")
    H, off, out = HIDDEN, 0, {}

    def take(name, *shape):
        nonlocal off
        k = int(np.prod(shape))
        out[name] = torch.from_numpy(p[off:off + k].reshape(shape).copy())
        off += k

    take("w_in", H, ACTOR_IN)
    take("b_in", H)
    for layer in range(DEPTH):
        take(f"w_ih{layer}", 3 * H, H)
        take(f"w_hh{layer}", 3 * H, H)
        take(f"b{layer}", 3 * H)
        take(f"bn{layer}", H)
    take("w_out", ACTOR_OUT, H)
    take("b_out", ACTOR_OUT)
    take("mean_bias", JOINTS)
    assert off == p.size
    return out


def _qmul(r: torch.Tensor, q: torch.Tensor) -> torch.Tensor:
    w1, x1, y1, z1 = r[0:1], r[1:2], r[2:3], r[3:4]
    w2, x2, y2, z2 = q[0:1], q[1:2], q[2:3], q[3:4]
    return torch.cat([w1 * w2 - x1 * x2 - y1 * y2 - z1 * z2, w1 * x2 + x1 * w2 + y1 * z2 - z1 * y2,
                      w1 * y2 - x1 * z2 + y1 * w2 + z1 * x2, w1 * z2 + x1 * y2 - y1 * x2 + z1 * w2])


def _unit(q: torch.Tensor, eps: float) -> torch.Tensor:
    return q / (torch.sqrt(torch.sum(q * q, dim=0, keepdim=True)) + eps)


def rotate_quat_by_quat(q: torch.Tensor, r: torch.Tensor, inverse: bool = False, eps: float = 1e-6) -> torch.Tensor:
    """convert.py:18-40: normalise both, conjugate the rotating quaternion if `inverse`, take the
    Hamilton product rotating (x) rotated, normalise again (each norm + eps)."""
    q, r = _unit(q, eps), _unit(r, eps)
    if inverse:
        r = torch.cat([r[0:1], -r[1:4]])
    return _unit(_qmul(r, q), eps)


def yaw_quat(yaw: torch.Tensor) -> torch.Tensor:
    """xax.euler_to_quat([0, 0, yaw]) [U]: (cos(yaw/2), 0, 0, sin(yaw/2))."""
    h = 0.5 * yaw.reshape(1)
    z = torch.zeros_like(h)
    return torch.cat([torch.cos(h), z, z, torch.sin(h)])


class ActorStep(torch.nn.Module):
    """convert.py:69-97 step_fn for one robot: (action = dist.mode(), carry')."""

    def __init__(self, params: np.ndarray):
        super().__init__()
        for k, v in _split_actor(params).items():
            self.register_buffer(k, v)

    def observation(self, joint_angles, joint_angular_velocities, quaternion, initial_heading, command):
        heading_quat = yaw_quat(command[2:3])
        init_quat = yaw_quat(initial_heading)
        rel = rotate_quat_by_quat(quaternion, init_quat, inverse=True)
        spun = rotate_quat_by_quat(rel, heading_quat, inverse=True)
        spun = torch.where(spun[0:1] < 0, -spun, spun)
        return torch.cat([joint_angles, joint_angular_velocities, spun, command[0:2], command[2:3], command[3:6]])

    def forward(self, joint_angles, joint_angular_velocities, quaternion, initial_heading, command, carry):
        obs = self.observation(joint_angles, joint_angular_velocities, quaternion, initial_heading, command)
        return self.act(obs, carry)

    def act(self, obs, carry):
        """Actor.forward + dist.mode() on a 50-float observation (train.py:885-967)."""
        H = HIDDEN
        x = torch.matmul(self.w_in, obs) + self.b_in
        hs = []
        for layer in range(DEPTH):  # equinox GRUCell stack (train.py:885-967)
            h = carry[layer]
            gi = torch.matmul(getattr(self, f"w_ih{layer}"), x) + getattr(self, f"b{layer}")
            gh = torch.matmul(getattr(self, f"w_hh{layer}"), h)
            r = torch.sigmoid(gi[0:H] + gh[0:H])
            z = torch.sigmoid(gi[H:2 * H] + gh[H:2 * H])
            n = torch.tanh(gi[2 * H:3 * H] + r * (gh[2 * H:3 * H] + getattr(self, f"bn{layer}")))
            x = n + z * (h - n)
            hs.append(x)
        out = torch.matmul(self.w_out, x) + self.b_out
        mu = out[0:JOINTS * MIX].reshape(JOINTS, MIX) + self.mean_bias.reshape(JOINTS, 1)
        logits = out[2 * JOINTS * MIX:3 * JOINTS * MIX].reshape(JOINTS, MIX)
        # mixture mode: the mean of the most likely component (first on ties)
        idx = torch.argmax(logits, dim=1, keepdim=True)
        action = torch.gather(mu, 1, idx).reshape(JOINTS)
        return action, torch.stack(hs)


class ActorInit(torch.nn.Module):
    """convert.py:63-67 init_fn: the zero carry [depth, hidden]."""

    def forward(self):
        return torch.zeros(DEPTH, HIDDEN)


@contextlib.contextmanager
def _torchscript_exporter():
    """torch's TorchScript ONNX exporter serialises the graph in C++; its last pass, which splices
    custom onnxscript functions into the ModelProto, imports the `onnx` package even when there
    are none. Without `onnx` installed that pass is skipped (these graphs use standard ops only)."""
    try:
        import onnx  # noqa: F401

        have_onnx = True
    except ImportError:
        have_onnx = False
    if have_onnx:
        yield
        return
    from torch.onnx._internal.torchscript_exporter import onnx_proto_utils as U

    orig = U._add_onnxscript_fn

    def passthrough(model_bytes, custom_opsets):
        if custom_opsets:
            raise RuntimeError("custom ONNX opsets need the onnx package")
        return model_bytes

    U._add_onnxscript_fn = passthrough
    try:
        yield
    finally:
        U._add_onnxscript_fn = orig


def _export(module: torch.nn.Module, args: tuple, input_names, output_names) -> bytes:
    f = io.BytesIO()
    with _torchscript_exporter(), torch.no_grad(), warnings.catch_warnings():
        warnings.simplefilter("ignore")  # the TorchScript exporter's deprecation notices
        torch.onnx.export(module, args, f, dynamo=False, opset_version=OPSET, input_names=list(input_names),
                          output_names=list(output_names), do_constant_folding=True)
    return f.getvalue()


def step_example_inputs() -> tuple:
    return (torch.zeros(JOINTS), torch.zeros(JOINTS), torch.tensor([1.0, 0.0, 0.0, 0.0]), torch.zeros(1),
            torch.zeros(NUM_COMMANDS), torch.zeros(DEPTH, HIDDEN))


def export_onnx(params: np.ndarray) -> tuple[bytes, bytes]:
    """(init_fn.onnx, step_fn.onnx) ModelProto bytes for the actor parameters."""
    init = _export(ActorInit(), (), [], INIT_OUTPUTS)
    step = _export(ActorStep(params).eval(), step_example_inputs(), STEP_INPUTS, STEP_OUTPUTS)
    return init, step


def metadata(joint_names: list[str], num_commands: int = NUM_COMMANDS) -> dict:
    """PyModelMetadata(joint_names, num_commands, carry_size) (convert.py:99-103)."""
    if len(joint_names) != JOINTS:
        raise ValueError(f"expected {JOINTS} joint names (the hinges without the root, convert.py:60)")
    return {"joint_names": list(joint_names), "num_commands": int(num_commands), "carry_size": [DEPTH, HIDDEN]}


def pack(init_onnx: bytes, step_onnx: bytes, meta: dict) -> bytes:
    """gzip'd tar: init_fn.onnx, step_fn.onnx, metadata.json [U: kinfer.export.serialize.pack]."""
    buf = io.BytesIO()
    now = int(time.time())
    with tarfile.open(fileobj=buf, mode="w:gz") as tar:
        for name, data in (("init_fn.onnx", init_onnx), ("step_fn.onnx", step_onnx),
                           ("metadata.json", json.dumps(meta, indent=2).encode())):
            info = tarfile.TarInfo(name)
            info.size = len(data)
            info.mtime = now
            tar.addfile(info, io.BytesIO(data))
    return buf.getvalue()


def unpack(blob: bytes) -> tuple[bytes, bytes, dict]:
    with tarfile.open(fileobj=io.BytesIO(blob), mode="r:gz") as tar:
        files = {m.name: tar.extractfile(m).read() for m in tar.getmembers() if m.isfile()}
    return files["init_fn.onnx"], files["step_fn.onnx"], json.loads(files["metadata.json"])


def export_kinfer(params: np.ndarray, path: str | None = None, joint_names: list[str] | None = None) -> bytes:
    """convert.py:main for actor parameters in the natural layout (GruPolicy / zb_policy_create)."""
    if joint_names is None:
        from .model import JOINT_BIASES

        joint_names = [n for n, _, _ in JOINT_BIASES]
    init, step = export_onnx(params)
    blob = pack(init, step, metadata(joint_names))
    if path is not None:
        with open(path, "wb") as f:
            f.write(blob)
    return blob


if __name__ == "__main__":
    import argparse

    from .policy import init_params

    ap = argparse.ArgumentParser(description="export GRU actor parameters (.npy, natural layout) as .kinfer")
    ap.add_argument("params", help=".npy of the actor parameters, or 'random' for a seeded init")
    ap.add_argument("output")
    a = ap.parse_args()
    prm = init_params(ACTOR, 0) if a.params == "random" else np.load(a.params, allow_pickle=False)
    export_kinfer(prm, a.output)
    print(f"Kinfer model written to {a.output}")
