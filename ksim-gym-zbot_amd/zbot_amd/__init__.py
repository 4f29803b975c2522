"""zbot_amd — MI355X-native batched Z-Bot rollout engine (host side).

The compute path is libzbot_hip.so (HIP, gfx950) behind the C ABI in
include/zbot.h; this package compiles the robot descriptor, loads the library
through ctypes and exposes a ksim-shaped engine/task interface over PyTorch
device tensors.
"""

from . import cstructs
from .config import default_config
from .constants import JOINT_BIASES
from .model import compile_model

__all__ = ["cstructs", "default_config", "JOINT_BIASES", "compile_model"]
