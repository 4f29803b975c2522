"""Measurement definitions shared by bench.py and the tests."""

from __future__ import annotations

from . import cstructs as cs

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md: 8.0 TB/s)
FP32_PEAK_TFLOPS = 157.3  # MI355X FP32 vector peak (MI355X_MICROARCH.md)


def bytes_per_env_step(extras: bool = False, terms: bool = True, stats: bool = True) -> int:
    """Algorithmic HBM bytes one env-step of zb_step moves, from the layouts in
    include/zbot_layout.h: the env's action row in, its state row in and out,
    its observation / reward / done outputs, and the episode-statistics
    read-modify-write. The model descriptor (11.5 KB, shared by all envs and
    cache-resident) is not counted per env."""
    f = 4
    b = cs.NJ * f  # action
    b += 2 * cs.STATE_STRIDE * f  # state row read + write
    b += (cs.OBS_ACTOR + cs.OBS_CRITIC) * f
    if extras:
        b += cs.OBS_EXTRA * f
    if terms:
        b += cs.NUM_TERMS * f
    b += f + 1  # reward (fp32) + done (u8)
    if stats:
        b += 2 * cs.NUM_STATS * f + 4  # stats read+write, solver-iteration counter
    return b
