"""Post-rollout PPO inputs on the GPU.

Mirrors ksim 0.1.99's ``compute_ppo_inputs`` (un-vendored ksim/task/ppo.py
[U]) — the step PPOTask runs on a finished rollout, after get_ppo_variables
(train.py:1683-1729) has produced the critic values:

    inputs = compute_ppo_inputs(values_t, rewards_t, dones_t, successes_t,
                                decay_gamma=0.99, gae_lambda=0.95,
                                normalize_advantages=True)
    inputs.advantages_t, inputs.value_targets_t, inputs.gae_t, inputs.returns_t

All arrays are [T, n] torch device tensors, time-major with the env axis
contiguous — the buffers zb_step fills when handed row t of a rollout buffer.
The arithmetic runs in libzbot_hip.so (include/zbot_ppo.h); there is no
PyTorch or CPU fallback.

Multi-GPU: each rank holds its own envs. The advantage mean/std are global:
every rank's (sum, sum of squares) is all-gathered (RCCL over xGMI; gloo on
CPU in the tests) and combined in rank order by the same pairwise tree the
kernel uses, so normalized advantages are bit-identical on every rank and —
for power-of-two env counts per rank — independent of the world size.
"""

from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

from .engine import ZbError, _check, load_library

DEFAULT_GAMMA = 0.99  # ksim PPOConfig.gamma default [U]
DEFAULT_LAMBDA = 0.95  # ksim PPOConfig.lam default [U]
ADV_EPS = 1e-6  # (gae - mean) / (std + 1e-6) [U]


@dataclass
class PPOInputs:
    advantages_t: object
    value_targets_t: object
    gae_t: object
    returns_t: object


def _stream(torch, dev) -> int:
    return torch.cuda.current_stream(dev).cuda_stream


def _as(t, dtype, dev, torch):
    if t is None:
        return None
    if t.dtype != dtype or t.device != dev or not t.is_contiguous():
        t = t.to(device=dev, dtype=dtype).contiguous()
    return t


def gae(rewards_t, values_t, dones_t, decay_gamma: float = DEFAULT_GAMMA, gae_lambda: float = DEFAULT_LAMBDA,
        successes_t=None, bootstrap=None, with_moments: bool = True):
    """GAE + value targets on the GPU -> (gae [T, n], value_targets [T, n], moments [2] fp64 or None)."""
    import torch  # noqa: PLC0415

    L = load_library()
    dev = values_t.device
    if dev.type != "cuda":
        raise ZbError("ppo.gae runs on the GPU (libzbot_hip.so); got tensors on " + str(dev))
    T, n = values_t.shape
    rewards_t = _as(rewards_t, torch.float32, dev, torch)
    values_t = _as(values_t, torch.float32, dev, torch)
    dones_t = _as(dones_t, torch.uint8, dev, torch)
    successes_t = _as(successes_t, torch.uint8, dev, torch)
    bootstrap = _as(bootstrap, torch.float32, dev, torch)
    for name, t in (("rewards_t", rewards_t), ("dones_t", dones_t), ("successes_t", successes_t)):
        if t is not None and tuple(t.shape) != (T, n):
            raise ZbError(f"{name} must be [{T}, {n}], got {tuple(t.shape)}")
    if bootstrap is not None and tuple(bootstrap.shape) != (n,):
        raise ZbError(f"bootstrap must be [{n}]")
    g = torch.empty(T, n, dtype=torch.float32, device=dev)
    vt = torch.empty(T, n, dtype=torch.float32, device=dev)
    part = mom = None
    if with_moments:
        part = torch.empty(max(int(L.zb_gae_partials_words(n)), 2), dtype=torch.float64, device=dev)
        mom = torch.empty(2, dtype=torch.float64, device=dev)
    p = lambda t: None if t is None else t.data_ptr()  # noqa: E731
    _check(L.zb_gae(p(rewards_t), p(values_t), p(dones_t), p(successes_t), p(bootstrap), T, n,
                    C.c_float(decay_gamma), C.c_float(gae_lambda), p(g), p(vt), p(part), p(mom),
                    _stream(torch, dev)))
    return g, vt, mom


def pairwise_tree_host(pairs):
    """The kernel's rank-combine tree on host fp64 values ([k, 2] -> [2]); used for CPU (gloo) tensors."""
    import torch  # noqa: PLC0415

    a = [[float(x[0]), float(x[1])] for x in pairs.tolist()]
    p = 1
    while p < len(a):
        p <<= 1
    a += [[0.0, 0.0]] * (p - len(a))
    s = 1
    while s < p:
        for i in range(0, p - s, 2 * s):
            a[i] = [a[i][0] + a[i + s][0], a[i][1] + a[i + s][1]]
        s <<= 1
    return torch.tensor(a[0] if a else [0.0, 0.0], dtype=torch.float64)


def combine_moments(moments, group=None):
    """Global (sum, sum^2) from per-rank moments: all-gather + rank-order pairwise tree (every rank)."""
    import torch  # noqa: PLC0415
    import torch.distributed as dist  # noqa: PLC0415

    if not dist.is_available() or not dist.is_initialized() or dist.get_world_size(group) == 1:
        return moments
    world = dist.get_world_size(group)
    parts = [torch.zeros_like(moments) for _ in range(world)]
    dist.all_gather(parts, moments, group=group)
    stacked = torch.stack(parts).contiguous()
    if stacked.device.type != "cuda":
        # gloo on CPU tensors: the same tree on the host, handed back on the caller's device
        return pairwise_tree_host(stacked).to(moments.device)
    out = torch.empty(2, dtype=torch.float64, device=stacked.device)
    _check(load_library().zb_moments_combine(stacked.data_ptr(), world, out.data_ptr(),
                                             _stream(torch, stacked.device)))
    return out


def global_count(local: int, group=None) -> int:
    import torch.distributed as dist  # noqa: PLC0415

    if not dist.is_available() or not dist.is_initialized() or dist.get_world_size(group) == 1:
        return local
    import torch  # noqa: PLC0415

    t = torch.tensor([local], dtype=torch.int64)
    if dist.get_backend(group) == "nccl":
        t = t.cuda()
    dist.all_reduce(t, group=group)
    return int(t.item())


def normalize(gae_t, moments, total: float, eps: float = ADV_EPS, out=None):
    """(gae - mean) / (std + eps) with mean/std from global moments over `total` elements."""
    import torch  # noqa: PLC0415

    dev = gae_t.device
    if dev.type != "cuda":
        raise ZbError("ppo.normalize runs on the GPU (libzbot_hip.so)")
    if (not isinstance(moments, torch.Tensor) or moments.dtype != torch.float64 or moments.numel() != 2
            or moments.device != dev or not moments.is_contiguous()):
        # the kernel dereferences moments[0..1] on the device: a host pointer would fault the GPU
        raise ZbError(f"moments must be a contiguous float64 tensor of 2 elements on {dev}")
    if gae_t.dtype != torch.float32 or not gae_t.is_contiguous():
        raise ZbError("gae_t must be a contiguous float32 tensor")
    if out is None:
        out = torch.empty_like(gae_t)
    elif (out.dtype != torch.float32 or out.device != dev or not out.is_contiguous()
          or out.numel() != gae_t.numel()):
        raise ZbError(f"out must be a contiguous float32 tensor of {gae_t.numel()} elements on {dev}")
    _check(load_library().zb_adv_normalize(gae_t.data_ptr(), out.data_ptr(), gae_t.numel(), moments.data_ptr(),
                                           float(total), C.c_float(eps), _stream(torch, dev)))
    return out


def compute_ppo_inputs(values_t, rewards_t, dones_t, successes_t=None, decay_gamma: float = DEFAULT_GAMMA,
                       gae_lambda: float = DEFAULT_LAMBDA, normalize_advantages: bool = True,
                       monte_carlo_returns: bool = False, bootstrap=None, group=None) -> PPOInputs:
    """ksim-shaped entry point (argument names follow ksim's compute_ppo_inputs [U])."""
    if monte_carlo_returns:
        raise ZbError("monte_carlo_returns is not built (ksim's default is False [U])")
    g, vt, mom = gae(rewards_t, values_t, dones_t, decay_gamma, gae_lambda, successes_t, bootstrap,
                     with_moments=normalize_advantages)
    adv = g
    if normalize_advantages:
        gm = combine_moments(mom, group)
        total = global_count(g.numel(), group)
        adv = normalize(g, gm, total)
    return PPOInputs(advantages_t=adv, value_targets_t=vt, gae_t=g, returns_t=vt)
