"""ctypes binding of libzbot_hip.so over PyTorch-ROCm device tensors.

This is the product path: every call goes to the HIP engine. There is no CPU
fallback — when the library or a GPU is missing, construction raises.
The C ABI is documented in include/zbot.h.
"""

from __future__ import annotations

import ctypes as C
import os

from . import cstructs as cs

LIB_NAME = "libzbot_hip.so"
ABI_VERSION = 3  # include/zbot.h: 2 added zb_step / zb_rollout's `success`, 3 the exact FeetAirtime patch
LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), LIB_NAME)
CSRC_DIR = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "csrc")

_lib: C.CDLL | None = None


class ZbError(RuntimeError):
    pass


def build_library(force: bool = False) -> str:
    """Compile libzbot_hip.so in-tree for gfx950 (hipcc; no GPU needed)."""
    import subprocess  # noqa: PLC0415

    if force and os.path.exists(LIB_PATH):
        os.remove(LIB_PATH)
    subprocess.run(["make", "-C", CSRC_DIR, "-s"], check=True)  # no-op when up to date
    return LIB_PATH


def load_library(path: str | None = None) -> C.CDLL:
    """Load the engine library; raises if it has not been built.

    `path` selects another build of the same sources (the -DZB_STAMPS
    diagnostic library used by tests/diag_stamps.py)."""
    global _lib
    if path is None and _lib is not None:
        return _lib
    lp = path or LIB_PATH
    if not os.path.exists(lp):
        raise ZbError(f"{lp} not found: build it with `make -C {CSRC_DIR}` (or __graft_entry__.build())")
    L = C.CDLL(lp)
    vp = C.c_void_p
    L.zb_abi_version.restype = C.c_int
    L.zb_model_struct_bytes.restype = C.c_size_t
    L.zb_config_struct_bytes.restype = C.c_size_t
    L.zb_state_stride.restype = C.c_int
    L.zb_rand_stride.restype = C.c_int
    L.zb_last_error.restype = C.c_char_p
    L.zb_default_config.argtypes = [C.POINTER(cs.ZbEnvConfig)]
    L.zb_create.argtypes = [C.POINTER(cs.ZbModel), C.POINTER(cs.ZbEnvConfig), C.c_int, C.c_int, C.c_int, C.c_uint64,
                            C.POINTER(vp)]
    L.zb_destroy.argtypes = [vp]
    L.zb_reset.argtypes = [vp, vp, vp, vp, vp, vp]
    L.zb_step.argtypes = [vp, vp, vp, vp, vp, vp, vp, vp, vp, C.c_float, vp]
    L.zb_rollout.argtypes = [vp, vp, C.c_int, vp, vp, vp, vp, vp, C.c_float, vp]
    for f in ("zb_get_state", "zb_set_state", "zb_get_rand", "zb_set_rand", "zb_get_solver_iters"):
        getattr(L, f).argtypes = [vp, vp, vp]
    L.zb_get_stats.argtypes = [vp, vp, C.c_int, vp]
    L.zb_set_step_chunks.argtypes = [vp, C.c_int]
    L.zb_debug_forward.argtypes = [vp, vp, vp, vp, vp]
    L.zb_mark_rollout_start.argtypes = [vp]
    L.zb_check.argtypes = [vp]
    L.zb_feet_airtime_exact.argtypes = [vp, vp, vp, C.c_float, vp]
    for f in ("zb_create", "zb_destroy", "zb_reset", "zb_step", "zb_rollout", "zb_get_state", "zb_set_state",
              "zb_get_rand", "zb_set_rand", "zb_get_stats", "zb_get_solver_iters", "zb_debug_forward",
              "zb_set_step_chunks", "zb_mark_rollout_start", "zb_feet_airtime_exact", "zb_check"):
        getattr(L, f).restype = C.c_int
    # post-rollout PPO inputs (include/zbot_ppo.h)
    L.zb_gae_partials_words.argtypes = [C.c_int]
    L.zb_gae_partials_words.restype = C.c_size_t
    L.zb_gae.argtypes = [vp, vp, vp, vp, vp, C.c_int, C.c_int, C.c_float, C.c_float, vp, vp, vp, vp, vp]
    L.zb_moments_combine.argtypes = [vp, C.c_int, vp, vp]
    L.zb_adv_normalize.argtypes = [vp, vp, C.c_longlong, vp, C.c_double, C.c_float, vp]
    for f in ("zb_gae", "zb_moments_combine", "zb_adv_normalize"):
        getattr(L, f).restype = C.c_int
    # GRU actor / critic (include/zbot_policy.h)
    L.zb_policy_param_count.argtypes = [C.c_int]
    L.zb_policy_param_count.restype = C.c_size_t
    L.zb_policy_create.argtypes = [C.c_int, C.POINTER(C.c_float), C.c_size_t, C.c_int, C.POINTER(vp)]
    L.zb_policy_destroy.argtypes = [vp]
    L.zb_policy_actor.argtypes = [vp, vp, C.c_int, C.c_int, vp, vp, C.c_int, C.c_uint64, C.c_int, C.c_uint32, vp, vp,
                                  vp]
    L.zb_policy_critic.argtypes = [vp, vp, C.c_int, C.c_int, vp, vp, vp, vp]
    L.zb_policy_set_layout.argtypes = [vp, C.c_int]
    L.zb_policy_set_persistent.argtypes = [vp, C.c_int]
    for f in ("zb_policy_create", "zb_policy_destroy", "zb_policy_actor", "zb_policy_critic", "zb_policy_set_layout",
              "zb_policy_set_persistent"):
        getattr(L, f).restype = C.c_int
    if L.zb_abi_version() != ABI_VERSION:
        raise ZbError(f"{lp}: ABI version {L.zb_abi_version()}, this binding speaks {ABI_VERSION}: rebuild it")
    if L.zb_model_struct_bytes() != C.sizeof(cs.ZbModel):
        raise ZbError("ZbModel layout mismatch between cstructs.py and the library")
    if L.zb_config_struct_bytes() != C.sizeof(cs.ZbEnvConfig):
        raise ZbError("ZbEnvConfig layout mismatch between cstructs.py and the library")
    if path is None:
        _lib = L
    return L


def _check(rc: int) -> None:
    if rc != 0:
        raise ZbError(f"libzbot_hip error {rc}: {load_library().zb_last_error().decode()}")


def _ptr(t) -> int | None:
    return None if t is None else t.data_ptr()


DBG_STRIDE = 1760
DBG = dict(qM=0, bias=1024, qacc_smooth=1056, qacc=1088, xpos=1120, cinert=1216, cvel=1536, misc=1728)


def state_flags(state) -> dict:
    """The sticky diagnostic flags of a [n, ZB_STATE_STRIDE] state (get_state()), as boolean [n]
    tensors (include/zbot_layout.h ZB_S_NAN): `nonfinite` - the env's state went non-finite;
    `bank_overflow` - in some substep more colliders beyond the soles were within reach of the floor
    than the contact-row banks hold (four; two beside the sole pair), and the extra ones' contacts were
    not simulated (zb_engine.hip select_bank2).
    Both are sticky for the life of the env's state row (resets keep them; set_state() can clear
    them). `bank_overflow_step`: the same overflow in the last control step alone (the kernel clears
    it at the start of every step), so the step that ends an episode still shows it. Works on CPU or
    device tensors."""
    import torch

    bits = state[:, cs.S_NAN].contiguous().view(torch.int32)
    return {"nonfinite": (bits & cs.NAN_NONFINITE) != 0, "bank_overflow": (bits & cs.NAN_BANK_OVERFLOW) != 0,
            "bank_overflow_step": (bits & cs.NAN_BANK_OVERFLOW_STEP) != 0}


class HipEngine:
    """N Z-Bot environments on one GPU (one handle)."""

    def __init__(self, model, cfg: cs.ZbEnvConfig, n_envs: int, env_offset: int = 0, device: int = 0,
                 seed: int = 0, lib_path: str | None = None):
        import torch  # noqa: PLC0415

        if not torch.cuda.is_available():
            raise ZbError("HipEngine needs a ROCm GPU (torch.cuda.is_available() is False)")
        self.torch = torch
        self.L = load_library(lib_path)
        self.cmodel = model.cmodel if hasattr(model, "cmodel") else model
        self.cfg = cfg
        self.n = n_envs
        self.env_offset = env_offset
        self.device = torch.device("cuda", device)
        self.seed = seed
        h = C.c_void_p()
        _check(self.L.zb_create(C.byref(self.cmodel), C.byref(cfg), n_envs, env_offset, device, seed, C.byref(h)))
        self.h = h
        f32 = dict(dtype=torch.float32, device=self.device)
        self.obs_actor = torch.zeros(n_envs, cs.OBS_ACTOR, **f32)
        self.obs_critic = torch.zeros(n_envs, cs.OBS_CRITIC, **f32)
        self.obs_extra = torch.zeros(n_envs, cs.OBS_EXTRA, **f32)
        self.reward_terms = torch.zeros(n_envs, cs.NUM_TERMS, **f32)
        self.reward = torch.zeros(n_envs, **f32)
        self.done = torch.zeros(n_envs, dtype=torch.uint8, device=self.device)
        self.success = torch.zeros(n_envs, dtype=torch.uint8, device=self.device)

    def __del__(self):
        h = getattr(self, "h", None)
        if h is not None and h.value:
            try:
                self.L.zb_destroy(h)
            except Exception:  # noqa: BLE001
                pass
            self.h = None

    def _stream(self) -> int:
        return self.torch.cuda.current_stream(self.device).cuda_stream

    def outputs(self) -> dict:
        return dict(obs_actor=self.obs_actor, obs_critic=self.obs_critic, obs_extra=self.obs_extra,
                    reward_terms=self.reward_terms, reward=self.reward, done=self.done, success=self.success)

    def reset(self, mask=None, extras: bool = True) -> dict:
        m = None
        if mask is not None:
            m = mask.to(device=self.device, dtype=self.torch.uint8).contiguous()
        _check(self.L.zb_reset(self.h, _ptr(m), _ptr(self.obs_actor), _ptr(self.obs_critic),
                               _ptr(self.obs_extra) if extras else None, self._stream()))
        return self.outputs()

    def step(self, action, curriculum: float = 1.0, extras: bool = True, terms: bool = True, reward=None,
             done=None) -> dict:
        """One control step of every env. reward [n] / done [n] (optional): write those two outputs
        there instead of the engine's buffers (a row of a [T, n] rollout buffer, no copy)."""
        a = action
        if a.dtype != self.torch.float32 or not a.is_contiguous() or a.device != self.device:
            a = a.to(device=self.device, dtype=self.torch.float32).contiguous()
        if tuple(a.shape) != (self.n, cs.NJ):
            raise ZbError(f"action must be [{self.n}, {cs.NJ}], got {tuple(a.shape)}")
        if reward is not None:
            self._check_out(reward, "reward", (self.n,), self.torch.float32)
        if done is not None:
            self._check_out(done, "done", (self.n,), self.torch.uint8)
        _check(self.L.zb_step(self.h, _ptr(a), _ptr(self.obs_actor), _ptr(self.obs_critic),
                              _ptr(self.obs_extra) if extras else None, _ptr(self.reward_terms) if terms else None,
                              _ptr(self.reward if reward is None else reward),
                              _ptr(self.done if done is None else done), _ptr(self.success), float(curriculum),
                              self._stream()))
        return self.outputs()

    def _check_out(self, t, name: str, shape: tuple, dtype) -> None:
        """An output buffer the kernel writes through its raw pointer: exact shape, dtype, device, contiguity."""
        if (tuple(t.shape) != shape or t.dtype != dtype or t.device != self.device or not t.is_contiguous()):
            raise ZbError(f"{name} must be a contiguous {dtype} {list(shape)} tensor on {self.device}, got "
                          f"{t.dtype} {list(t.shape)} on {t.device}")

    def rollout(self, actions, curriculum: float = 1.0, reward_sum=None) -> dict:
        a = actions.to(device=self.device, dtype=self.torch.float32).contiguous()
        T = a.shape[0]
        if a.dim() != 3 or tuple(a.shape) != (T, self.n, cs.NJ) or T < 1:
            raise ZbError("actions must be [T, n_envs, 20] with T >= 1")
        if reward_sum is not None:
            self._check_out(reward_sum, "reward_sum", (self.n,), self.torch.float32)
        _check(self.L.zb_rollout(self.h, _ptr(a), T, _ptr(self.obs_actor), _ptr(self.obs_critic), _ptr(reward_sum),
                                 _ptr(self.done), _ptr(self.success), float(curriculum), self._stream()))
        return self.outputs()

    def join(self) -> None:
        """Nothing to join: one handle runs on the caller's current stream (EnvGroups.join's twin)."""

    def mark_rollout_start(self) -> None:
        """The next step() / rollout() is step 0 of a rollout (zb_mark_rollout_start): it saves what
        feet_airtime_exact() needs to give ksim's FeetAirtime row 0."""
        _check(self.L.zb_mark_rollout_start(self.h))

    def feet_airtime_exact(self, reward0=None, terms0=None, curriculum: float = 1.0) -> None:
        """After the last step of a marked rollout: patch row 0 to ksim's FeetAirtimeReward
        (prev contact False at t = 0, airtime roll(air, 1) -> air[T-1]; train.py:515-546).
        reward0 [n] gets scale * (ksim term - causal term) added, terms0 [n, 12] (nullable) its
        FeetAirtime slot overwritten. Rows t >= 1 of the fused step are already ksim's."""
        if reward0 is not None:
            self._check_out(reward0, "reward0", (self.n,), self.torch.float32)
        if terms0 is not None:
            self._check_out(terms0, "terms0", (self.n, cs.NUM_TERMS), self.torch.float32)
        _check(self.L.zb_feet_airtime_exact(self.h, _ptr(reward0), _ptr(terms0), float(curriculum), self._stream()))

    def get_state(self):
        out = self.torch.empty(self.n, cs.STATE_STRIDE, dtype=self.torch.float32, device=self.device)
        _check(self.L.zb_get_state(self.h, _ptr(out), self._stream()))
        return out

    def flags(self) -> dict:
        """state_flags(get_state()): per-env boolean `nonfinite` and `bank_overflow` [n]."""
        return state_flags(self.get_state())

    def set_state(self, state) -> None:
        s = state.to(device=self.device, dtype=self.torch.float32).contiguous()
        if tuple(s.shape) != (self.n, cs.STATE_STRIDE):
            raise ZbError("state must be [n_envs, ZB_STATE_STRIDE]")
        _check(self.L.zb_set_state(self.h, _ptr(s), self._stream()))
        self.torch.cuda.current_stream(self.device).synchronize()

    def get_rand(self):
        out = self.torch.empty(self.n, cs.RAND_STRIDE, dtype=self.torch.float32, device=self.device)
        _check(self.L.zb_get_rand(self.h, _ptr(out), self._stream()))
        return out

    def set_rand(self, rand) -> None:
        r = rand.to(device=self.device, dtype=self.torch.float32).contiguous()
        if tuple(r.shape) != (self.n, cs.RAND_STRIDE):
            raise ZbError(f"rand must be [n_envs, ZB_RAND_STRIDE] = [{self.n}, {cs.RAND_STRIDE}], got {tuple(r.shape)}")
        _check(self.L.zb_set_rand(self.h, _ptr(r), self._stream()))
        self.torch.cuda.current_stream(self.device).synchronize()

    def get_stats(self, clear: bool = False):
        out = self.torch.empty(self.n, cs.NUM_STATS, dtype=self.torch.float32, device=self.device)
        _check(self.L.zb_get_stats(self.h, _ptr(out), int(clear), self._stream()))
        return out

    def set_step_chunks(self, k: int) -> None:
        """Work units per pair of envs in step() (0: the automatic choice, 1: whole control steps;
        DESIGN.md §4e). The same bits for every k."""
        _check(self.L.zb_set_step_chunks(self.h, int(k)))

    def check(self) -> None:
        """Synchronise and raise ZbError if a launch since the last check flagged its results
        invalid (zb_check: a chunked step's bounded hand-off wait timed out)."""
        _check(self.L.zb_check(self.h))

    def solver_iters(self):
        out = self.torch.empty(self.n, dtype=self.torch.int32, device=self.device)
        _check(self.L.zb_get_solver_iters(self.h, _ptr(out), self._stream()))
        return out

    def debug_forward(self, state, ctrl=None):
        s = state.to(device=self.device, dtype=self.torch.float32).contiguous()
        c = None if ctrl is None else ctrl.to(device=self.device, dtype=self.torch.float32).contiguous()
        out = self.torch.zeros(self.n, DBG_STRIDE, dtype=self.torch.float32, device=self.device)
        _check(self.L.zb_debug_forward(self.h, _ptr(s), _ptr(c), _ptr(out), self._stream()))
        return out


_GROUP_STREAMS: dict = {}


def group_streams(torch, device, k: int, priority: int = 0) -> list:
    """The first k of the process's env-group streams on `device`, shared by every EnvGroups.

    HIP runs a process's streams on a few hardware queues (GPU_MAX_HW_QUEUES, 4 by default) and
    assigns them round-robin as streams are created. Two groups whose streams land on one queue
    run in series, and the actor-in-the-loop then ran at 4.6 M env-steps/s instead of 6.8 M
    (DESIGN.md §4f). Reusing one set of streams keeps the count at the largest group count, so
    up to three groups, plus the caller's stream, get a queue each."""
    lst = _GROUP_STREAMS.setdefault((device.index, priority), [])
    while len(lst) < k:
        lst.append(torch.cuda.Stream(device=device, priority=priority))
    return lst[:k]


def group_bounds(n_envs: int, groups: int) -> list[tuple[int, int]]:
    """Consecutive env ranges of EnvGroups: cut on even env indices (whole pairs of envs, one wave
    each) where that leaves every group non-empty, else evenly."""
    if groups < 1 or n_envs < groups:
        raise ZbError(f"need 1 <= groups <= n_envs, got groups={groups}, n_envs={n_envs}")
    cuts = [0] + [min(n_envs, 2 * ((n_envs * g // groups + 1) // 2)) for g in range(1, groups)] + [n_envs]
    if any(b <= a for a, b in zip(cuts[:-1], cuts[1:])):
        cuts = [n_envs * g // groups for g in range(groups + 1)]
    return list(zip(cuts[:-1], cuts[1:]))


class EnvGroups:
    """N envs on one GPU as G engine handles over consecutive env ranges, each stepping on its own
    HIP stream.

    A zb_step launch ends in a drain: its last round of waves finishes ragged, and the next launch
    cannot start before the slowest pair of envs is done. With G groups, step t of group g waits
    only on step t - 1 of group g, so the other group's waves fill the slots the drain frees. Every
    group keeps the global env ids of its range (env_offset), so each env's RNG streams, and with
    them the results, are bit-identical to one handle over all N envs, as for the shards of a
    multi-GPU run.

    The outputs are views into full [N, ...] buffers. step() returns them pending: work on the
    caller's stream that reads them must come after join(), which makes the current stream wait
    for every group's last launch. Calls that read or write engine state (reset, get_state, ...)
    join first and run on the current stream; the next step() orders every group after them.

    The group streams come from one per-process set (group_streams). With HIP's default of four
    hardware queues per process, up to three groups and the caller's stream get a queue each;
    more groups share queues and run partly in series."""

    OUTPUTS = ("obs_actor", "obs_critic", "obs_extra", "reward_terms", "reward", "done", "success")

    def __init__(self, model, cfg: cs.ZbEnvConfig, n_envs: int, groups: int = 2, env_offset: int = 0,
                 device: int = 0, seed: int = 0, lib_path: str | None = None, priority: int = 0,
                 chunks: int = 1):
        import torch  # noqa: PLC0415

        self.torch = torch
        self.n = n_envs
        self.env_offset = env_offset
        self.G = groups
        self.bounds = group_bounds(n_envs, groups)
        self.engines = [HipEngine(model, cfg, b - a, env_offset=env_offset + a, device=device, seed=seed,
                                  lib_path=lib_path) for a, b in self.bounds]
        # the groups fill each other's drains, so a partial last round needs no chunking (§4e);
        # chunks=0 keeps zb_create's automatic choice
        for e in self.engines:
            e.set_step_chunks(chunks)
        e0 = self.engines[0]
        self.L, self.device, self.cfg, self.seed = e0.L, e0.device, cfg, seed
        for name in self.OUTPUTS:
            t = getattr(e0, name)
            full = torch.zeros((n_envs,) + tuple(t.shape[1:]), dtype=t.dtype, device=self.device)
            setattr(self, name, full)
            for e, (a, b) in zip(self.engines, self.bounds):
                setattr(e, name, full[a:b])
        # priority < 0: high-priority group streams (torch.cuda.Stream priority)
        self.streams = group_streams(torch, self.device, groups, priority)
        self._tail = [None] * groups  # each group's last enqueued event
        # events are re-recorded, not created per step: a stream wait captures the event's record
        # at the time the wait is enqueued (CUDA / HIP semantics), so reuse is safe, and no
        # hipEventCreate / Destroy pair runs per step and group
        self._fork_ev = torch.cuda.Event()
        self._mark_ev = [torch.cuda.Event() for _ in range(groups)]

    def groups(self):
        """(engine, stream, env range) of every group."""
        return list(zip(self.engines, self.streams, self.bounds))

    def outputs(self) -> dict:
        return {k: getattr(self, k) for k in self.OUTPUTS}

    def fork(self) -> None:
        """Order every group stream after the work enqueued so far on the current stream."""
        ev = self._fork_ev
        ev.record(self.torch.cuda.current_stream(self.device))
        for s in self.streams:
            s.wait_event(ev)

    def mark(self, g: int) -> None:
        """Record group g's tail (after the work just enqueued on its stream)."""
        ev = self._mark_ev[g]
        ev.record(self.streams[g])
        self._tail[g] = ev

    def join(self) -> None:
        """Make the current stream wait for every group's enqueued work."""
        cur = self.torch.cuda.current_stream(self.device)
        for ev in self._tail:
            if ev is not None:
                cur.wait_event(ev)

    def step(self, action, curriculum: float = 1.0, extras: bool = True, terms: bool = True, events=None,
             reward=None, done=None) -> dict:
        """events: optional per-group (start, end) torch.cuda.Event pairs recorded around each group's
        launch on its stream (bench.py's per-launch timing). reward [n] / done [n]: as HipEngine.step
        (each group writes its slice; pending until join())."""
        a = action
        if a.dtype != self.torch.float32 or not a.is_contiguous() or a.device != self.device:
            a = a.to(device=self.device, dtype=self.torch.float32).contiguous()
        if tuple(a.shape) != (self.n, cs.NJ):
            raise ZbError(f"action must be [{self.n}, {cs.NJ}], got {tuple(a.shape)}")
        self.fork()
        for s in self.streams:
            # the group streams read `a` (and write reward / done) after step() returns (no join):
            # keep those blocks from being reused on the caller's stream before they are done
            for t in (a, reward, done):
                if t is not None:
                    t.record_stream(s)
        for g, (e, s, (lo, hi)) in enumerate(self.groups()):
            with self.torch.cuda.stream(s):
                if events is not None:
                    events[g][0].record(s)
                e.step(a[lo:hi], curriculum=curriculum, extras=extras, terms=terms,
                       reward=None if reward is None else reward[lo:hi], done=None if done is None else done[lo:hi])
                if events is not None:
                    events[g][1].record(s)
            self.mark(g)
        return self.outputs()

    def rollout(self, actions, curriculum: float = 1.0, reward_sum=None) -> dict:
        a = actions.to(device=self.device, dtype=self.torch.float32).contiguous()
        if a.dim() != 3 or tuple(a.shape[1:]) != (self.n, cs.NJ):
            raise ZbError("actions must be [T, n_envs, 20] with T >= 1")
        if reward_sum is not None:
            self.engines[0]._check_out(reward_sum, "reward_sum", (self.n,), self.torch.float32)
        self.fork()
        for g, (e, s, (lo, hi)) in enumerate(self.groups()):
            with self.torch.cuda.stream(s):
                part = a[:, lo:hi].contiguous()  # allocated on the group stream
                a.record_stream(s)
                e.rollout(part, curriculum=curriculum,
                          reward_sum=None if reward_sum is None else reward_sum[lo:hi])
            self.mark(g)
        return self.outputs()

    def mark_rollout_start(self) -> None:
        """Every group's next step is step 0 of a rollout (HipEngine.mark_rollout_start)."""
        for e in self.engines:
            e.mark_rollout_start()

    def feet_airtime_exact(self, reward0=None, terms0=None, curriculum: float = 1.0) -> None:
        """HipEngine.feet_airtime_exact per group, on the group's stream after its last step;
        reward0 [n] / terms0 [n, 12] are the rollout's row-0 buffers (nullable). Pending like step().
        The group streams first wait for the caller's stream (fork): the row-0 buffers may have been
        written there after the last step() (e.g. a trajectory stacked after the loop)."""
        self.fork()
        for s in self.streams:
            for t in (reward0, terms0):
                if t is not None:
                    t.record_stream(s)
        for g, (e, s, (lo, hi)) in enumerate(self.groups()):
            with self.torch.cuda.stream(s):
                e.feet_airtime_exact(None if reward0 is None else reward0[lo:hi],
                                     None if terms0 is None else terms0[lo:hi], curriculum=curriculum)
            self.mark(g)

    def _each(self, fn):
        self.join()
        return [fn(e, lo, hi) for e, (lo, hi) in zip(self.engines, self.bounds)]

    def reset(self, mask=None, extras: bool = True) -> dict:
        m = None if mask is None else mask.to(device=self.device, dtype=self.torch.uint8).contiguous()
        self._each(lambda e, lo, hi: e.reset(None if m is None else m[lo:hi], extras=extras))
        return self.outputs()

    def flags(self) -> dict:
        """state_flags(get_state()) over all groups' envs (HipEngine.flags)."""
        return state_flags(self.get_state())

    def get_state(self):
        return self.torch.cat(self._each(lambda e, lo, hi: e.get_state()))

    def set_state(self, state) -> None:
        s = state.to(device=self.device, dtype=self.torch.float32).contiguous()
        if tuple(s.shape) != (self.n, cs.STATE_STRIDE):
            raise ZbError("state must be [n_envs, ZB_STATE_STRIDE]")
        self._each(lambda e, lo, hi: e.set_state(s[lo:hi]))

    def get_rand(self):
        return self.torch.cat(self._each(lambda e, lo, hi: e.get_rand()))

    def set_rand(self, rand) -> None:
        r = rand.to(device=self.device, dtype=self.torch.float32).contiguous()
        if tuple(r.shape) != (self.n, cs.RAND_STRIDE):
            raise ZbError(f"rand must be [n_envs, ZB_RAND_STRIDE] = [{self.n}, {cs.RAND_STRIDE}], got {tuple(r.shape)}")
        self._each(lambda e, lo, hi: e.set_rand(r[lo:hi]))

    def get_stats(self, clear: bool = False):
        return self.torch.cat(self._each(lambda e, lo, hi: e.get_stats(clear=clear)))

    def solver_iters(self):
        return self.torch.cat(self._each(lambda e, lo, hi: e.solver_iters()))

    def check(self) -> None:
        self._each(lambda e, lo, hi: e.check())
