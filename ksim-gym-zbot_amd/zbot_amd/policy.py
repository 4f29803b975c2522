"""GRU actor / critic of ZbotWalkingTask in the rollout loop.

Mirrors train.py's Model (Actor :885-967, Critic :970-1023, get_model
:1604-1614) and ZbotWalkingTask.run_actor / run_critic / sample_action
(:1616-1681, :1737-1763). The networks run in libzbot_hip.so on the f32
matrix cores (include/zbot_policy.h); there is no PyTorch or CPU fallback.

    actor = GruPolicy(ACTOR, init_params(ACTOR, seed=0))
    carry = actor.initial_carry(n)                          # get_initial_model_carry
    actions, log_prob = actor.actor(obs_actor, carry, reset=done, log_prob=True)   # sample_action
    critic = GruPolicy(CRITIC, init_params(CRITIC, seed=1))
    values = critic.critic(obs_critic_t, critic.initial_carry(n), reset=resets_t)  # [T, n]
    (obs_critic_t[t] is the observation of the state acted in at step t; PolicyRollout records it)

`PolicyRollout` is ksim's rollout loop with the actor in it: per control step
one actor launch then one zb_step launch, rows written straight into [T, n]
buffers on the GPU.
"""

from __future__ import annotations

import contextlib
import ctypes as C

import numpy as np

from .constants import JOINT_BIASES
from .engine import ZbError, _check, load_library

HIDDEN, DEPTH, MIXTURES, JOINTS = 128, 5, 5, 20
ACTOR_IN, CRITIC_IN, ACTOR_OUT = 50, 484, 300
ACTOR, CRITIC = 0, 1
SAMPLE, MODE, EVAL = 0, 1, 2
LAYOUT_BLOCK, LAYOUT_WAVE, LAYOUT_WAVE2, LAYOUT_WAVE4 = 0, 1, 2, 3  # include/zbot_policy.h ZB_POL_LAYOUT_*
# matrix-core FLOP per env per step (FMA = 2): the roofline unit bench.py reports
FLOP_ACTOR = 2 * (ACTOR_IN * HIDDEN + DEPTH * 6 * HIDDEN * HIDDEN + HIDDEN * ACTOR_OUT)
FLOP_CRITIC = 2 * (CRITIC_IN * HIDDEN + DEPTH * 6 * HIDDEN * HIDDEN + HIDDEN)


def _dims(kind: int) -> tuple[int, int]:
    if kind == ACTOR:
        return ACTOR_IN, ACTOR_OUT
    if kind == CRITIC:
        return CRITIC_IN, 1
    raise ZbError(f"unknown policy kind {kind}")


def param_count(kind: int) -> int:
    I, O = _dims(kind)
    H, D = HIDDEN, DEPTH
    return H * I + H + D * (6 * H * H + 4 * H) + O * H + O + (JOINTS if kind == ACTOR else 0)


def init_params(kind: int, seed: int = 0) -> np.ndarray:
    """Parameters in the natural (equinox) layout of include/zbot_policy.h.

    Initialised like equinox [U]: Linear weight and bias ~ U(-1/sqrt(in), 1/sqrt(in)),
    GRUCell weights and biases ~ U(-1/sqrt(hidden), 1/sqrt(hidden)). The actor's trailing
    20 floats are the JOINT_BIASES mean offsets (train.py:61-82, 960)."""
    I, O = _dims(kind)
    H, D = HIDDEN, DEPTH
    rng = np.random.default_rng(seed)

    def u(lim, *shape):
        return rng.uniform(-lim, lim, size=shape)

    parts = [u(1 / np.sqrt(I), H, I), u(1 / np.sqrt(I), H)]
    for _ in range(D):
        g = 1 / np.sqrt(H)
        parts += [u(g, 3 * H, H), u(g, 3 * H, H), u(g, 3 * H), u(g, H)]
    parts += [u(1 / np.sqrt(H), O, H), u(1 / np.sqrt(H), O)]
    if kind == ACTOR:
        parts.append(np.array([b for _, b, _ in JOINT_BIASES]))
    out = np.concatenate([np.asarray(p, dtype=np.float32).ravel() for p in parts])
    assert out.size == param_count(kind)
    return out


class GruPolicy:
    """One actor or critic network on one GPU (a zb_policy handle)."""

    def __init__(self, kind: int, params=None, device: int = 0, seed: int = 0, layout: int | None = None):
        import torch  # noqa: PLC0415

        if not torch.cuda.is_available():
            raise ZbError("GruPolicy needs a ROCm GPU (torch.cuda.is_available() is False)")
        self.torch = torch
        self.L = load_library()
        self.kind = kind
        self.I, self.O = _dims(kind)
        self.device = torch.device("cuda", device)
        p = init_params(kind, seed) if params is None else np.asarray(params, dtype=np.float32).ravel()
        p = np.ascontiguousarray(p)
        if p.size != param_count(kind):
            raise ZbError(f"{p.size} parameters, expected {param_count(kind)}")
        self.params = p
        h = C.c_void_p()
        _check(self.L.zb_policy_create(kind, p.ctypes.data_as(C.POINTER(C.c_float)), p.size, device, C.byref(h)))
        self.h = h
        if layout is not None:
            self.set_layout(layout)

    def set_layout(self, layout: int) -> None:
        """LAYOUT_BLOCK (32 envs x 8 waves a workgroup) or LAYOUT_WAVE (16 envs on one wave, the size
        of a zb_step wave's slot); bit-identical results (include/zbot_policy.h)."""
        _check(self.L.zb_policy_set_layout(self.h, int(layout)))

    def set_persistent(self, on: bool) -> None:
        """Block layout: a call over T steps as one persistent launch with the carry in registers
        (default), or one launch per step; bit-identical (include/zbot_policy.h)."""
        _check(self.L.zb_policy_set_persistent(self.h, 1 if on else 0))

    def __del__(self):
        h = getattr(self, "h", None)
        if h is not None and h.value:
            try:
                self.L.zb_policy_destroy(h)
            except Exception:  # noqa: BLE001
                pass
            self.h = None

    def initial_carry(self, n: int):
        """get_initial_model_carry (train.py:1731-1735): zeros [n, depth, hidden] per env."""
        return self.torch.zeros(n, DEPTH, HIDDEN, dtype=self.torch.float32, device=self.device)

    def _stream(self) -> int:
        return self.torch.cuda.current_stream(self.device).cuda_stream

    def _dev(self, t, dtype):
        if t.dtype != dtype or t.device != self.device or not t.is_contiguous():
            t = t.to(device=self.device, dtype=dtype).contiguous()
        return t

    def _check_carry(self, carry, n):
        if (tuple(carry.shape) != (n, DEPTH, HIDDEN) or carry.dtype != self.torch.float32
                or carry.device != self.device or not carry.is_contiguous()):
            raise ZbError(f"carry must be a contiguous float32 [{n}, {DEPTH}, {HIDDEN}] tensor on {self.device}")

    def _out(self, t, shape, dtype):
        if t is None:
            return self.torch.empty(*shape, dtype=dtype, device=self.device)
        if (t.numel() != int(np.prod(shape)) or t.dtype != dtype or t.device != self.device
                or not t.is_contiguous()):
            raise ZbError(f"output must be a contiguous {dtype} tensor of {int(np.prod(shape))} elements")
        return t.view(*shape)

    def actor(self, obs, carry, reset=None, mode: int = SAMPLE, seed: int = 0, env_offset: int = 0, step: int = 0,
              actions=None, log_prob=False):
        """obs [n, 50] or [T, n, 50]; carry [n, 5, 128] updated in place; reset [n] / [T, n] uint8
        (the engine's done flags: carry zeroed before that step). mode SAMPLE / MODE write `actions`,
        EVAL reads them. log_prob: False, True or an output tensor (per joint, [..., 20]).
        Returns (actions, log_prob or None) shaped like obs."""
        torch = self.torch
        if self.kind != ACTOR:
            raise ZbError("actor() on a critic handle")
        single = obs.dim() == 2
        o = self._dev(obs.unsqueeze(0) if single else obs, torch.float32)
        T, n, I = o.shape
        if I != ACTOR_IN:
            raise ZbError(f"actor observations must have {ACTOR_IN} features, got {I}")
        self._check_carry(carry, n)
        r = None if reset is None else self._dev(reset.reshape(T, n), torch.uint8)
        if mode == EVAL:
            if actions is None:
                raise ZbError("EVAL needs the actions")
            a = self._dev(actions.reshape(T, n, JOINTS), torch.float32)
        else:
            a = self._out(actions, (T, n, JOINTS), torch.float32)
        lp = None
        if log_prob is not False and log_prob is not None:
            lp = self._out(None if log_prob is True else log_prob, (T, n, JOINTS), torch.float32)
        _check(self.L.zb_policy_actor(self.h, o.data_ptr(), T, n, carry.data_ptr(),
                                      None if r is None else r.data_ptr(), int(mode), C.c_uint64(seed), int(env_offset),
                                      C.c_uint32(step), a.data_ptr(), None if lp is None else lp.data_ptr(),
                                      self._stream()))
        if single:
            return a[0], (None if lp is None else lp[0])
        return a, lp

    def critic(self, obs, carry, reset=None, value=None):
        """obs [n, 484] or [T, n, 484]; carry [n, 5, 128] updated in place -> value [n] / [T, n]."""
        torch = self.torch
        if self.kind != CRITIC:
            raise ZbError("critic() on an actor handle")
        single = obs.dim() == 2
        o = self._dev(obs.unsqueeze(0) if single else obs, torch.float32)
        T, n, I = o.shape
        if I != CRITIC_IN:
            raise ZbError(f"critic observations must have {CRITIC_IN} features, got {I}")
        self._check_carry(carry, n)
        r = None if reset is None else self._dev(reset.reshape(T, n), torch.uint8)
        v = self._out(value, (T, n), torch.float32)
        _check(self.L.zb_policy_critic(self.h, o.data_ptr(), T, n, carry.data_ptr(),
                                       None if r is None else r.data_ptr(), v.data_ptr(), self._stream()))
        return v[0] if single else v


class PolicyRollout:
    """ksim's rollout loop with the GRU actor in it (sample_action -> env.step, train.py:1737-1763),
    entirely on the GPU: per control step one actor launch and one zb_step launch, whose rows go
    straight into [T, n] buffers. Episode ends reset the actor carry (get_ppo_variables,
    train.py:1719-1723). `engine` is a HipEngine, or an EnvGroups whose groups each run their own
    actor -> zb_step chain on their own stream (bit-identical: the actor's RNG is keyed by global
    env id)."""

    def __init__(self, engine, actor: GruPolicy, seed: int = 0, curriculum: float = 1.0, stagger: bool = False,
                 exact_airtime: bool = True):
        if actor.kind != ACTOR:
            raise ZbError("PolicyRollout needs an actor")
        self.eng = engine
        self.actor = actor
        self.seed = seed
        self.curriculum = curriculum
        # each run() is one ksim trajectory: its FeetAirtime row 0 is patched to ksim's form
        # (prev contact False at t = 0, airtime roll -> air[T-1]; include/zbot.h
        # zb_feet_airtime_exact). False keeps the fused step's causal row 0.
        self.exact_airtime = exact_airtime
        # with env groups: at the first step of a run(), group g's chain starts after group g-1's
        # first actor launch, offsetting the groups' phases (bit-identical either way)
        self.stagger = stagger
        self.carry = actor.initial_carry(engine.n)
        self.step_count = 0
        self.obs = None
        self.obs_c = None  # critic observation of the current state (known after reset / recording)
        self.done = None

    def reset(self):
        out = self.eng.reset(extras=False)
        self.obs = out["obs_actor"].clone()
        self.obs_c = out["obs_critic"].clone()
        self.carry.zero_()
        self.done = None

    def run(self, T: int, record_critic: bool = False, critic: GruPolicy | None = None,
            critic_carry=None) -> dict:
        """T control steps. With record_critic, out["obs_critic"][t] is the critic observation of
        the state the actor acted in at step t (what get_ppo_variables evaluates the critic on,
        train.py:1683-1729) and out["obs_critic_next"] that of the state after step T-1 (the
        bootstrap value's input). out["success"][t] flags the steps whose episode ended at the
        time limit without a failure (ksim's successes_t for compute_ppo_inputs).

        With `critic` (and record_critic), the critic runs inside the loop: V(s_t) right after
        step t's launch, in the same group chain, with `critic_carry` ([n, 5, 128], updated in
        place) reset where the previous step ended an episode (none at t = 0), then the bootstrap
        V(s_T) (reset where step T-1 ended one). out["value"] [T, n] and out["value_next"] [n] are
        bit-identical to critic.critic(out["obs_critic"], carry, reset=[0, done[:-1]]) followed by
        critic.critic(out["obs_critic_next"], carry, reset=done[-1]) after the rollout."""
        torch = self.actor.torch
        n, dev = self.eng.n, self.eng.device
        if self.obs is None:
            self.reset()
        if record_critic and self.obs_c is None:
            raise ZbError("the current state's critic observation is unknown (a run without "
                          "record_critic came before): reset() first")
        f32 = dict(dtype=torch.float32, device=dev)
        obs = torch.empty(T + 1, n, ACTOR_IN, **f32)
        obs[0].copy_(self.obs)
        crit = torch.empty(T + 1, n, CRITIC_IN, **f32) if record_critic else None
        if record_critic:
            crit[0].copy_(self.obs_c)
        acts = torch.empty(T, n, JOINTS, **f32)
        lp = torch.empty(T, n, JOINTS, **f32)
        rew = torch.empty(T, n, **f32)
        done = torch.zeros(T, n, dtype=torch.uint8, device=dev)
        success = torch.zeros(T, n, dtype=torch.uint8, device=dev)
        if critic is not None:
            if not record_critic or critic.kind != CRITIC or critic_carry is None:
                raise ZbError("an in-loop critic needs record_critic=True, a critic handle and its carry")
            critic._check_carry(critic_carry, n)
            val = torch.empty(T + 1, n, **f32)
        L = self.eng.L
        # an EnvGroups engine runs each group's actor -> zb_step chain on the group's own stream
        # (DESIGN.md §4f); a HipEngine is one group on the current stream
        grouped = hasattr(self.eng, "groups")
        parts = self.eng.groups() if grouped else [(self.eng, None, (0, n))]
        if grouped:
            self.eng.fork()
        if self.exact_airtime:
            for e, _, _ in parts:
                _check(L.zb_mark_rollout_start(e.h))
        for t in range(T):
            for g, (e, s, (lo, hi)) in enumerate(parts):
                with (torch.cuda.stream(s) if s is not None else contextlib.nullcontext()):
                    stream = torch.cuda.current_stream(dev).cuda_stream
                    r = done[t - 1][lo:hi] if t > 0 else (None if self.done is None else self.done[lo:hi])
                    if self.stagger and grouped and t == 0 and g > 0:
                        s.wait_event(prev_actor)
                    self.actor.actor(obs[t][lo:hi], self.carry[lo:hi], reset=r, mode=SAMPLE, seed=self.seed,
                                     env_offset=e.env_offset, step=self.step_count, actions=acts[t][lo:hi],
                                     log_prob=lp[t][lo:hi])
                    if self.stagger and grouped and t == 0:
                        prev_actor = torch.cuda.Event()
                        prev_actor.record(s)
                    _check(L.zb_step(e.h, acts[t][lo:hi].data_ptr(), obs[t + 1][lo:hi].data_ptr(),
                                     crit[t + 1][lo:hi].data_ptr() if record_critic else None, None, None,
                                     rew[t][lo:hi].data_ptr(), done[t][lo:hi].data_ptr(),
                                     success[t][lo:hi].data_ptr(), float(self.curriculum), stream))
                    if self.exact_airtime and t == T - 1:
                        _check(L.zb_feet_airtime_exact(e.h, rew[0][lo:hi].data_ptr(), None, float(self.curriculum),
                                                       stream))
                    if critic is not None:  # V(s_t): its input crit[t] is ready since step t-1
                        critic.critic(crit[t][lo:hi], critic_carry[lo:hi],
                                      reset=done[t - 1][lo:hi] if t > 0 else None, value=val[t][lo:hi])
                        if t == T - 1:  # the bootstrap V(s_T)
                            critic.critic(crit[T][lo:hi], critic_carry[lo:hi], reset=done[T - 1][lo:hi],
                                          value=val[T][lo:hi])
                if grouped:
                    self.eng.mark(g)
            self.step_count += 1
        if grouped:
            self.eng.join()
        self.obs = obs[T].clone()
        self.obs_c = crit[T].clone() if record_critic else None
        self.done = done[T - 1].clone()
        out = dict(obs_actor=obs, actions=acts, log_prob=lp, reward=rew, done=done, success=success)
        if record_critic:
            out["obs_critic"] = crit[:T]
            out["obs_critic_next"] = crit[T]
        if critic is not None:
            out["value"] = val[:T]
            out["value_next"] = val[T]
        return out
