"""ksim-shaped environment API over the HIP engine.

Mirrors the names the reference task uses so a train.py-style caller can swap
ksim's MjxEngine rollout for this engine:

  * observations: the dict keys ksim builds from train.py:1478-1537
    (``joint_position_observation``, ``imu_orientation_observation``, ...);
  * rewards: the registered terms of train.py:1546-1586 with their scales;
  * ``actor_inputs`` / ``critic_inputs``: the concatenations of
    ZbotWalkingTask.run_actor (train.py:1629-1639) and run_critic
    (train.py:1664-1679), produced directly by the kernel (50 / 484 floats);
  * episode statistics reduced across ranks for the curriculum / logging.

All tensors are torch device tensors (views into the engine's output buffers;
clone them if they must survive the next step).
"""

from __future__ import annotations

from . import cstructs as cs
from .config import default_config
from .constants import JOINT_BIASES, REWARDS
from .curriculum import EpisodeLengthCurriculum, rollout_episode_length
from .engine import EnvGroups, HipEngine
from .model import compile_model

# obs_critic layout (train.py:1664-1679)
_CRITIC = dict(
    joint_positions=(0, 20),
    joint_velocity_div10=(20, 40),
    com_inertia=(40, 290),
    com_velocity=(290, 440),
    imu_acc=(440, 443),
    imu_gyro=(443, 446),
    imu_quat=(446, 450),
    cmd_all=(450, 457),
    act_force_div100=(457, 477),
    base_pos=(477, 480),
    base_quat=(480, 484),
)


def observation_dict(out: dict) -> dict:
    """ksim observation names -> tensors, from the engine outputs."""
    oa, oc, ox = out["obs_actor"], out["obs_critic"], out["obs_extra"]

    def c(k):
        a, b = _CRITIC[k]
        return oc[:, a:b]

    obs = {
        "joint_position_observation": oa[:, 0:20],
        "joint_velocity_observation": oa[:, 20:40],
        "imu_orientation_observation": oa[:, 40:44],
        "actuator_force_observation": c("act_force_div100") * 100.0,
        "center_of_mass_inertia_observation": c("com_inertia"),
        "center_of_mass_velocity_observation": c("com_velocity"),
        "base_position_observation": c("base_pos"),
        "base_orientation_observation": c("base_quat"),
        "sensor_observation_imu_acc": c("imu_acc"),
        "sensor_observation_imu_gyro": c("imu_gyro"),
    }
    if ox is not None:
        obs.update({
            "base_linear_velocity_observation": ox[:, cs.X_BASE_LINVEL:cs.X_BASE_LINVEL + 3],
            "base_angular_velocity_observation": ox[:, cs.X_BASE_ANGVEL:cs.X_BASE_ANGVEL + 3],
            "base_linear_acceleration_observation": ox[:, cs.X_BASE_LINACC:cs.X_BASE_LINACC + 3],
            "base_angular_acceleration_observation": ox[:, cs.X_BASE_ANGACC:cs.X_BASE_ANGACC + 3],
            "base_height_observation": ox[:, cs.X_BASE_HEIGHT:cs.X_BASE_HEIGHT + 1],
            "sensor_observation_left_foot_touch": ox[:, cs.X_TOUCH:cs.X_TOUCH + 1],
            "sensor_observation_right_foot_touch": ox[:, cs.X_TOUCH + 1:cs.X_TOUCH + 2],
            "sensor_observation_left_foot_force": ox[:, cs.X_FORCE:cs.X_FORCE + 3],
            "sensor_observation_right_foot_force": ox[:, cs.X_FORCE + 3:cs.X_FORCE + 6],
            "feet_position_observation": ox[:, cs.X_FEET_POS:cs.X_FEET_POS + 6],
            "feetech_torque_observation": ox[:, cs.X_FEETECH_TAU:cs.X_FEETECH_TAU + 20],
            "actuator_acceleration_observation": ox[:, cs.X_ACT_ACC:cs.X_ACT_ACC + 20],
        })
        for i, (name, _, _) in enumerate(JOINT_BIASES):  # ActPosObservation per joint [U: = joint position]
            obs[f"act_pos_observation_{name}"] = oa[:, i:i + 1]
    return obs


class StepResult:
    """One step's outputs under ksim's names (views into the engine's output buffers).

    With env groups (ZbotWalkingEnv(groups=G > 1)) the buffers are still being written on the group
    streams when step() returns. Every read of a field makes the stream that is current at that read
    wait for every group (EnvGroups.join: one stream-wait per group, no host synchronisation), so a
    loop that only steps, as an open-loop rollout does, never serialises the groups, and a read under
    any stream context (e.g. `with torch.cuda.stream(side)`) sees the outputs complete on that stream.
    It is not a dataclass (reads are properties); as_dict() gives the fields as a plain dict."""

    FIELDS = ("obs", "actor_inputs", "critic_inputs", "reward", "reward_terms", "done", "success")

    def __init__(self, obs, actor_inputs, critic_inputs, reward, reward_terms, done, success=None, join=None):
        self._v = dict(obs=obs, actor_inputs=actor_inputs, critic_inputs=critic_inputs, reward=reward,
                       reward_terms=reward_terms, done=done, success=success)
        self._join = join

    def _get(self, k):
        if self._join is not None:
            self._join()  # on every read: the join orders only the stream current at this read
        return self._v[k]

    def as_dict(self) -> dict:
        """Every field (joined on the current stream), for callers that used dataclasses.asdict."""
        return {k: self._get(k) for k in self.FIELDS}

    obs = property(lambda self: self._get("obs"))
    actor_inputs = property(lambda self: self._get("actor_inputs"))
    critic_inputs = property(lambda self: self._get("critic_inputs"))
    reward = property(lambda self: self._get("reward"))
    reward_terms = property(lambda self: self._get("reward_terms"))
    done = property(lambda self: self._get("done"))
    success = property(lambda self: self._get("success"))  # time-limit ends without a failure (ksim successes_t)


def default_groups(num_envs: int) -> int:
    """Env groups of ZbotWalkingEnv: two from 4096 envs up (one step-kernel round per group fills the
    other's drain), else one handle."""
    return 2 if num_envs >= 4096 else 1


class ZbotWalkingEnv:
    """Batched ZbotWalkingTask environment (train.py:1311-1763) on one GPU.

    `num_envs`, `dt`, `ctrl_dt`, `iterations`, `ls_iterations` default to
    train.py:1768-1781 (512 envs, 0.001, 0.02, 8, 8).

    `groups`: env groups, each a handle stepping on its own HIP stream (zbot_amd.EnvGroups,
    DESIGN.md §4f); the default is two from 4096 envs up. Results are the same bits for every
    group count; StepResult fields join the groups when first read.

    `curriculum` is ksim's EpisodeLengthCurriculum of get_curriculum (train.py:1595-1602);
    `curriculum_level` starts at its initial level (0.5, the curriculum's floor) and moves when
    update_curriculum() is called once per rollout (a training step). Assigning
    `curriculum_level` directly overrides it.
    """

    def __init__(self, num_envs: int = 512, *, seed: int = 0, device: int = 0, env_offset: int = 0,
                 push: bool = False, randomize: bool = False, obs_noise: bool = True, model=None,
                 curriculum: EpisodeLengthCurriculum | None = None, groups: int | None = None, **cfg_kw):
        self.model = model or compile_model()
        self.cfg = default_config(push=push, randomize=randomize, obs_noise=obs_noise, **cfg_kw)
        self.groups = default_groups(num_envs) if groups is None else int(groups)
        if self.groups > 1:
            self.engine = EnvGroups(self.model, self.cfg, num_envs, groups=self.groups, env_offset=env_offset,
                                    device=device, seed=seed)
        else:
            self.engine = HipEngine(self.model, self.cfg, num_envs, env_offset=env_offset, device=device, seed=seed)
        self.num_envs = num_envs
        self.curriculum = curriculum or EpisodeLengthCurriculum()
        self.curriculum_state = self.curriculum.initial_state()
        self.curriculum_level = self.curriculum_state.level
        self._last_done = None

    def join(self) -> None:
        """Make the caller's current stream wait for every group's enqueued steps (a no-op with one
        handle). StepResult does this on its first read."""
        self.engine.join()

    def _result(self, out: dict, with_reward: bool) -> StepResult:
        terms = {}
        if with_reward:
            rt = out["reward_terms"]
            terms = {name: rt[:, i] for i, (name, _, _) in enumerate(REWARDS)}
        return StepResult(
            obs=observation_dict(out),
            actor_inputs=out["obs_actor"],
            critic_inputs=out["obs_critic"],
            reward=out["reward"] if with_reward else None,
            reward_terms=terms,
            done=out["done"] if with_reward else None,
            success=out["success"] if with_reward else None,
            join=self.engine.join if self.groups > 1 else None,
        )

    def reset(self, mask=None) -> StepResult:
        return self._result(self.engine.reset(mask=mask), with_reward=False)

    def step(self, action) -> StepResult:
        """One control step (20 physics substeps) for every env; done envs auto-reset."""
        out = self.engine.step(action, curriculum=self.curriculum_level)
        self._last_done = out["done"]
        return self._result(out, with_reward=True)

    def begin_rollout(self) -> None:
        """Open a rollout (one ksim trajectory): clear the episode-statistics window that
        update_curriculum() reads, and mark step 0 for the exact FeetAirtime row
        (end_rollout; include/zbot.h zb_feet_airtime_exact)."""
        self.engine.get_stats(clear=True)
        self.engine.mark_rollout_start()

    def end_rollout(self, reward0=None, terms0=None) -> None:
        """Patch the rollout's row 0 (its reward [n] / reward terms [n, 12] buffers, as recorded from
        the first step() after begin_rollout) to ksim's FeetAirtimeReward (train.py:515-546)."""
        self.engine.feet_airtime_exact(reward0, terms0, curriculum=self.curriculum_level)
        self.engine.join()  # the patched row is read on the caller's stream next

    def update_curriculum(self) -> float:
        """EpisodeLengthCurriculum update after a rollout (train.py:1595-1602; zbot_amd.curriculum):
        the mean episode length of the rollout's window (begin_rollout) over every env of every rank
        (RCCL all_gather when distributed), then the level law. Returns the new level."""
        if self._last_done is None:
            raise RuntimeError("update_curriculum() needs a rollout: step() first")
        self.engine.join()
        state = self.engine.get_state()
        self.check_bank_overflow(state)
        length = rollout_episode_length(self.engine.get_stats(), state, self._last_done, self.cfg.ctrl_dt)
        self.curriculum_state = self.curriculum.update(self.curriculum_state, length)
        self.curriculum_level = self.curriculum_state.level
        return self.curriculum_level

    def check_bank_overflow(self, state=None) -> int:
        """Envs whose second contact-row bank overflowed at some substep (more colliders beyond the soles
        within reach of the floor than the banks hold: four, two beside the sole pair; the extra ones' contacts were not simulated: zb_engine.hip
        select_bank2, engine.state_flags). Warns once per env object the first time any env has; called
        by update_curriculum() after every rollout. Returns the count."""
        from .engine import state_flags  # noqa: PLC0415

        n = int(state_flags(self.engine.get_state() if state is None else state)["bank_overflow"].sum().item())
        if n and not getattr(self, "_overflow_warned", False):
            import warnings  # noqa: PLC0415

            warnings.warn(f"{n} env(s) had more colliders beyond the soles within reach of the floor in one "
                          "substep than the contact-row banks hold; the extra contacts were not simulated (DESIGN.md §4j)", RuntimeWarning,
                          stacklevel=2)
            self._overflow_warned = True
        return n

    def default_action(self):
        """FeetechActuators.get_default_action: current joint positions (train.py:1282-1283)."""
        return self.engine.get_state()[:, 7:27].clone()

    def episode_stats(self, clear: bool = True) -> dict:
        """Globally reduced episode statistics (RCCL all_gather when distributed)."""
        from .dist import reduce_episode_stats  # noqa: PLC0415

        tot = reduce_episode_stats(self.engine.get_stats(clear=clear))
        n = max(float(tot[cs.ST_DONE]), 1.0)
        return {
            "episodes": float(tot[cs.ST_DONE]),
            "mean_return": float(tot[cs.ST_RETURN]) / n,
            "mean_length_steps": float(tot[cs.ST_LENGTH]) / n,
            "reward_sum": float(tot[cs.ST_REWARD]),
        }
