"""ksim's EpisodeLengthCurriculum as train.py registers it (train.py:1595-1602), on the engine's
episode statistics.

    cur = EpisodeLengthCurriculum()                      # 30 levels, 30 / 10, min_level_steps 10, min 0.5
    state = cur.initial_state()
    for each training step:
        eng.get_stats(clear=True)                        # open the rollout's statistics window
        ... T zb_steps at curriculum level state.level ...
        length = rollout_episode_length(eng.get_stats(), eng.get_state(), done[T-1], ctrl_dt)
        state = cur.update(state, length)                 # the same level on every rank

The level is one global scalar: zb_step takes it as `curriculum_level`, and it
scales the terms registered with scale_by_curriculum (StraightLeg, AnkleKnee, ArmPose,
train.py:1576-1585) and, as ksim's PushEvent does [U], the push velocity (train.py:1459-1468).

ksim 0.1.99's curriculum module is not vendored here, so the law below is restated
from ksim's documented behaviour. Every choice it could not confirm is marked [U]:
  [U1] the measured quantity is ksim's Trajectory.episode_length(): per env, the mean over the
       rollout's episode ends (the last step counts as an end) of the time since the episode
       started, in seconds; then the mean over all envs of all ranks. The thresholds are seconds
       (30 s / 10 s against EpisodeLengthTermination's 80 s, train.py:1592).
  [U2] an episode's time at its end counts its terminal step: env-steps x ctrl_dt.
  [U3] the level moves by 1 / num_levels, up when the length is above increase_threshold, down
       when below decrease_threshold, only after min_level_steps updates at the current level;
       it is clipped to [min_level, 1] and the counter restarts at every change.
  [U4] the initial level is min_level.
"""

from __future__ import annotations

from dataclasses import dataclass

from . import cstructs as cs


@dataclass(frozen=True)
class CurriculumState:
    level: float
    steps: int  # updates since the level last changed


@dataclass(frozen=True)
class EpisodeLengthCurriculum:
    """train.py:1596-1602 defaults."""

    num_levels: int = 30
    increase_threshold: float = 30.0
    decrease_threshold: float = 10.0
    min_level_steps: int = 10
    min_level: float = 0.5

    def __post_init__(self):
        if self.num_levels < 1 or self.min_level_steps < 1:
            raise ValueError("num_levels and min_level_steps must be >= 1")
        if not 0.0 <= self.min_level <= 1.0:
            raise ValueError("min_level must lie in [0, 1]")

    def initial_state(self) -> CurriculumState:
        return CurriculumState(level=float(self.min_level), steps=0)  # [U4]

    def update(self, state: CurriculumState, episode_length_sec: float) -> CurriculumState:
        """One training step's update from the mean episode length (seconds) [U1, U3]."""
        can_move = state.steps >= self.min_level_steps
        delta = 0.0
        if can_move and episode_length_sec > self.increase_threshold:
            delta = 1.0 / self.num_levels
        elif can_move and episode_length_sec < self.decrease_threshold:
            delta = -1.0 / self.num_levels
        level = min(1.0, max(self.min_level, state.level + delta))
        if level != state.level:
            return CurriculumState(level=level, steps=0)
        return CurriculumState(level=state.level, steps=state.steps + 1)


def rollout_episode_length(stats, state, done_last, ctrl_dt: float, group=None) -> float:
    """Mean episode length in seconds of one rollout, over every env of every rank [U1, U2].

    stats [n, ZB_NUM_STATS]: zb_get_stats since the rollout started (Σ length in env-steps and
    the count of the episodes that ended); state [n, ZB_STATE_STRIDE]: the rows after the last
    step (ZB_S_EP_STEPS: env-steps of the episode still running); done_last [n]: the last step's
    done flags (an episode that ended on the last step is not counted twice). Each rank sums its
    per-env means in float64; the partials and env counts are all-gathered and summed in rank
    order, so every rank gets the same bits (zbot_amd.dist.reduce_fixed_order)."""
    import torch  # noqa: PLC0415

    st = stats.double()
    running = state[:, cs.S_EP_STEPS].contiguous().view(torch.int32).double()
    open_end = (done_last == 0).double()
    num = st[:, cs.ST_LENGTH] + open_end * running
    den = st[:, cs.ST_DONE] + open_end
    per_env = (num / den.clamp(min=1.0)) * float(ctrl_dt)
    part = torch.stack([per_env.sum(), torch.tensor(float(per_env.numel()), dtype=torch.float64,
                                                    device=per_env.device)])
    from .dist import reduce_fixed_order  # noqa: PLC0415

    tot = reduce_fixed_order(part, group=group)
    return float(tot[0] / tot[1]) if float(tot[1]) > 0 else 0.0
