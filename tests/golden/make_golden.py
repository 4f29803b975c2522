"""Generate the committed golden vectors from the CPU oracle (fp32 build).

    python tests/golden/make_golden.py

The reference (JAX/MJX/ksim) cannot run in this container, so
the fixtures pin the build's own oracle: BASELINE's C1 rollout (64 envs x 128
env-steps, seed 0, default train.py configuration incl. observation noise), a
domain-randomized + push variant (configs 3/5 features) and a CG-solver case. Tests re-run the
oracle against them (regression pin) and compare the HIP engine to them.
"""

import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "ksim-gym-zbot_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import oracle as O  # noqa: E402
from zbot_amd import compile_model, default_config  # noqa: E402

CASES = {
    # BASELINE.json configs[0]: 64 parallel envs, 128-step rollout (round 4: was 32 x 16)
    "c1_64x128_seed0": dict(n=64, steps=128, seed=0, push=False, randomize=False, std=0.05),
    "c5_push_seed1": dict(n=16, steps=16, seed=1, push=True, randomize=True, std=0.1),
    # round 3: the CG solver variant (ZbEnvConfig.solver)
    "c2_cg_seed2": dict(n=16, steps=16, seed=2, push=False, randomize=False, std=0.05, solver="cg"),
    # round 4: CG at C1's ensemble size, with pushes (the GPU test compares its first 8 rewards and
    # the 64-step ensemble statistics)
    "c2_cg_64x64_seed4": dict(n=64, steps=64, seed=4, push=True, randomize=False, std=0.1, solver="cg"),
    # round 5: CG at BASELINE C1's own shape (64 envs x 128 steps, seed 0, the C1 actions)
    "c1_cg_64x128_seed0": dict(n=64, steps=128, seed=0, push=False, randomize=False, std=0.05, solver="cg"),
    # round 5: mj_Euler's implicit joint damping (ZB_F_EULERDAMP), with each solver
    "c2_eulerdamp_seed5": dict(n=16, steps=16, seed=5, push=False, randomize=False, std=0.05, eulerdamp=True),
    "c5_cg_eulerdamp_seed6": dict(n=16, steps=16, seed=6, push=True, randomize=True, std=0.1, solver="cg",
                                  eulerdamp=True),
    # round 5: the convex-mesh collider model (assets/zbot_like_mesh.xml; CPU regression pin of the
    # oracle's plane_mesh through a rollout with pushes: the GPU side is tests/test_gpu_colliders.py)
    "mesh_32x24_seed7": dict(n=32, steps=24, seed=7, push=True, randomize=False, std=0.2, model="zbot_like_mesh.xml"),
    # round 5: nine floor colliders (model v9; the oracle collides all of them)
    "many_32x24_seed8": dict(n=32, steps=24, seed=8, push=True, randomize=True, std=0.2, model="zbot_like_many.xml"),
}


def case_model(model=None):
    """The compiled model of a case: the default descriptor, or an MJCF asset of the package."""
    if model is None:
        return compile_model()
    from zbot_amd.mjcf import load_mjcf  # noqa: PLC0415

    return compile_model(load_mjcf(os.path.join(ROOT, "ksim-gym-zbot_amd", "assets", str(model))))


EXACT_STEPS = 16  # tests/test_gpu_parity.py GOLDEN_EXACT_STEPS: the per-env state is also kept at this step


def run_case(name, n, steps, seed, push, randomize, std, solver="newton", eulerdamp=False, model=None):
    cm = case_model(model)
    cfg = default_config(push=push, randomize=randomize, solver=solver, eulerdamp=eulerdamp)
    env = O.OracleEnv(cm.cmodel, cfg, n, seed=seed)
    oa0, oc0, _ = env.reset()
    rewards, dones, actions = [], [], []
    for t in range(steps):
        a = O.synthetic_actions(cm.cmodel, seed, n, 0, t, std=std)
        out = env.step(a)
        actions.append(a)
        rewards.append(out["reward"])
        dones.append(out["done"])
        if t + 1 == EXACT_STEPS:
            state_exact = env.state.copy()
    extra = {"state_at_exact": state_exact} if steps > EXACT_STEPS else {}
    return dict(**extra,
        reset_obs_actor=oa0, reset_obs_critic=oc0, actions=np.stack(actions), reward=np.stack(rewards),
        done=np.stack(dones), final_state=env.state.copy(), final_rand=env.rand.copy(),
        final_obs_actor=out["obs_actor"], final_obs_critic=out["obs_critic"], final_terms=out["reward_terms"],
        stats=env.stats.copy(),
    )


def main():
    only = sys.argv[1:]  # case names to (re)generate; default: all
    for name, kw in CASES.items():
        if only and name not in only:
            continue
        data = run_case(name, **kw)
        np.savez_compressed(os.path.join(HERE, f"{name}.npz"), **data, **{f"cfg_{k}": v for k, v in kw.items()})
        print(name, {k: v.shape for k, v in data.items()})


if __name__ == "__main__":
    main()
