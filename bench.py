"""Benchmark: env-steps/s of the fused HIP Z-Bot env.step on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--envs E] [--config c1|c2|c3|c5]
    torchrun --nproc-per-node N bench.py --gpus N ...   (one rank per GPU, RCCL)

--gpus N is authoritative: without torchrun (WORLD_SIZE unset) and N > 1, bench.py spawns the N
rank processes itself; under torchrun WORLD_SIZE must equal N; with nccl (RCCL) N GPUs must be
visible. Any mismatch exits with status 2 before a GPU call. The line reports `ranks_seen`.

A "step" is one zb_step over all E envs of a GPU (20 physics substeps each,
CG solver 8 / 8 line-search iterations -- MJX's SolverType.CG, as ksim sets it [U];
`--solver newton` for MuJoCo's Newton -- observations, rewards, auto-reset)
— the hot path of ksim's step_engine for train.py's ZbotWalkingTask
(SURVEY.md §3.2). Inputs are synthetic (actions = JOINT_BIASES + 0.05 N(0,1),
generated on the GPU before timing); the state is resident in HBM. Prints ONE
JSON line on rank 0 (contract: see the repository brief / DESIGN.md §Bench).
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "ksim-gym-zbot_amd"))

METRIC = "env-steps/sec at N envs per GPU, 1/2/4/8 MI355X; % HBM roofline"

CONFIGS = {
    "c1": dict(envs=64, push=False, randomize=False,
               name="C1: {n} envs, the reference's CPU-runnable case (its JAX-CPU path; here the GPU, with the "
                    "CPU twin timed over the same 64 envs x 128 steps)"),
    "c2": dict(envs=8192, push=False, randomize=False, name="C2: {n} envs/GPU, flat-floor stand"),
    "c3": dict(envs=32768, push=True, randomize=False, name="C3: {n} envs/GPU, push-perturbation curriculum"),
    "c5": dict(envs=16384, push=False, randomize=True, name="C5: {n} envs/GPU, per-env domain randomization"),
}


# algorithmic FLOPs per env-step counted by the instrumented CPU twin (scripts/count_flops.py) for each
# (solver, model variant) that the line prices; a variant without its own count gets no roofline_fp32
FLOPS_FILES = {
    ("cg", "base"): "r06_flops_count_cg.json",
    ("newton", "base"): "r06_flops_count_newton.json",
    ("cg", "mjxbox"): "r06_flops_count_cg_mjxbox.json",
    ("newton", "mjxbox"): "r05_flops_count_mjxbox.json",
    ("cg", "eulerdamp"): "r05_flops_count_cg_eulerdamp.json",
    ("newton", "eulerdamp"): "r05_flops_count_eulerdamp.json",
    ("cg", "solepair"): "r06_flops_count_cg_solepair.json",
    ("newton", "solepair"): "r06_flops_count_solepair.json",
}


def host_cpu() -> dict:
    """The host the CPU baseline ran on: logical CPUs, the ones this process may use, the model."""
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return {"nproc": os.cpu_count(), "affinity": len(os.sched_getaffinity(0)), "model": model}


def baseline_threads() -> tuple[int, str]:
    """OpenMP threads of the CPU twin and where that number came from: every CPU this process may
    run on (sched_getaffinity), unless the host caps the job's CPU share through OMP_NUM_THREADS
    (the GPU box sets it to its per-GPU share of 16 and asks jobs to keep it)."""
    aff = len(os.sched_getaffinity(0))
    env = os.environ.get("OMP_NUM_THREADS", "")
    cap = int(env or 0)
    if 0 < cap < aff:
        return cap, f"OMP_NUM_THREADS={env} (the host's per-job CPU share, of {aff} CPUs in the affinity mask)"
    return max(1, aff), f"sched_getaffinity: all {aff} CPUs this process may run on"


def _time_twin(O, cm, cfg, n_envs: int, budget_s: float, max_steps: int, min_steps: int = 2):
    env = O.OracleEnv(cm.cmodel, cfg, n_envs, seed=0)
    env.reset()
    acts = [O.synthetic_actions(cm.cmodel, 0, n_envs, 0, t) for t in range(4)]
    env.step(acts[0])  # warm-up (thread pool, first touch)
    steps = 0
    t0 = time.perf_counter()
    while True:
        env.step(acts[steps % 4])
        steps += 1
        el = time.perf_counter() - t0
        if (max_steps and steps >= max_steps) or (not max_steps and el >= budget_s and steps >= min_steps):
            break
    return steps, el


def cpu_baseline(cm, cfg, budget_s: float, workload: str, n_envs: int, max_steps: int = 0, c1_leg: bool = True) -> dict:
    """Time the CPU twin (the oracle: fp32 C restatement, OpenMP over the env axis) on a bounded
    sample of the headline workload: the same env count, as many env-steps as fit in budget_s
    (max_steps > 0: exactly that many, the C1 rollout). With c1_leg, the reference's own
    CPU-runnable case (C1: 64 envs x 128 env-steps) is timed beside it."""
    threads, cap_src = baseline_threads()
    os.environ["OMP_NUM_THREADS"] = str(threads)  # read by the OpenMP runtime at the oracle's first load
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O  # noqa: PLC0415  (cpu_baseline leg: the oracle is the CPU twin being timed)

    steps, el = _time_twin(O, cm, cfg, n_envs, budget_s, max_steps)
    out = {
        "value": n_envs * steps / el,
        "unit": "env-steps/s",
        "cores": threads,
        "kind": "port",
        "sample": f"{n_envs} envs x {steps} env-steps of the same workload ({workload}) on the CPU twin "
                  f"(oracle/zb_oracle.c, fp32, OpenMP {threads} threads), {el:.1f} s",
        "envs": n_envs,
        "threads_cap": cap_src,
        "per_core": n_envs * steps / el / threads,
        "per_core_unit": "env-steps/s per thread (one thread per core)",
        "host": host_cpu(),
    }
    if c1_leg:
        s1, e1 = _time_twin(O, cm, cfg, 64, 0.0, 128)
        out["c1"] = {"value": 64 * s1 / e1, "unit": "env-steps/s", "sample": f"64 envs x {s1} env-steps (C1), "
                     f"{e1:.2f} s", "cores": threads, "per_core": 64 * s1 / e1 / threads}
    return out


def bench_ppo_inputs(n: int, T: int, reps: int, dev, world: int) -> dict:
    """Post-rollout PPO inputs over a [T, n] rollout resident in HBM:
    zb_gae (GAE reverse scan + value targets + moment partials), the moment tree, the
    cross-rank combine (RCCL all_gather when world > 1) and zb_adv_normalize."""
    import ctypes as C  # noqa: PLC0415

    import torch  # noqa: PLC0415
    from zbot_amd import ppo as P  # noqa: PLC0415
    from zbot_amd.metrics import HBM_PEAK_GBS  # noqa: PLC0415

    g = torch.Generator(device=dev)
    g.manual_seed(99)
    rew = torch.randn(T, n, device=dev, generator=g)
    val = torch.randn(T, n, device=dev, generator=g)
    done = (torch.rand(T, n, device=dev, generator=g) < 0.01).to(torch.uint8)
    L = P.load_library()
    gae = torch.empty(T, n, device=dev)
    vt = torch.empty(T, n, device=dev)
    part = torch.empty(int(L.zb_gae_partials_words(n)), dtype=torch.float64, device=dev)
    stream = torch.cuda.current_stream(dev)
    sp = stream.cuda_stream

    def gae_only():
        rc = L.zb_gae(rew.data_ptr(), val.data_ptr(), done.data_ptr(), None, None, T, n, C.c_float(P.DEFAULT_GAMMA),
                      C.c_float(P.DEFAULT_LAMBDA), gae.data_ptr(), vt.data_ptr(), part.data_ptr(), None, sp)
        assert rc == 0

    for _ in range(3):
        gae_only()
        P.compute_ppo_inputs(val, rew, done)
    torch.cuda.synchronize(dev)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for a, b in ev:
        a.record(stream)
        gae_only()
        b.record(stream)
    torch.cuda.synchronize(dev)
    warm_ms = sum(a.elapsed_time(b) for a, b in ev) / reps
    # cold: a 512 MB write between launches evicts the rollout from L2 and the 256 MB MALL, so the
    # kernel reads its inputs from HBM as after a real rollout of other work; this is the roofline
    flush = torch.empty(128 * 1024 * 1024, dtype=torch.float32, device=dev)
    evc = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for a, b in evc:
        flush.fill_(1.0)
        a.record(stream)
        gae_only()
        b.record(stream)
    torch.cuda.synchronize(dev)
    gae_ms = sum(a.elapsed_time(b) for a, b in evc) / reps
    del flush
    t0 = time.perf_counter()
    for _ in range(reps):
        out = P.compute_ppo_inputs(val, rew, done)
    torch.cuda.synchronize(dev)
    full_ms = (time.perf_counter() - t0) * 1e3 / reps
    bpu = 17  # per (t, env): reward 4 + value 4 + done 1 read; gae 4 + value target 4 written
    achieved = bpu * T * n / (gae_ms * 1e-3) / 1e9
    traffic = None
    tpath = os.path.join(ROOT, "profiles", "pmc_traffic_gae.json")
    if os.path.exists(tpath):
        with open(tpath) as f:
            tj = json.load(f)
        if tj.get("envs") == n and tj.get("T") == T:
            traffic = tj.get("hbm_bytes_per_launch")
    assert torch.isfinite(out.advantages_t).all()
    return {
        "workload": f"GAE + value targets + global advantage normalization over a [{T}, {n}] rollout per GPU "
                    f"(x{world} ranks, moments combined over RCCL)",
        "gae_kernel_ms": gae_ms,
        "gae_kernel_ms_warm": warm_ms,
        "compute_ppo_inputs_ms": full_ms,
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "kernel": "zb::gae_kernel",
                     "algorithmic_bytes_per_unit": bpu, "unit_note": "one (step, env) element",
                     "note": "cold: L2 and MALL flushed by a 512 MB write before each launch (inputs from HBM); "
                             "gae_kernel_ms_warm is back to back with the rollout cache-resident"},
    }


def bench_c2_rollout(eng, n: int, T: int, dev, rank: int, world: int, sigma: float = 0.2) -> dict:
    """C2 as BASELINE.json states it: one T = 256-step rollout of all n envs, timed whole, with
    automatic resets inside the window (actions JOINT_BIASES + sigma N(0,1), sigma = 0.2 as in the
    soak test, so robots fall and episodes end), the reward / done rows of every step kept as a
    [T, n] rollout buffer, and the FeetAirtime row 0 patched to ksim's trajectory form after the
    last step (include/zbot.h zb_feet_airtime_exact)."""
    import torch  # noqa: PLC0415
    import torch.distributed as dist  # noqa: PLC0415
    from zbot_amd import cstructs as cs  # noqa: PLC0415
    from zbot_amd.constants import JOINT_BIASES  # noqa: PLC0415

    g = torch.Generator(device=dev)
    g.manual_seed(4321 + rank)
    bias = torch.tensor([b for _, b, _ in JOINT_BIASES], device=dev)
    acts = bias + sigma * torch.randn(T, n, cs.NJ, device=dev, generator=g)
    rew = torch.empty(T, n, device=dev)
    done = torch.empty(T, n, dtype=torch.uint8, device=dev)
    grouped = hasattr(eng, "groups")

    def rollout():
        eng.mark_rollout_start()
        for t in range(T):  # zb_step writes the reward / done rows of the rollout buffer directly
            eng.step(acts[t], extras=False, reward=rew[t], done=done[t])
        eng.feet_airtime_exact(rew[0], None)
        if grouped:
            eng.join()

    eng.reset(extras=False)
    rollout()  # untimed: first use of the buffers
    eng.reset(extras=False)
    eng.get_stats(clear=True)
    torch.cuda.synchronize(dev)
    if dist.is_initialized():
        dist.barrier()
    t0 = time.perf_counter()
    rollout()
    torch.cuda.synchronize(dev)
    if dist.is_initialized():
        dist.barrier()
    wall = torch.tensor([time.perf_counter() - t0], device=dev, dtype=torch.float64)
    if dist.is_initialized():
        dist.all_reduce(wall, op=dist.ReduceOp.MAX)
    wall = float(wall.item())
    eng.check()
    ends = int(done.sum().item())
    assert bool(torch.isfinite(rew).all())
    return {
        "workload": f"C2 as stated: one {T}-step rollout of {n} envs per GPU from reset, actions JOINT_BIASES + "
                    f"{sigma} N(0,1), automatic resets inside the window, [T, n] reward / done rows, FeetAirtime "
                    "row 0 patched to ksim's trajectory form",
        "env_steps_per_s": world * n * T / wall,
        "ms_per_rollout": 1e3 * wall,
        "rollout_steps": T,
        "episodes_done": ends,
    }


def _timed_steps(step, steps: int, warmup: int, dev, world: int) -> float:
    """Wall seconds of `steps` calls of step(t) after `warmup` untimed ones, bracketed by
    synchronize (+ barrier when distributed), max over ranks."""
    import torch  # noqa: PLC0415
    import torch.distributed as dist  # noqa: PLC0415

    for t in range(warmup):
        step(t)
    torch.cuda.synchronize(dev)
    if dist.is_initialized():
        dist.barrier()
    t0 = time.perf_counter()
    for t in range(steps):
        step(warmup + t)
    torch.cuda.synchronize(dev)
    if dist.is_initialized():
        dist.barrier()
    wall = torch.tensor([time.perf_counter() - t0], device=dev, dtype=torch.float64)
    if dist.is_initialized():
        dist.all_reduce(wall, op=dist.ReduceOp.MAX)
    return float(wall.item())


def _synthetic_actions(n: int, T: int, dev, seed: int, sigma: float):
    import torch  # noqa: PLC0415
    from zbot_amd import cstructs as cs  # noqa: PLC0415
    from zbot_amd.constants import JOINT_BIASES  # noqa: PLC0415

    g = torch.Generator(device=dev)
    g.manual_seed(seed)
    bias = torch.tensor([b for _, b, _ in JOINT_BIASES], device=dev)
    return bias + sigma * torch.randn(T, n, cs.NJ, device=dev, generator=g)


def bench_ksim_env(cm, n: int, steps: int, warmup: int, dev, rank: int, world: int, seed: int) -> dict:
    """The headline workload driven through the ksim-shaped API (zbot_amd.task.ZbotWalkingEnv.step,
    train.py's ZbotWalkingTask): its default env groups (two from 4096 envs up), every output a
    StepResult (observations incl. the extra ones, reward terms), curriculum level passed per
    step. The loop does not read the results, as an open-loop rollout does not, so the groups are
    never joined between steps."""
    from zbot_amd.task import ZbotWalkingEnv  # noqa: PLC0415

    env = ZbotWalkingEnv(n, seed=seed, device=dev.index, env_offset=rank * n, model=cm)
    acts = _synthetic_actions(n, 64, dev, 1234 + rank, 0.05)
    env.reset()
    wall = _timed_steps(lambda t: env.step(acts[t % 64]), steps, warmup, dev, world)
    return {
        "workload": f"C2 through ZbotWalkingEnv.step: {n} envs/GPU, {env.groups} env groups, {steps} timed steps "
                    f"(after {warmup}), every StepResult output written (obs_extra and reward terms included)",
        "env_steps_per_s": world * n * steps / wall,
        "ms_per_step": 1e3 * wall / steps,
        "groups": env.groups,
    }


# the step kernel's SQ wave-cycle PMC pass (scripts/pmc_latency.sh -> profiles/), per (solver, envs)
LATENCY_FILE = "r06_pmc_latency.json"


def latency_block(solver: str, n: int, kernel_ms: float, substeps: int, cus: int, train_leg: dict | None) -> dict | None:
    """The step kernel against its latency floor: from the SQ wave-cycle PMC pass of the
    same kernel (scripts/pmc_latency.sh, LATENCY_FILE), per physics substep and wave, the wave's lifetime
    (SQ_WAVE_CYCLES) and its issue floor (SQ_ACTIVE_INST_ANY: the cycles the wave spends issuing, its
    lifetime if no instruction ever waited on a dependency); latency_frac = floor / lifetime. At 512 envs
    (train.py's size: 256 waves, each alone on its SIMD) that is the kernel's whole budget; at the
    headline's 8192 two waves share each SIMD and the partner's issue counts as wait. The live part:
    the kernel's HIP-event time over rounds x the PMC wave lifetime gives the clock the live run ran at
    (a check that the profile and the timed run are the same kernel: MI355X runs 1.9-2.4 GHz)."""
    path = os.path.join(ROOT, "profiles", LATENCY_FILE)
    if not os.path.exists(path):
        return None
    with open(path) as f:
        lj = json.load(f)

    def row(envs):
        r = lj.get(f"{solver}_{envs}")
        if r is None:
            return None
        ps = r["per_substep"]
        return {"envs": envs, "wave_lifetime_cycles_per_substep": ps["lifetime_cycles"],
                "issue_floor_cycles_per_substep": ps["issue_floor_cycles"], "latency_frac": r["latency_frac"],
                "valu_insts_per_wave": r["per_wave"]["INSTS_VALU"]}

    out = {"kernel": "zb::step_kernel", "solver": solver, "source": f"profiles/{LATENCY_FILE} (scripts/pmc_latency.sh)",
           "train_size": row(512), "bench_size": row(n)}
    b = out["bench_size"]
    if b is not None and kernel_ms > 0:
        # the n envs' waves over all of the GPU's wave slots (the env groups' launches run concurrently,
        # each lasting about as long as the rounds of the whole set)
        waves = n // 2  # two envs per wave
        rounds = -(-waves // (cus * 4 * 2))  # 256 VGPRs: two waves per SIMD, four SIMDs per CU
        out["live"] = {"kernel_ms": kernel_ms, "rounds": rounds,
                       "implied_clock_ghz": rounds * b["wave_lifetime_cycles_per_substep"] * substeps / (kernel_ms * 1e6)}
    if train_leg is not None:
        out["train_defaults_ms_per_step"] = train_leg.get("ms_per_step")
    return out


def bench_train_defaults(cm, dev, rank: int, world: int, seed: int, n: int = 512, T: int = 200) -> dict:
    """train.py's own training size (train.py:1770 num_envs=512, :1775 rollout_length_seconds 4.0 at
    ctrl_dt 0.02 = 200 steps): one 200-step rollout of 512 envs per GPU from reset through
    ZbotWalkingEnv (one handle below 4096 envs), [T, n] reward / done rows, FeetAirtime row 0
    patched; actions JOINT_BIASES + 0.2 N(0,1). Latency-bound: 512 envs are 256 waves on 1024
    SIMDs."""
    import torch  # noqa: PLC0415
    from zbot_amd.task import ZbotWalkingEnv  # noqa: PLC0415

    env = ZbotWalkingEnv(n, seed=seed, device=dev.index, env_offset=rank * n, model=cm)
    eng = env.engine
    acts = _synthetic_actions(n, T, dev, 777 + rank, 0.2)
    rew = torch.empty(T, n, device=dev)
    done = torch.empty(T, n, dtype=torch.uint8, device=dev)

    def rollout(_):
        eng.mark_rollout_start()
        for t in range(T):
            eng.step(acts[t], curriculum=env.curriculum_level, reward=rew[t], done=done[t])
        eng.feet_airtime_exact(rew[0], None, curriculum=env.curriculum_level)

    env.reset()
    wall = _timed_steps(rollout, 2, 1, dev, world)
    assert bool(torch.isfinite(rew).all())
    return {
        "workload": f"train.py defaults: {n} envs/GPU x {T}-step rollout (train.py:1770,1775), one handle, automatic "
                    "resets inside, [T, n] reward / done rows, FeetAirtime row 0 patched; 2 timed rollouts after 1",
        "env_steps_per_s": world * n * T * 2 / wall,
        "ms_per_rollout": 1e3 * wall / 2,
        "ms_per_step": 1e3 * wall / (2 * T),
        "episodes_done": int(done.sum().item()),
    }


def bench_c1(cm, dev, rank: int, world: int, seed: int, n: int = 64, T: int = 128) -> dict:
    """BASELINE configs[0] on the GPU: the reference's own CPU case (64 envs x 128-step rollout) as
    one handle's 128 zb_step launches from reset, beside cpu_baseline.c1 (the CPU twin on the same
    shape). 64 envs are 32 waves: each control step lasts as long as its slowest env."""
    import torch  # noqa: PLC0415
    from zbot_amd.config import default_config  # noqa: PLC0415
    from zbot_amd.engine import HipEngine  # noqa: PLC0415

    eng = HipEngine(cm, default_config(), n, env_offset=rank * n, device=dev.index, seed=seed)
    acts = _synthetic_actions(n, T, dev, 64 + rank, 0.05)

    def rollout(_):
        eng.reset()
        for t in range(T):
            eng.step(acts[t], extras=False)

    wall = _timed_steps(rollout, 2, 1, dev, world)
    return {
        "workload": f"C1 on the GPU: {n} envs/GPU x {T}-step rollout from reset (BASELINE configs[0]), one handle, "
                    "2 timed rollouts after 1",
        "env_steps_per_s": world * n * T * 2 / wall,
        "ms_per_rollout": 1e3 * wall / 2,
        "ms_per_step": 1e3 * wall / (2 * T),
    }


def bench_general_colliders(cfg, n: int, steps: int, warmup: int, dev, rank: int, world: int, seed: int,
                            groups: int, asset: str = "zbot_like_limbs.xml") -> dict:
    """C2 on the limbs model (assets/zbot_like_limbs.xml: a shin box and a hand capsule collide with
    the floor besides the soles), which runs the general-collider kernel instantiation (DESIGN.md
    §4j); same groups and actions as the headline. asset="zbot_like_cyl.xml": the cylinder foot,
    cylinder shin and ellipsoid hand model (the third instantiation); "zbot_like_mesh.xml": the convex
    mesh right sole, shin and hand (the same instantiation, MJX's plane_convex, §4j); "zbot_like_many.xml":
    nine colliders, the second bank chosen per substep (§4j)."""
    from zbot_amd import compile_model  # noqa: PLC0415
    from zbot_amd.engine import EnvGroups, HipEngine  # noqa: PLC0415
    from zbot_amd.mjcf import load_mjcf  # noqa: PLC0415

    path = os.path.join(ROOT, "ksim-gym-zbot_amd", "assets", asset)
    cm = compile_model(load_mjcf(path))
    if groups > 1:
        eng = EnvGroups(cm, cfg, n, groups=groups, env_offset=rank * n, device=dev.index, seed=seed)
    else:
        eng = HipEngine(cm, cfg, n, env_offset=rank * n, device=dev.index, seed=seed)
    acts = _synthetic_actions(n, 64, dev, 1234 + rank, 0.05)
    eng.reset()

    wall = _timed_steps(lambda t: eng.step(acts[t % 64], extras=False), steps, warmup, dev, world)
    eng.check()
    out = {
        "workload": f"C2 on {os.path.relpath(path, ROOT)} ({len(cm.geom_names)} floor colliders "
                    f"{cm.geom_names}), {n} envs/GPU, {groups} env groups, {steps} timed steps (after {warmup})",
        "env_steps_per_s": world * n * steps / wall,
        "ms_per_step": 1e3 * wall / steps,
    }
    if len(cm.geom_names) > 4:
        # the second bank's two-geom cap (select_bank2): envs that ever had more than two colliders beyond
        # the soles within reach of the floor in a substep of the run (their contacts not simulated)
        out["bank2_overflow_envs"] = int(eng.flags()["bank_overflow"].sum().item())
    return out


def bench_variant(cm, cfg, label: str, flops_file: str, n: int, steps: int, warmup: int, dev, rank: int, world: int,
                  seed: int, groups: int) -> dict:
    """C2 with one of the [U] physics switches flipped: the solver (CG instead of
    Newton) or mj_Euler's implicit joint damping (ZB_F_EULERDAMP). Same envs, groups, actions and
    timing as the headline (per-launch HIP events on each group's stream), with its own roofline:
    the same algorithmic bytes, and the counted FLOPs of that configuration (scripts/count_flops.py)."""
    import torch  # noqa: PLC0415
    from zbot_amd.engine import EnvGroups, HipEngine  # noqa: PLC0415
    from zbot_amd.metrics import FP32_PEAK_TFLOPS, HBM_PEAK_GBS, bytes_per_env_step  # noqa: PLC0415

    G = max(1, groups)
    eng = (EnvGroups(cm, cfg, n, groups=G, env_offset=rank * n, device=dev.index, seed=seed) if G > 1 else
           HipEngine(cm, cfg, n, env_offset=rank * n, device=dev.index, seed=seed))
    acts = _synthetic_actions(n, 64, dev, 1234 + rank, 0.05)
    eng.reset()
    stream = torch.cuda.current_stream(dev)
    ev = [[(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(G)]
          for _ in range(steps)]
    for evt in ev:
        for a, b in evt:
            a.record(stream)
            b.record(stream)

    def step(t):
        k = t - warmup
        if G > 1:
            eng.step(acts[t % 64], extras=False, events=ev[k] if k >= 0 else None)
        else:
            if k >= 0:
                ev[k][0][0].record(stream)
            eng.step(acts[t % 64], extras=False)
            if k >= 0:
                ev[k][0][1].record(stream)
        if G > 1 and t == warmup + steps - 1:
            eng.join()

    wall = _timed_steps(step, steps, warmup, dev, world)
    eng.check()
    avg_ms = sum(a.elapsed_time(b) for evt in ev for a, b in evt) / (steps * G)
    wall_ms = 1e3 * wall / steps
    rate_ms = avg_ms if G == 1 else max(avg_ms, wall_ms)
    bpe = bytes_per_env_step(extras=False, terms=True)
    hbm = bpe * n / (rate_ms * 1e-3) / 1e9
    out = {
        "workload": f"C2 with {label}: {n} envs/GPU, {G} env groups, {steps} timed steps (after {warmup})",
        "env_steps_per_s": world * n * steps / wall,
        "ms_per_step": wall_ms,
        "avg_solver_iters_per_env_step": eng.solver_iters().float().mean().item(),
        "roofline": {"bound": "hbm", "achieved": hbm, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": hbm / HBM_PEAK_GBS,
                     "kernel_avg_ms": avg_ms, "rate_ms": rate_ms, "algorithmic_bytes_per_env_step": bpe},
    }
    fpath = os.path.join(ROOT, "profiles", flops_file)
    if flops_file and os.path.exists(fpath):
        with open(fpath) as f:
            fl = json.load(f)["as_run"]["flops_per_env_step"]
        tf = fl * n / (rate_ms * 1e-3) / 1e12
        out["roofline_fp32"] = {"bound": "fp32-valu", "achieved": tf, "peak": FP32_PEAK_TFLOPS, "unit": "TFLOP/s",
                                "frac": tf / FP32_PEAK_TFLOPS, "algorithmic_flop_per_env_step": fl,
                                "flops_file": os.path.relpath(fpath, ROOT)}
    return out


def bench_policy_in_loop(eng, n: int, steps: int, dev, rank: int, grouped=None) -> dict:
    """The GRU actor in the rollout loop: per control step the actor samples
    every env's action from its observation on the f32 matrix cores, then zb_step advances the
    envs (ksim sample_action -> env.step, train.py:1737-1763). The actor's kernel time and roofline
    come from one handle on the current stream with the 8-wave actor (isolated launches). With
    `grouped` (an EnvGroups) the leg's throughput is PolicyRollout running
    each group's actor -> zb_step chain on its own stream with the two-wave slot-sized actor layout, whose
    workgroups fit the slots the other groups' step launches free."""
    import torch  # noqa: PLC0415
    from zbot_amd import policy as P  # noqa: PLC0415
    from zbot_amd.metrics import FP32_PEAK_TFLOPS  # noqa: PLC0415

    actor = P.GruPolicy(P.ACTOR, P.init_params(P.ACTOR, seed=0), device=dev.index)
    carry = actor.initial_carry(n)
    acts = torch.empty(n, P.JOINTS, device=dev)
    eng.reset(extras=False)
    stream = torch.cuda.current_stream(dev)

    def one(t, ev=None):
        if ev is not None:
            ev[0].record(stream)
        actor.actor(eng.obs_actor, carry, reset=eng.done if t > 0 else None, seed=1, env_offset=rank * n, step=t,
                    actions=acts)
        if ev is not None:
            ev[1].record(stream)
        eng.step(acts, extras=False)

    for t in range(2):
        one(t)
    torch.cuda.synchronize(dev)
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
    t0 = time.perf_counter()
    for t in range(steps):
        one(2 + t, evs[t])
    torch.cuda.synchronize(dev)
    wall = time.perf_counter() - t0
    actor_ms = sum(a.elapsed_time(b) for a, b in evs) / steps
    tf = P.FLOP_ACTOR * n / (actor_ms * 1e-3) / 1e12
    out = {
        "workload": f"GRU actor (5 x GRU 128, mixture-of-Gaussians head) sampling the actions of {n} envs, then "
                    "zb_step, per control step",
        "env_steps_per_s_with_policy": n * steps / wall,
        "actor_kernel_ms": actor_ms,
        "roofline": {"bound": "mfma", "achieved": tf, "peak": FP32_PEAK_TFLOPS, "unit": "TFLOP/s",
                     "frac": tf / FP32_PEAK_TFLOPS, "kernel": "zb::pol::policy_kernel<50, 300, true>",
                     "flop_per_env_step": P.FLOP_ACTOR, "dtype": "f32 (v_mfma_f32_16x16x4_f32)"},
    }
    if grouped is not None:
        actor.set_layout(P.LAYOUT_WAVE2)
        ro = P.PolicyRollout(grouped, actor, seed=1)
        ro.reset()
        ro.run(2)
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        ro.run(steps)
        torch.cuda.synchronize(dev)
        out["env_steps_per_s_with_policy_one_stream"] = out["env_steps_per_s_with_policy"]
        out["env_steps_per_s_with_policy"] = n * steps / (time.perf_counter() - t0)
        out["workload"] += (f"; {grouped.G} env groups, each running its actor (two-wave slot-sized layout) -> "
                            "zb_step chain on its own stream")
    return out


def bench_rollout_pipeline(eng, n: int, T: int, reps: int, dev, world: int, inloop_critic: int = 0) -> dict:
    """One PPO rollout per GPU end to end, everything before the PPO loss (SURVEY §8f f1 + f2):
    T control steps of GRU-actor sampling -> zb_step with the critic observations recorded
    (ksim rollout, sample_action train.py:1737-1763), the GRU critic over the T steps with the
    carry reset on episode ends (get_ppo_variables, train.py:1683-1729), then GAE, value targets
    and advantage normalization with the batch moments combined over RCCL (ksim
    compute_ppo_inputs [U]). Value: env-steps of the whole job per second of wall time."""
    import torch  # noqa: PLC0415
    import torch.distributed as dist  # noqa: PLC0415
    from zbot_amd import policy as P  # noqa: PLC0415
    from zbot_amd.ppo import compute_ppo_inputs  # noqa: PLC0415

    actor = P.GruPolicy(P.ACTOR, P.init_params(P.ACTOR, seed=0), device=dev.index,
                        layout=P.LAYOUT_WAVE2 if hasattr(eng, "groups") else P.LAYOUT_BLOCK)
    # the critic runs over the whole rollout afterwards, 8-wave layout on the current stream: inside
    # the group chains (PolicyRollout.run(critic=...), one-wave layout) it measured slower,
    # 5.49 M vs 6.02 M env-steps/s (profiles/r02_v16d_bench_inloop_critic.json)
    critic = P.GruPolicy(P.CRITIC, P.init_params(P.CRITIC, seed=1), device=dev.index)
    inloop = bool(inloop_critic) and hasattr(eng, "groups")
    if inloop:  # --inloop-critic L: V(s_t) inside the group chains with policy layout L
        critic.set_layout(inloop_critic)
    ro = P.PolicyRollout(eng, actor, seed=3)
    ro.reset()
    zeros = torch.zeros(1, n, dtype=torch.uint8, device=dev)

    def once():
        if inloop:
            cc = critic.initial_carry(n)
            traj = ro.run(T, record_critic=True, critic=critic, critic_carry=cc)
            return compute_ppo_inputs(traj["value"], traj["reward"], traj["done"], traj["success"],
                                      bootstrap=traj["value_next"])
        traj = ro.run(T, record_critic=True)
        cc = critic.initial_carry(n)
        # V(s_t) on the states acted in (carry reset where an episode starts), then the
        # bootstrap V(s_T) with the carry the rollout ends with
        values = critic.critic(traj["obs_critic"], cc, reset=torch.cat([zeros, traj["done"][:-1]]))
        boot = critic.critic(traj["obs_critic_next"], cc, reset=traj["done"][-1])
        return compute_ppo_inputs(values, traj["reward"], traj["done"], traj["success"], bootstrap=boot)

    once()  # first use of every kernel and of the moment collective, untimed
    torch.cuda.synchronize(dev)
    if dist.is_initialized():
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(reps):
        res = once()
    torch.cuda.synchronize(dev)
    if dist.is_initialized():
        dist.barrier()
    wall = torch.tensor([time.perf_counter() - t0], device=dev, dtype=torch.float64)
    if dist.is_initialized():
        dist.all_reduce(wall, op=dist.ReduceOp.MAX)
    wall = float(wall.item())
    assert bool(torch.isfinite(res.advantages_t).all())
    return {
        "workload": f"per GPU: {T}-step rollout of {n} envs with the GRU actor sampling every action, the GRU "
                    "critic over the rollout, GAE + value targets + advantage normalization (moments over RCCL)"
                    + (f"; the rollout over {eng.G} env groups (two-wave slot-sized actor), the critic (8-wave) "
                       "over the rollout afterwards" if hasattr(eng, "groups") else ""),
        "env_steps_per_s": world * n * T * reps / wall,
        "ms_per_rollout": 1e3 * wall / reps,
        "rollout_steps": T,
    }


def _free_port() -> int:
    import socket  # noqa: PLC0415

    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank_entry(local_rank: int, world: int, port: int, argv: list) -> None:
    """One spawned rank of a self-launched `bench.py --gpus N`: the torch.distributed.run environment
    (rank = local rank on this one node), then the same main() as under torchrun."""
    os.environ.update(RANK=str(local_rank), LOCAL_RANK=str(local_rank), WORLD_SIZE=str(world),
                      LOCAL_WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    main(argv)


def launch_ranks(world: int, argv: list) -> int:
    """`bench.py --gpus N` without torchrun: start N rank processes (spawn: fresh interpreters; this
    parent makes no GPU call, it only counts devices, which does not initialise HIP on this image)
    and wait for all of them. Returns the exit status (non-zero if any rank failed)."""
    import torch.multiprocessing as mp  # noqa: PLC0415

    try:
        mp.start_processes(_rank_entry, args=(world, _free_port(), argv), nprocs=world, join=True,
                           start_method="spawn")
    except mp.ProcessExitedException as e:  # a rank exited non-zero (2: a world / device mismatch)
        print(f"bench.py: a rank failed: {e}", file=sys.stderr, flush=True)
        return 2 if e.exit_code == 2 else 1
    except Exception as e:  # ProcessRaisedException: a rank raised
        print(f"bench.py: a rank failed: {e}", file=sys.stderr, flush=True)
        return 1
    return 0


def check_world(args) -> tuple[int, bool]:
    """The world size bench.py will run at, and whether this process must launch the ranks itself.
    --gpus N is authoritative: under torchrun WORLD_SIZE must equal it. Exits with status 2 on a
    mismatch. No device query here: a self-launching parent must not touch HIP (torch's device count
    falls back to hipGetDeviceCount when amdsmi is absent), so each rank checks the devices itself
    (check_devices)."""
    env = os.environ.get("WORLD_SIZE")
    if env is not None and int(env) != args.gpus:
        print(f"bench.py: WORLD_SIZE={env} but --gpus {args.gpus}: launch exactly --gpus ranks", file=sys.stderr)
        sys.exit(2)
    if args.gpus < 1:
        print(f"bench.py: --gpus {args.gpus} < 1", file=sys.stderr)
        sys.exit(2)
    return args.gpus, env is None and args.gpus > 1


def check_devices(args) -> None:
    """In a rank process (never the self-launching parent): the nccl backend (RCCL, one rank per GPU)
    needs --gpus visible devices. Exits with status 2 before any other GPU call."""
    import torch  # noqa: PLC0415

    if args.gpus > 1 and args.dist_backend == "nccl":
        ndev = torch.cuda.device_count()
        if ndev < args.gpus:
            print(f"bench.py: --gpus {args.gpus} with the nccl backend (RCCL, one rank per GPU) but only {ndev} "
                  "device(s) are visible", file=sys.stderr)
            sys.exit(2)


def launch_probe(world: int, backend: str) -> None:
    """--launch-probe: the multi-rank launch alone, no GPU work (CPU-testable with gloo): every rank
    joins the process group and all_gathers its rank; rank 0 prints the ranks it saw."""
    import torch  # noqa: PLC0415
    import torch.distributed as dist  # noqa: PLC0415

    rank = int(os.environ.get("RANK", "0"))
    if world > 1:
        dist.init_process_group(backend)
    seen = [None] * world
    if dist.is_initialized():
        dist.all_gather_object(seen, rank)
    else:
        seen = [rank]
    if rank == 0:
        print(json.dumps({"n_gpus": world, "ranks_seen": dist.get_world_size() if dist.is_initialized() else 1,
                          "ranks": seen, "pid_parent": os.getppid(), "torch": torch.__version__}), flush=True)
    if dist.is_initialized():
        dist.destroy_process_group()


def main(argv: list | None = None) -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=64)
    ap.add_argument("--warmup", type=int, default=8)
    ap.add_argument("--envs", type=int, default=0, help="envs per GPU (default: the config's)")
    ap.add_argument("--config", default="c2", choices=sorted(CONFIGS))
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--model", default=None,
                    help="robot: an MJCF (.xml) or descriptor (.json) file instead of the default Z-Bot-like "
                         "descriptor, e.g. ksim-gym-zbot_amd/assets/zbot_like_limbs.xml (colliders beyond the "
                         "soles: the general-collider kernels); roofline FLOP / traffic stay the default model's")
    ap.add_argument("--solver", default="cg", choices=["newton", "cg"],
                    help="constraint solver (ZbEnvConfig.solver): MJX's CG (default: the one ksim's model setup "
                         "selects, [U] DESIGN.md §8) or MuJoCo's Newton (the newton_solver leg)")
    ap.add_argument("--groups", type=int, default=2,
                    help="env groups per GPU, each stepping on its own HIP stream (zbot_amd.EnvGroups, "
                         "DESIGN.md §4f); 1 = one handle on the current stream")
    ap.add_argument("--policy-groups", type=int, default=3,
                    help="env groups of the actor-in-the-loop legs (two-wave slot-sized actor layout; DESIGN.md §4f); "
                         "1 = one handle, 8-wave actor, current stream")
    ap.add_argument("--cpu-baseline-sec", type=float, default=12.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-ppo", action="store_true", help="skip the post-rollout PPO-inputs leg")
    ap.add_argument("--no-policy", action="store_true", help="skip the policy-in-the-loop leg")
    ap.add_argument("--no-pipeline", action="store_true", help="skip the end-to-end rollout-pipeline leg")
    ap.add_argument("--no-c2-rollout", action="store_true",
                    help="skip the C2-as-stated leg (one 256-step rollout with resets inside, timed whole)")
    ap.add_argument("--no-extra-legs", action="store_true",
                    help="skip the ksim_env (ZbotWalkingEnv.step), train_defaults (512 x 200), c1_gpu, "
                         "general_colliders (limbs model), cylinder_colliders (cyl model), mesh_colliders (mesh "
                         "model), many_colliders (nine colliders), the other solver's "
                         "(cg_solver / newton_solver), sole_pair, sole_pair_limbs, mjx_box_rule and eulerdamp legs")
    ap.add_argument("--inloop-critic", type=int, default=0,
                    help="rollout-pipeline leg: run the critic inside the group chains with this policy layout "
                         "(1 one-wave, 2 two-wave, 3 four-wave; DESIGN.md §4f); 0 = the 8-wave critic afterwards")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="torch.distributed backend for N > 1 (nccl = RCCL over xGMI; gloo rehearses the "
                         "multi-rank path on a one-GPU box, ranks sharing device local_rank %% device_count)")
    ap.add_argument("--init-dist", action="store_true",
                    help="initialise the process group even at WORLD_SIZE 1 (under torch.distributed.run with one "
                         "rank): the barriers, the max-over-ranks timer and the statistics all_gather then run "
                         "through RCCL on a one-GPU box")
    ap.add_argument("--launch-probe", action="store_true",
                    help="run only the multi-rank launch (process group + all_gather of the ranks), no GPU work")
    argv = sys.argv[1:] if argv is None else argv
    args = ap.parse_args(argv)

    # --gpus N is authoritative (before any GPU call): torchrun's WORLD_SIZE must equal it, and
    # without torchrun this process starts the N ranks itself
    world, self_launch = check_world(args)
    if self_launch:
        sys.exit(launch_ranks(world, argv))
    if args.launch_probe:
        launch_probe(world, args.dist_backend)
        return
    check_devices(args)

    import torch  # noqa: PLC0415
    import torch.distributed as dist  # noqa: PLC0415
    from zbot_amd import compile_model, default_config  # noqa: PLC0415
    from zbot_amd import cstructs as cs  # noqa: PLC0415
    from zbot_amd.constants import JOINT_BIASES  # noqa: PLC0415
    from zbot_amd.dist import reduce_episode_stats  # noqa: PLC0415
    from zbot_amd.engine import EnvGroups, HipEngine  # noqa: PLC0415
    from zbot_amd.metrics import FP32_PEAK_TFLOPS, HBM_PEAK_GBS, bytes_per_env_step  # noqa: PLC0415

    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    dev = torch.device("cuda", local_rank % max(torch.cuda.device_count(), 1))
    torch.cuda.set_device(dev)
    if world > 1 or args.init_dist:
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group("gloo")
        if dist.get_world_size() != world:
            print(f"bench.py: the process group has {dist.get_world_size()} ranks, --gpus {world}", file=sys.stderr)
            sys.exit(2)

    conf = CONFIGS[args.config]
    n = args.envs or conf["envs"]
    if args.model is None:
        cm = compile_model()
    elif args.model.endswith(".xml"):
        from zbot_amd.mjcf import load_mjcf  # noqa: PLC0415

        cm = compile_model(load_mjcf(args.model))
    else:
        cm = compile_model(args.model)
    cfg = default_config(push=conf["push"], randomize=conf["randomize"], solver=args.solver)
    G = max(1, args.groups)
    if G > 1:
        eng = EnvGroups(cm, cfg, n, groups=G, env_offset=rank * n, device=dev.index, seed=args.seed)
    else:
        eng = HipEngine(cm, cfg, n, env_offset=rank * n, device=dev.index, seed=args.seed)

    # synthetic actions for the headline env-step leg, generated before timing (the
    # policy-in-the-loop leg below drives the same engine with the GRU actor instead)
    T = args.warmup + args.steps
    g = torch.Generator(device=dev)
    g.manual_seed(1234 + rank)
    bias = torch.tensor([b for _, b, _ in JOINT_BIASES], device=dev)
    acts = bias + 0.05 * torch.randn(min(T, 64), n, cs.NJ, device=dev, generator=g)

    def reduce_stats():
        # per-rollout episode statistics: per-GPU partials summed in fixed env order, then an RCCL
        # all_gather and a sequential rank-order sum (zbot_amd.dist.reduce_fixed_order: bit-reproducible)
        return reduce_episode_stats(eng.get_stats(clear=False))

    # The other legs run first: their work (about two seconds of GPU time) brings the GPU to its
    # steady clocks before the headline's own W warm-up steps and K timed steps; in a fresh
    # process the first timed window otherwise ran ~4 % slower kernels (profiles/r03_v3_probe20_g*.json)
    c2_leg = None if args.no_c2_rollout else bench_c2_rollout(eng, n, 256, dev, rank, world)
    ppo_leg = None if args.no_ppo else bench_ppo_inputs(n, 256, 20, dev, world)
    # the actor-in-the-loop legs: one handle on the current stream for the actor's kernel time, and
    # args.policy_groups env groups with the slot-sized two-wave actor
    eng1 = eng if G == 1 else None
    engp = None
    if not (args.no_policy and args.no_pipeline):
        if G > 1:
            eng1 = HipEngine(cm, cfg, n, env_offset=rank * n, device=dev.index, seed=args.seed)
        if args.policy_groups > 1:
            engp = EnvGroups(cm, cfg, n, groups=args.policy_groups, env_offset=rank * n, device=dev.index,
                             seed=args.seed)
    policy_leg = None if args.no_policy else bench_policy_in_loop(eng1, n, 48, dev, rank, engp)
    pipe_leg = None if args.no_pipeline else bench_rollout_pipeline(engp or eng1, n, 32, 2, dev, world,
                                                                     args.inloop_critic)

    extra_legs = {}
    if not args.no_extra_legs and args.config == "c2" and args.model is None:
        extra_legs["ksim_env"] = bench_ksim_env(cm, n, args.steps, args.warmup, dev, rank, world, args.seed)
        extra_legs["train_defaults"] = bench_train_defaults(cm, dev, rank, world, args.seed)
        extra_legs["c1_gpu"] = bench_c1(cm, dev, rank, world, args.seed)
        extra_legs["general_colliders"] = bench_general_colliders(cfg, n, args.steps, args.warmup, dev, rank, world,
                                                                  args.seed, G)
        extra_legs["cylinder_colliders"] = bench_general_colliders(cfg, n, args.steps, args.warmup, dev, rank, world,
                                                                   args.seed, G, "zbot_like_cyl.xml")
        extra_legs["mesh_colliders"] = bench_general_colliders(cfg, n, args.steps, args.warmup, dev, rank, world,
                                                               args.seed, G, "zbot_like_mesh.xml")
        extra_legs["many_colliders"] = bench_general_colliders(cfg, n, args.steps, args.warmup, dev, rank, world,
                                                               args.seed, G, "zbot_like_many.xml")
        # the [U] physics switches timed both ways: the other solver, and implicit damping
        other = "cg" if args.solver == "newton" else "newton"
        extra_legs[f"{other}_solver"] = bench_variant(
            cm, default_config(solver=other), f"the {other.upper() if other == 'cg' else 'Newton'} solver (ZbEnvConfig.solver)",
            FLOPS_FILES[(other, "base")], n, args.steps, args.warmup, dev, rank, world, args.seed, G)
        from zbot_amd.mjcf import load_mjcf  # noqa: PLC0415
        from zbot_amd.model import load_description  # noqa: PLC0415

        pdesc = load_description()
        pdesc["self_pairs"] = [["left_foot_sole", "right_foot_sole"]]
        extra_legs["sole_pair"] = bench_variant(
            compile_model(pdesc), default_config(solver=args.solver),
            "the sole-pair model (the soles also collide with each other, box-box; the XG 3 kernels, DESIGN.md §4l)",
            FLOPS_FILES[(args.solver, "solepair")], n, args.steps, args.warmup, dev, rank, world, args.seed, G)
        ldesc = load_mjcf(os.path.join(ROOT, "ksim-gym-zbot_amd", "assets", "zbot_like_limbs.xml"))
        ldesc["self_pairs"] = [["left_foot_sole", "right_foot_sole"]]
        extra_legs["sole_pair_limbs"] = bench_variant(
            compile_model(ldesc), default_config(solver=args.solver),
            "the sole pair beside the limbs model's shin box and hand capsule (the XG 4 kernels: floor colliders in "
            "the second bank, the pair in a third; DESIGN.md §4l)",
            "", n, args.steps, args.warmup, dev, rank, world, args.seed, G)
        extra_legs["mjx_box_rule"] = bench_variant(
            compile_model(box_rule="mjx"), default_config(solver=args.solver),
            "the box soles collided by MJX's plane_convex manifold (compile_model(box_rule='mjx'): each an 8-corner "
            "convex mesh, the XG 2 kernels, DESIGN.md §8)",
            FLOPS_FILES[(args.solver, "mjxbox")], n, args.steps, args.warmup, dev, rank, world, args.seed, G)
        extra_legs["eulerdamp"] = bench_variant(
            cm, default_config(solver=args.solver, eulerdamp=True),
            f"mj_Euler's implicit joint damping (ZB_F_EULERDAMP), {args.solver} solver",
            FLOPS_FILES[(args.solver, "eulerdamp")], n, args.steps, args.warmup, dev, rank, world, args.seed, G)

    eng.reset()
    for t in range(args.warmup):
        eng.step(acts[t % acts.shape[0]], extras=False)
    # the reduction's kernels and collective run once untimed: their first use loads code
    # objects / sets up the RCCL communicator, one-time costs that are not per-step work
    reduce_stats()
    eng.get_stats(clear=True)
    stream = torch.cuda.current_stream(dev)
    # per-launch HIP events on the stream each launch runs on (one per group and step); torch
    # creates an event's HIP handle at its first record: do that here, not inside the timed loop
    ev = [[(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(G)]
          for _ in range(args.steps)]
    for evt in ev:
        for a, b in evt:
            a.record(stream)
            b.record(stream)
    torch.cuda.synchronize(dev)
    if dist.is_initialized():
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for t in range(args.steps):
        a_t = acts[(args.warmup + t) % acts.shape[0]]
        if G > 1:
            eng.step(a_t, extras=False, events=ev[t])
        else:
            ev[t][0][0].record(stream)
            eng.step(a_t, extras=False)
            ev[t][0][1].record(stream)
    if G > 1:
        eng.join()
    total_stats = reduce_stats()
    torch.cuda.synchronize(dev)
    if dist.is_initialized():
        dist.barrier()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    el_t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
    if dist.is_initialized():
        dist.all_reduce(el_t, op=dist.ReduceOp.MAX)
    elapsed = float(el_t.item())

    eng.check()  # no launch flagged its results invalid (zb_check)
    kern_ms = [a.elapsed_time(b) for evt in ev for a, b in evt]
    avg_ms = sum(kern_ms) / len(kern_ms)
    wall_ms = 1e3 * elapsed / args.steps
    bpe = bytes_per_env_step(extras=False, terms=True)
    # G launches of n/G envs run concurrently, one per group stream. G x (bytes of n/G envs) / the
    # average launch duration assumes they overlap fully; when they do not, the wall time per step
    # is the longer one, so the rate is taken over max(launch average, wall time per step)
    rate_ms = avg_ms if G == 1 else max(avg_ms, wall_ms)
    achieved = bpe * n / (rate_ms * 1e-3) / 1e9
    iters = eng.solver_iters().float().mean().item()

    # HBM bytes per launch and issued fp32 FLOP per env-step from the separate
    # rocprofv3 PMC passes of the same kernel (scripts/pmc_traffic.sh)
    traffic = None
    flop_per_env_step = None
    tpath = os.path.join(ROOT, "profiles", f"pmc_traffic_{args.config}.json")
    if os.path.exists(tpath):
        with open(tpath) as f:
            tj = json.load(f)
        # the PMC passes ran one solver's kernel (the file records which; round-5 files: Newton)
        if tj.get("envs") == n and tj.get("solver", "newton") == args.solver:
            traffic = tj.get("hbm_bytes_per_launch")
            flop_per_env_step = tj.get("issued_fp32_flop_per_env_step")
    # algorithmic FLOPs per env-step, counted by the instrumented CPU twin on the C2 workload
    # (scripts/count_flops.py)
    algo_flop = None
    fpath = os.path.join(ROOT, "profiles", FLOPS_FILES[(args.solver, "base")])
    if os.path.exists(fpath):
        with open(fpath) as f:
            algo_flop = json.load(f)["as_run"]["flops_per_env_step"]

    if rank == 0:
        value = world * n * args.steps / elapsed
        out = {
            "metric": METRIC,
            "value": value,
            "unit": "env-steps/s",
            "n_gpus": world,
            "ranks_seen": dist.get_world_size() if dist.is_initialized() else 1,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": 1e3 * elapsed / args.steps,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic: actions = JOINT_BIASES + 0.05*N(0,1) on the Z-Bot-like descriptor",
            "config": {
                # what the timed region ran: K back-to-back zb_step launches, each one control
                # step (20 physics substeps) of every env, continuing one episode stream
                "workload": conf["name"].format(n=n) + f", {args.steps} timed zb_step launches of one control step "
                                                       f"each (after {args.warmup} warm-up steps)",
                "envs_per_gpu": n,
                "global_envs": world * n,
                "substeps_per_step": cfg.n_substeps,
                "solver": f"{args.solver}, {cfg.iterations} iters / {cfg.ls_iterations} ls iters",
                "parallelism": f"env-shard x{world} (one process per GPU)" + (
                    "" if world == 1 or args.dist_backend == "nccl" else f", {args.dist_backend} rehearsal")
                + (f"; {G} env groups of {n // G} per GPU, each zb_step-ing on its own HIP stream" if G > 1 else ""),
                "groups_per_gpu": G,
                "avg_solver_iters_per_env_step": iters,
                **({"model": args.model, "colliders": cm.geom_names} if args.model else {}),
            },
            "roofline": {
                "bound": "hbm",
                "achieved": achieved,
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBS,
                "traffic": traffic,
                "kernel": "zb::step_kernel",
                "kernel_avg_ms": avg_ms,
                "rate_ms": rate_ms,
                "concurrent_launches": G,
                "envs_per_launch": n // G,
                "traffic_note": "HBM bytes per n env-steps (one launch over all n envs in a separate rocprofv3 --pmc pass, "
                                "FETCH_SIZE x2 + WRITE_SIZE); achieved = algorithmic bytes of the n env-steps of a step / "
                                "rate_ms: the average launch duration by HIP events on the launch's stream (G = 1), or with "
                                "G concurrent group launches the larger of that and the wall time per step",
                "algorithmic_bytes_per_env_step": bpe,
                "note": "the path is FP32-VALU/latency bound (DESIGN.md §Roofline); HBM fraction reported as required",
            },
            "roofline_fp32": None if algo_flop is None else {
                "bound": "fp32-valu",
                "achieved": algo_flop * n / (rate_ms * 1e-3) / 1e12,
                "peak": FP32_PEAK_TFLOPS,
                "unit": "TFLOP/s",
                "frac": algo_flop * n / (rate_ms * 1e-3) / 1e12 / FP32_PEAK_TFLOPS,
                "algorithmic_flop_per_env_step": algo_flop,
                "issued_flop_per_env_step": flop_per_env_step,
                "issued_achieved": None if flop_per_env_step is None else
                flop_per_env_step * n / (rate_ms * 1e-3) / 1e12,
                "note": "achieved = algorithmic FLOPs per env-step (counted by the instrumented CPU twin on the C2 "
                        f"workload with this solver, FMA=2, {os.path.relpath(fpath, ROOT)}) x envs / rate_ms (as "
                        "roofline); issued = PMC "
                        "SQ_INSTS_VALU_{FMA,ADD,MUL,TRANS}_F32 lane-FLOP; the binding resource of this "
                        "latency/VALU-bound kernel",
            },
            "latency": latency_block(args.solver, n, avg_ms, cfg.n_substeps,
                                     torch.cuda.get_device_properties(dev).multi_processor_count,
                                     extra_legs.get("train_defaults")),
            "process_group": dist.get_backend() if dist.is_initialized() else None,
            "episode_stats": {
                "episodes_done": float(total_stats[2].item()),
                "mean_return": float((total_stats[0] / total_stats[2].clamp(min=1)).item()),
            },
        }
        if c2_leg is not None:
            out["c2_rollout"] = c2_leg
        if ppo_leg is not None:
            out["ppo_inputs"] = ppo_leg
        if policy_leg is not None:
            out["policy_in_loop"] = policy_leg
        if pipe_leg is not None:
            out["rollout_pipeline"] = pipe_leg
        for k, leg in extra_legs.items():
            leg["vs_headline"] = leg["env_steps_per_s"] / value
            out[k] = leg
        if world == 1 and not args.no_cpu_baseline:
            if args.config == "c1":  # the whole C1 rollout on the CPU twin: 64 envs x 128 env-steps
                out["cpu_baseline"] = cpu_baseline(cm, cfg, args.cpu_baseline_sec, "C1", n_envs=n, max_steps=128,
                                                   c1_leg=False)
            else:  # the headline's env count (C2: 8192), a bounded number of env-steps
                out["cpu_baseline"] = cpu_baseline(cm, cfg, args.cpu_baseline_sec, args.config.upper(), n_envs=n)
            c1cpu = out["cpu_baseline"].get("c1")
            if c1cpu and "c1_gpu" in out:
                # the same C1 shape on the GPU and on the CPU twin, in one run
                out["c1_gpu"]["vs_cpu_baseline_c1"] = out["c1_gpu"]["env_steps_per_s"] / c1cpu["value"]
        print(json.dumps(out), flush=True)
    if dist.is_initialized():
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
