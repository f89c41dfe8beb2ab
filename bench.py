#!/usr/bin/env python3
"""Headline benchmark: env-steps/s of batched FourRooms 11x11 Hansen-4 (BASELINE.json configs[1]).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--envs B] [--mode numpy|philox] [--strong]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N

Workload (per GPU): `MultistoryFourRoomsEnv(B, grid_z=1, obs_type="hansen")` (FR_MAP, cardinal,
p_fail 1/3, goal (0,7,9), T=500), reset(seed=rank's SeedSequence(0).spawn), random int32 actions in
[0,4) from a pre-generated device buffer. A "step" = one batched env.step over all B envs, with the
reference's RNG reproduced bit-exactly (rng_mode=numpy, the parity-tested mode) — reset draws,
autoreset and obs included. Envs are independent shards: each rank owns its own B envs (weak
scaling, no data-path collective); RCCL only reduces the timing max and the episode metrics.

Prints ONE JSON line (rank 0) with value = total env-steps / max-over-ranks wall time, the live
roofline of the step kernel (HIP-event kernel time on its stream) and the CPU baseline (the numpy
oracle, i.e. the reference's algorithm, timed on this host for a bounded sample).
"""
import argparse
import hashlib
import json
import os
import sys
import time

# Kernel arguments in device memory (a HIP runtime setting, read when HIP initialises: set before torch loads).
# The headline's windowed kernel takes a 52-B argument block (a pointer to its device-resident parameters, K and
# five buffers); the older fused kernels and the C-ROOMS exact-mode draw calls take parameter blocks of ~200-600 B
# by value, which every wave reads at launch: +1.5-8 µs per launch, by box, where the runtime keeps them in host
# memory. The package itself leaves the variable alone; an explicit setting wins.
os.environ.setdefault("HIP_FORCE_DEV_KERNARG", "1")
ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "gym-po-taxi_amd"))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md chip table (spec); 6.29 TB/s measured float4 copy
# Algorithmic bytes per env-step of a ONE-step numpy-mode launch of the two-kernel path (grid_step_numpy +
# grid_resolve_numpy; only used when a timed launch is a single step, never by the default or driver lines):
#   read  action int32 (4) + state agent|elapsed uint32 (4)
#   write state (4) + obs int32 (4) + reward f32 (4) + terminated u8 (1) + truncated u8 (1)
BYTES_PER_ENV_STEP = 22
# Philox fused rollout: per env-step action 4 + obs 4 + reward 4 + term 1 + trunc 1; state once per launch
ROLLOUT_BYTES_PER_ENV_STEP = 14
HEADLINE_METRIC = "env steps/sec (whole node), FourRooms 11x11 Hansen-4 at 1M envs, 1/2/4/8 GPUs"


def _fourrooms(B, dev, mode):
    from gym_po_amd import MultistoryFourRoomsEnv
    return MultistoryFourRoomsEnv(B, grid_z=1, obs_type="hansen", device=dev, rng_mode=mode)


def _taxi_onehot(B, dev, mode):
    from gym_po_amd import HansenTaxiVecEnv
    return HansenTaxiVecEnv(B, device=dev, rng_mode=mode, one_hot=True)


def _crooms(B, dev, mode):
    from gym_po_amd import CRoomsEnv
    return CRoomsEnv(B, obs_type="vector_mdp", device=dev, rng_mode=mode)


def _anttag(B, dev, mode):
    from gym_po_amd import AntTagGridEnv
    return AntTagGridEnv(B, device=dev, rng_mode=mode)


# The headline (BASELINE.json configs[1]) and the other single-GPU configs, measured the same way.
# bytes: algorithmic bytes per env-step of a fused rollout launch; state: bytes per env read + written
# once per launch in SURVEY.md §8(d)'s canonical layout (agent / goal / elapsed int32 = 12 B each way: "14 B + 24/K";
# C-ROOMS 20 B each way): the byte model of `roofline.frac`. state_packed: what the kernels actually keep (one
# packed uint32 per env each way; C-ROOMS its float64 SoA), reported beside it as `frac_packed_state`.
WORKLOADS = {
    "fourrooms": dict(make=_fourrooms, envs=1 << 20, n_actions=4, mode="numpy", bytes=14, state=24, state_packed=8, chunk=128,
                      metric=HEADLINE_METRIC, dtype="int32",
                      desc="configs[1]: FourRooms 11x11 (FR_MAP) Hansen-4 obs, {B} envs per GPU, "
                           "MultistoryFourRoomsEnv(grid_z=1, obs_type='hansen')"),
    "taxi": dict(make=_taxi_onehot, envs=1 << 22, n_actions=5, mode="philox", bytes=4 + 320 + 4 + 1 + 1, state=24, state_packed=8,
                 metric="env steps/sec, PO-Taxi 5x5 Hansen one-hot obs (uint8[320]) at 4M envs per GPU",
                 dtype="uint8", kernel="taxi_rollout<16,false>", chunk=4,
                 desc="configs[2]: PO-Taxi 5x5 (TAXI_MAP) Hansen obs one-hot uint8[B,320], {B} envs per GPU, "
                      "HansenTaxiVecEnv(one_hot=True)"),
    "crooms": dict(make=_crooms, envs=1 << 21, n_actions=None, mode="philox", bytes=8 + 8 + 4 + 1 + 1, state=40, state_packed=40,
                   metric="env steps/sec, C-ROOMS layout 4 continuous (y,x) + N(0,0.2) action noise, 2M envs per GPU",
                   dtype="f64 state / f32 I/O", kernel="crooms_rollout<GP_OBS_F32,false>", chunk=128,
                   desc="configs[4]: C-ROOMS layout 4, yx actions f32 U[-1,1]^2, vector_mdp obs f32[B,2], {B} envs per "
                        "GPU, CRoomsEnv(obs_type='vector_mdp')"),
    "anttag": dict(make=_anttag, envs=1 << 21, n_actions=5, mode="philox", bytes=4 + 16 + 4 + 1 + 1, state=24, state_packed=8,
                   metric="env steps/sec, grid Ant-Tag 10x10 (build-defined), 2M envs per GPU (16M on 8 GPUs)",
                   dtype="int32", kernel="anttag_rollout<false>",
                   desc="configs[3]: grid Ant-Tag 10x10, {B} envs per GPU (2M x 8 GPUs = 16M), AntTagGridEnv()"),
}


def lib_hash():
    p = os.path.join(ROOT, "gym-po-taxi_amd", "gym_po_amd", "libgympo_amd.so")
    with open(p, "rb") as f:
        return hashlib.sha1(f.read()).hexdigest()[:12]


# sources that determine each measured kernel's code (PMC traffic is reused only for the same sources)
KERNEL_SOURCES = {"fourrooms": ("wgrid.hip", "grid.hip", "grid_shared.h", "gp_common.h", "gp_internal.h"),
                  "taxi": ("taxi.hip", "gp_common.h", "gp_internal.h", "gp_libm.h"),
                  "crooms": ("crooms.hip", "gp_common.h", "gp_internal.h", "ziggurat_tables.h", "gp_libm.h"),
                  "anttag": ("anttag.hip", "gp_common.h", "gp_internal.h")}


def src_hash(workload):
    h = hashlib.sha1()
    for name in KERNEL_SOURCES[workload]:
        p = os.path.join(ROOT, "gym-po-taxi_amd", "csrc", name)
        with open(p, "rb") as f:  # a missing file is a stale KERNEL_SOURCES entry: fail, never hash less
            h.update(f.read())
    return h.hexdigest()[:12]


def measured_hbm_peaks(dev, nbytes=1 << 31, reps=10):
    """Measured HBM ceilings on this GPU (reported beside the spec peak): a device-to-device
    copy (read + write bytes counted) and a write-only fill, 2 GiB buffers, HIP events, best of `reps`."""
    import torch
    a = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    b = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    a.fill_(1)
    out = {}
    for name, fn, moved in (("copy", lambda: b.copy_(a), 2 * nbytes), ("fill", lambda: b.fill_(7), nbytes)):
        fn()
        best = float("inf")
        for _ in range(reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            fn()
            e1.record()
            e1.synchronize()
            best = min(best, e0.elapsed_time(e1) * 1e-3)
        out[name] = moved / best / 1e9
    del a, b
    torch.cuda.empty_cache()
    return out


def cpu_model():
    """`lscpu` model name of this host (reported with the CPU baseline)."""
    try:
        import subprocess
        out = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=10).stdout
        for line in out.splitlines():
            if line.startswith("Model name:"):
                return line.split(":", 1)[1].strip()
    except Exception:  # noqa: BLE001
        pass
    return None


def effective_cpus():
    """CPUs this process can really use: the scheduler affinity mask, capped by the cgroup CPU quota
    (cgroup v2 `cpu.max` "quota period", v1 `cpu.cfs_quota_us` / `cpu.cfs_period_us`). Returns (effective,
    os.cpu_count(), affinity, quota or None). A container that sees 256 CPUs may hold a quota of a few."""
    count = os.cpu_count() or 1
    try:
        aff = len(os.sched_getaffinity(0))
    except Exception:  # noqa: BLE001
        aff = count
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = int(q) / int(per)
    except Exception:  # noqa: BLE001
        try:
            q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
            per = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
            if q > 0:
                quota = q / per
        except Exception:  # noqa: BLE001
            pass
    eff = aff if quota is None else max(1, min(aff, int(quota)))
    return eff, count, aff, quota


def cpu_baseline(workload="fourrooms", target_s=12.0, procs=None):
    """The numpy oracle (the reference's algorithm restated, fixture-pinned) on the host: one process on one
    core, then P independent processes, each on its own 2^16-env batch, P = the CPUs this
    process may really use (affinity and cgroup quota: effective_cpus; os.cpu_count() is reported beside it).
    The aggregate is every process's env-steps over the wall span from the first process's start to the last
    one's end (so processes that time-share fewer cores than P are not over-counted)."""
    one = _cpu_baseline_1(workload, target_s)
    eff, count, usable, quota = effective_cpus()
    procs = procs or eff
    if procs <= 1:
        one.update(cpu_count=count, cpus_usable=usable, cgroup_quota_cpus=quota)
        return one
    import multiprocessing as mp
    ctx = mp.get_context("spawn")  # fresh interpreters (numpy only): never fork a process that holds the GPU

    def pool_run(P):
        t0 = time.perf_counter()
        with ctx.Pool(P) as pool:
            res = pool.starmap(_cpu_baseline_1, [(workload, target_s, 1 << 16)] * P)
        wall = time.perf_counter() - t0
        span = max(r["t_end"] for r in res) - min(r["t_start"] for r in res)
        agg = sum(r["env_steps"] for r in res) / span
        per_proc = [r["env_steps"] / max(r["t_end"] - r["t_start"], 1e-9) for r in res]
        return res, wall, span, agg, per_proc

    res, wall, span, agg, per_proc = pool_run(procs)
    oversub = None
    per1 = one["value"]  # one process alone (2^18 envs)
    if sorted(per_proc)[len(per_proc) // 2] < 0.5 * per1 and procs > 1:
        # the P processes time-shared fewer cores than P (a quota the files above do not show): measure again
        # with as many processes as cores were actually available, so that `cores` states what ran
        oversub = procs
        procs = max(1, min(procs, int(round(agg / per1))))
        res, wall, span, agg, per_proc = pool_run(procs)
    return {"value": agg, "unit": "env-steps/s", "cores": procs, "kind": "port",
            "cpu_model": cpu_model(), "cpu_count": count, "cpus_usable": usable, "cgroup_quota_cpus": quota,
            "per_process_median": float(sorted(per_proc)[len(per_proc) // 2]),
            "oversubscribed_first_try": oversub,
            "sample": f"P = {procs} processes (effective CPUs: affinity {usable}, cgroup quota {quota}, "
                      f"os.cpu_count() {count}) x "
                      f"({res[0]['sample']}); aggregate = total env-steps / {span:.1f} s span ({wall:.1f} s pool "
                      f"wall); 1 process on 2^18 envs: {one['value']:.4g} env-steps/s. The oracle is the "
                      f"reference's numpy step restated (fixture-pinned); per core it runs ~1.5x faster than the "
                      f"reference itself (SURVEY.md §6: 5.0M vs 3.18M env-steps/s on one core)",
            "value_1core": one["value"]}


def _cpu_baseline_1(workload="fourrooms", target_s=12.0, B=1 << 18):
    """One process of the CPU baseline (see cpu_baseline)."""
    import numpy as np
    if workload == "crooms":
        from oracle.crooms import CRoomsOracle
        ora = CRoomsOracle(B, obs_type="vector_mdp")
        name = "oracle.crooms.CRoomsOracle(vector_mdp, float64)"
        acts = np.random.default_rng(1).uniform(-1, 1, (8, B, 2))
        return _time_oracle(ora, acts, name, B, target_s)
    if workload == "anttag":
        from oracle.anttag import AntTagOracle
        from oracle.philox import philox_key
        ora = AntTagOracle(B)
        key = philox_key(0)
        ora.reset(ora.philox_draws(0, key))
        ctr = [0]

        def step(a):
            ctr[0] += 1
            return ora.step(a, ora.philox_draws(ctr[0], key))
        ora.step_seeded = step
        ora.reset_seed = lambda seed: None
        acts = np.random.default_rng(1).integers(0, 5, (8, B))
        return _time_oracle(ora, acts, "oracle.anttag.AntTagOracle (numpy, philox draws; build-defined spec, "
                                       "no reference to pin)", B, target_s)
    if workload == "taxi":
        from oracle.taxi import TaxiOracle
        ora = TaxiOracle(B, hansen_obs=True)
        name, na = "oracle.taxi.TaxiOracle(hansen_obs=True) + one-hot np.eye gather", 5
        eye = np.eye(ora.no, dtype=np.uint8)
        step = ora.step_seeded
        ora.step_seeded = lambda a: (lambda r: (eye[r[0]],) + tuple(r[1:]))(step(a))
    else:
        from oracle.gridworld import FourRoomsOracle
        ora = FourRoomsOracle(B, 1, obs_type="hansen")
        name, na = "oracle.gridworld.FourRoomsOracle", 4
    acts = np.random.default_rng(1).integers(0, na, (8, B))
    return _time_oracle(ora, acts, name, B, target_s)


def _time_oracle(ora, acts, name, B, target_s):
    ora.reset_seed(0)
    ora.step_seeded(acts[0])  # warm
    t_start = time.time()
    t0 = time.perf_counter()
    n = 0
    while True:
        ora.step_seeded(acts[n % 8])
        n += 1
        dt = time.perf_counter() - t0
        if dt >= target_s or n >= 400:
            break
    return {"value": B * n / dt, "unit": "env-steps/s", "cores": 1, "kind": "port",
            "env_steps": B * n, "t_start": t_start, "t_end": time.time(),
            "sample": f"{name} (numpy{'' if 'build-defined' in name else ', reference-pinned'}), "
                      f"2^{B.bit_length() - 1} envs x {n} steps, 1 process ({dt:.1f} s)"}


def load_pmc(cfg_key, workload, steps_per_launch, kernel=None):
    """HBM traffic per launch of `steps_per_launch` steps from profiles/*pmc_*.json (rocprofv3 FETCH_SIZE /
    WRITE_SIZE passes, tools/pmc_to_json.py), only from records of the same kernel sources and config.
    A record at exactly this launch shape is used as is; otherwise, from records at two or more launch
    shapes, the per-launch traffic T(K) = fixed + per_step * K is fitted (least squares) and evaluated at K.
    Returns (bytes, source text) or (None, None)."""
    import glob
    recs = {}
    for fn in sorted(glob.glob(os.path.join(ROOT, "profiles", "*pmc_*.json"))):
        try:
            d = json.load(open(fn))
        except Exception:  # noqa: BLE001
            continue
        if kernel and d.get("kernel") and d["kernel"] not in kernel:
            continue  # another kernel's record (numpy FourRooms has two for the same launch shape)
        if d.get("src_hash") == src_hash(workload) and d.get("config") == cfg_key and d.get("steps_per_launch"):
            recs[float(d["steps_per_launch"])] = (d["hbm_bytes_per_launch"], os.path.basename(fn))
    if not recs:
        return None, None
    for k, (v, fn) in recs.items():
        if abs(k - steps_per_launch) < 1e-9:
            return v, f"{fn} (PMC pass at {k:g} steps per launch)"
    if len(recs) < 2:
        return None, None
    import numpy as np
    ks = np.array(sorted(recs))
    ts = np.array([recs[k][0] for k in ks])
    per_step, fixed = np.polyfit(ks, ts, 1)
    return float(fixed + per_step * steps_per_launch), (
        f"fit T(K) = {fixed:.4g} + {per_step:.4g}*K bytes over PMC passes at K = {[float(k) for k in ks]}")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=2000)
    ap.add_argument("--warmup", type=int, default=200)
    ap.add_argument("--workload", default="fourrooms", choices=sorted(WORKLOADS),
                    help="fourrooms = the BASELINE headline (default); others = the other single-GPU configs")
    ap.add_argument("--envs", type=int, default=None, help="envs per GPU (weak scaling)")
    ap.add_argument("--strong", action="store_true", help="split --envs across GPUs instead")
    ap.add_argument("--mode", default=None, choices=["numpy", "philox"])
    ap.add_argument("--chunk", type=int, default=None, help="steps per gp_rollout call")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--kernel", default="auto", choices=["auto", "windowed", "fused"],
                    help="numpy FourRooms: gp_autotune's choice (default) or one kernel for every launch")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    # the CPU baseline first, before this process touches the GPU (its worker processes are spawned)
    cpu = None if (args.no_cpu_baseline or world > 1) else cpu_baseline(args.workload)

    import torch
    import torch.distributed as dist

    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        # one rank per GPU; GP_BENCH_BACKEND=gloo rehearses N ranks on fewer GPUs (ranks share devices)
        backend = os.environ.get("GP_BENCH_BACKEND", "nccl")
        dev = torch.device("cuda", local % max(torch.cuda.device_count(), 1))
        torch.cuda.set_device(dev)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)
    else:
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)

    W = WORKLOADS[args.workload]
    args.envs = args.envs or W["envs"]
    args.mode = args.mode or W["mode"]
    args.chunk = args.chunk or W.get("chunk", 64)
    from gym_po_amd import shard
    B = shard.shard_size(args.envs, world, rank, args.strong)
    C = max(1, min(args.chunk, args.steps))
    from gym_po_amd._lib import debug_knobs
    # GP_KNOBS="key=value,...": diagnostic library knobs for in-call A/Bs (never set by the driver's command)
    knobs = dict((kv.split("=")[0], int(kv.split("=")[1])) for kv in os.environ.get("GP_KNOBS", "").split(",") if kv)
    if args.kernel != "auto":  # numpy-mode FourRooms kernel forced for every launch length (PMC records per kernel)
        knobs["wg_kmax"] = 1 << 20 if args.kernel == "windowed" else 0
    with debug_knobs(**knobs):
        env = W["make"](B, dev, args.mode)
    persist = None
    if args.workload != "fourrooms":  # the streaming rollouts' persistent grid (persistent_grid, csrc/gp_internal.h)
        persist = {"blocks": env.query("persist_blocks"), "resident_per_cu": env.query("persist_occupancy")}
    shard.seed_shard(env, 0, rank, world)  # shard g: SeedSequence(0, spawn_key=(g,))
    env.reset()
    # numpy-mode FourRooms: the faster of the two bit-identical kernels for C-step launches on this board, timed
    # on scratch state by the library before anything is timed here (gp_autotune; -1 elsewhere: a no-op)
    # (20 launches per kernel: with 5 the choice flipped in 1 of 5 driver-command runs on one box, to the slower one;
    # the library keeps the launch length's default kernel unless the other is >= 2% faster)
    tuned = env.autotune(C, reps=20) if args.kernel == "auto" and hasattr(env, "autotune") else -1
    pretimed = None
    if tuned >= 0:  # GPU work before the warmup, on scratch state (the env's state is restored exactly)
        na, ka = env.query("autotune_launches"), env.query("autotune_steps")
        pretimed = {"autotune_launches": na, "autotune_steps_per_launch": ka, "autotune_env_steps": na * ka * B,
                    "autotune_us_per_launch": {"windowed": env.query("autotune_wgrid_ns") / 1e3,
                                               "fused": env.query("autotune_fused_ns") / 1e3},
                    "note": "both kernels timed on scratch actions/outputs before the warmup; the default kernel for "
                            "the launch length is kept unless the other is >= 2% faster"}
    g = torch.Generator(device=dev)
    g.manual_seed(1 + rank)
    if W["n_actions"] is None:  # continuous (y, x) actions, float32 U[-1, 1]^2
        acts = torch.rand((C, B, 2), device=dev, dtype=torch.float32, generator=g) * 2 - 1
    else:
        acts = torch.randint(0, W["n_actions"], (C, B), device=dev, dtype=torch.int32, generator=g)
    out = env._alloc_outputs(C)
    for o in out:  # first touch at allocation, not inside the timed region
        o.zero_()
    # prepared launches (validated once, no per-call Python work beyond the C call): full chunks of C steps
    # and, lazily, the one shorter chunk size a step count not divisible by C needs
    plans = {C: env.rollout_plan(acts, out)[0]}

    def run(n):
        done = 0
        while done < n:
            k = min(C, n - done)
            if k not in plans:
                plans[k] = env.rollout_plan(acts[:k], tuple(o[:k] for o in out))[0]
            plans[k]()
            done += k

    def barrier():
        if world > 1:
            dist.barrier()

    def warm(runner, n):
        # The W warmup steps, issued as two launches (1 step, then W - 1) when W >= 2: a process's second launch
        # of the kernel carries a one-time runtime cost (≈15 µs host-side; tools/first_call_probe.py), which
        # belongs in the warmup rather than in the first timed call. Same steps, same stream position.
        if n >= 2:
            runner(1)
            runner(n - 1)
        else:
            runner(n)

    warm(run, args.warmup)
    torch.cuda.synchronize(dev)
    barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    run(args.steps)
    torch.cuda.synchronize(dev)
    if world > 1:  # (one rank: the barrier is a no-op and a second synchronize would only time an idle device)
        barrier()
        torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    tmax = shard.max_over_ranks(elapsed, dev)

    # live roofline: HIP events bracketing every step-kernel launch on its stream
    env.set_profiling(True)
    # whole launches of the timed region's shape (C steps each), so steps_per_launch is exactly C; at least 10
    # launches (a 3-launch average of 20-step launches moved by ±4% between runs of one build)
    prof_steps = C * max(10, min(2000 // C, max(args.steps // (2 * C), 1)))
    run(prof_steps)
    kms, nk = env.profile_read()
    rms, nr = env.profile_read_resolver()
    env.set_profiling(False)
    kavg_ms = kms / max(nk, 1)
    ravg_ms = rms / max(nr, 1)
    steps_per_launch = prof_steps / max(nk, 1)
    if args.workload != "fourrooms" or steps_per_launch > 1.5:
        # fused launch of several steps; state read+written once per launch
        bytes_per_launch = B * (W["bytes"] * steps_per_launch + W["state"])
        bytes_packed = B * (W["bytes"] * steps_per_launch + W["state_packed"])
    else:
        bytes_per_launch = bytes_packed = B * BYTES_PER_ENV_STEP
    achieved = bytes_per_launch / (kavg_ms * 1e-3) / 1e9
    achieved_packed = bytes_packed / (kavg_ms * 1e-3) / 1e9

    m = shard.allreduce_metrics(env.metrics(), dev)  # RCCL: the only collective (episode statistics)

    # SURVEY.md §8(d)'s primary curve is STRONG scaling (1M envs split over the N GPUs); `value` is the
    # contract's weak-scaling number (1M envs per GPU). With N > 1 each rank also times its strong-scaling
    # shard (2^20 / N envs, same kernel path, same warmup / step counts) and the line carries it.
    strong = None
    if world > 1 and not args.strong and args.workload == "fourrooms":
        Bs = shard.shard_size(args.envs, world, rank, True)
        env_s = W["make"](Bs, dev, args.mode)
        shard.seed_shard(env_s, 0, rank, world)
        env_s.reset()
        Cs = max(1, min(args.chunk, args.steps))
        acts_s = torch.randint(0, W["n_actions"], (Cs, Bs), device=dev, dtype=torch.int32, generator=g)
        out_s = env_s._alloc_outputs(Cs)
        for o in out_s:
            o.zero_()
        plan_s = env_s.rollout_plan(acts_s, out_s)[0]
        plans_s = {Cs: plan_s}

        def run_s(n):
            done = 0
            while done < n:
                k = min(Cs, n - done)
                if k not in plans_s:
                    plans_s[k] = env_s.rollout_plan(acts_s[:k], tuple(o[:k] for o in out_s))[0]
                plans_s[k]()
                done += k
        warm(run_s, args.warmup)
        torch.cuda.synchronize(dev)
        barrier()
        torch.cuda.synchronize(dev)
        t0s = time.perf_counter()
        run_s(args.steps)
        torch.cuda.synchronize(dev)
        barrier()
        torch.cuda.synchronize(dev)
        ts = shard.max_over_ranks(time.perf_counter() - t0s, dev)
        env_s.metrics()  # raises on a device-side failure
        env_s.close()
        strong = {"global_envs": args.envs, "envs_per_gpu": Bs, "value": args.envs * args.steps / ts,
                  "ms_per_step": ts / args.steps * 1e3, "scaling": "strong"}

    kernel_name = None
    if args.workload == "fourrooms" and args.mode == "numpy" and env.query("wgrid"):
        # launches of up to wgrid_kmax steps run the windowed kernel, longer ones the fused kernel (grid.hip)
        kernel_name = (f"wgrid_rollout<{env.query('wgrid_block_envs') // 512},{W['n_actions']}>"
                       if steps_per_launch <= env.query("wgrid_kmax") else "grid_rollout_numpy<GP_OBS_HANSEN,2,4,true>")
    total_steps = (args.envs if args.strong else B * world) * args.steps
    cfg_key = (f"fourrooms_hansen4_B{B}_{args.mode}" if args.workload == "fourrooms" else
               f"{args.workload}_B{B}_{args.mode}")
    kname = W.get("kernel") or (kernel_name if kernel_name else ("grid_rollout_numpy<GP_OBS_HANSEN,2,4,true>"
                                                             if steps_per_launch > 1.5 else "grid_step_numpy<GP_OBS_HANSEN>")
                                if args.mode == "numpy" else "grid_rollout_counter<GP_OBS_HANSEN,false>")
    traffic, traffic_src = load_pmc(cfg_key, args.workload, steps_per_launch, kname)
    line = {
        "metric": W["metric"],
        "value": total_steps / tmax,
        "unit": "env-steps/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": tmax / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "strong" if args.strong else "weak",
        "vs_baseline": None,
        "dtype": W["dtype"],
        "data": "synthetic (uniform random actions, seeded); " + (
            "reference RNG stream reproduced bit-exactly" if args.mode == "numpy" else
            "counter-based Philox draws from the reference's exact laws"),
        "config": {"workload": W["desc"].format(B=B),
                   "envs_per_gpu": B, "global_envs": args.envs if args.strong else B * world, "rng_mode": args.mode,
                   "parallelism": f"independent env shards x{world}", "steps_per_launch_call": C,
                   "kernel_autotune": {1: "windowed", 0: "fused", -1: None}[tuned] if args.kernel == "auto" else
                   f"forced: {args.kernel}",
                   "pretimed": pretimed, **({"knobs": knobs} if knobs else {}),
                   **({"persistent_grid": persist} if persist else {})},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                     "byte_model": (f"SURVEY 8(d): {W['bytes']} B per env-step + {W['state']} B per env per launch "
                                    "(canonical state layout)"),
                     "frac_packed_state": achieved_packed / HBM_PEAK_GBS,
                     "bytes_per_launch_packed_state": bytes_packed,
                     "traffic_over_algorithmic": traffic / bytes_per_launch if traffic else None,
                     "traffic_source": traffic_src,
                     "kernel": kname,
                     "steps_per_launch": steps_per_launch,
                     "kernel_avg_us": kavg_ms * 1e3,
                     "bytes_per_launch": bytes_per_launch,
                     "kernel_launches_timed": nk,
                     # the two-kernel path's reset resolver (only launched when neither fused kernel runs)
                     "resolver_kernel": "grid_resolve_numpy<GP_OBS_HANSEN>" if nr else None,
                     "resolver_avg_us": ravg_ms * 1e3 if nr else None},
        "episodes": {"count": m["episodes"], "mean_return": m["return_sum"] / max(m["episodes"], 1),
                     "mean_length": m["length_sum"] / max(m["episodes"], 1)},
        "lib_hash": lib_hash(),
    }
    if strong is not None:
        line["strong"] = strong
    if rank == 0:
        if world == 1:
            pk = measured_hbm_peaks(dev)
            line["roofline"]["measured_copy_gbs"] = pk["copy"]
            line["roofline"]["measured_fill_gbs"] = pk["fill"]
            line["roofline"]["frac_of_measured_fill"] = achieved / pk["fill"]
        line["cpu_baseline"] = cpu
        print(json.dumps(line), flush=True)
    env.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
