"""Independent env shards across the GPUs of one node.

Every env of a gym_po vector env is independent of every other, so the batch partitions with no
data-path exchange: rank g owns its own shard of envs, seeded `SeedSequence(seed, spawn_key=(g,))`
(= `SeedSequence(seed).spawn(G)[g]`), i.e. shard g IS the reference env
`MultistoryFourRoomsEnv(num_envs=B_g)` reset with that seed sequence (msrooms.py:369-388 seeding via
gymnasium `seeding.np_random`). A single numpy stream spanning GPUs would need a per-step cross-GPU
scan of reset counts; it is deliberately not offered.

The only collectives are at the end of a run: MAX of the timed region and SUM of the on-device episode
statistics (32 B per rank) — RCCL (`nccl` backend) on the GPU box, `gloo` in the CPU tests.
"""
import numpy as np

METRIC_KEYS = ("episodes", "return_sum", "length_sum", "env_steps")


def shard_size(num_envs, world, rank=0, strong=False):
    """Envs owned by `rank`: all `num_envs` (weak scaling) or a contiguous split of them (strong)."""
    if not strong:
        return int(num_envs)
    base, extra = divmod(int(num_envs), int(world))
    return base + (1 if rank < extra else 0)


def shard_offset(num_envs, world, rank, strong=False):
    """Global index of the shard's first env (strong split: envs [offset, offset + size))."""
    if not strong:
        return int(rank) * int(num_envs)
    return sum(shard_size(num_envs, world, r, True) for r in range(rank))


def shard_seed_sequence(seed, rank):
    """The numpy SeedSequence shard `rank` is seeded with."""
    return np.random.SeedSequence(seed, spawn_key=(int(rank),))


def seed_shard(env, seed, rank, world):
    """Seed `env` (a gym_po_amd vector env) as shard `rank` of `world`. With world == 1 this is plain
    `reset(seed=seed)` seeding (no spawn key), so a 1-GPU run equals the reference env exactly."""
    if world == 1:
        env.seed(seed)
    else:
        env.seed(seed, spawn_key=(int(rank),))


def _dist():
    import torch.distributed as dist
    return dist if dist.is_available() and dist.is_initialized() else None


def max_over_ranks(value, device="cpu"):
    """MAX of a float over all ranks (identity without a process group)."""
    import torch
    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    d = _dist()
    if d is not None and d.get_world_size() > 1:
        d.all_reduce(t, op=d.ReduceOp.MAX)
    return float(t.item())


def allreduce_metrics(metrics, device="cpu"):
    """SUM of the episode statistics dict (`NativeVecEnv.metrics()`) over all ranks."""
    import torch
    t = torch.tensor([float(metrics[k]) for k in METRIC_KEYS], dtype=torch.float64, device=device)
    d = _dist()
    if d is not None and d.get_world_size() > 1:
        d.all_reduce(t)
    return {k: float(v) for k, v in zip(METRIC_KEYS, t.tolist())}
