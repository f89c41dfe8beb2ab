"""Multi-rank path of bench.py on CPU: world_size-2 `gloo` process group, independent env shards
(SURVEY.md §8(e)). Each rank steps ITS shard with the numpy oracle (the GPU box runs the HIP path;
the shard plan, the seeding and the two end-of-run collectives are the same code, gym_po_amd.shard),
and the reduced metrics must equal the serial run of both shards.
"""
import os
import socket

import numpy as np
import pytest

from gym_po_amd import shard
from oracle.draws import NumpyDraws
from oracle.gridworld import FourRoomsOracle

B, K, T = 96, 120, 30


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def run_shard(rank, world, seed=0):
    """One shard of the bench workload on the oracle: (episode statistics, last obs)."""
    b = shard.shard_size(B, world, rank, strong=True)
    ora = FourRoomsOracle(b, grid_z=1, obs_type="hansen", time_limit=T)
    ss = shard.shard_seed_sequence(seed, rank) if world > 1 else np.random.SeedSequence(seed)
    ora.gen = np.random.Generator(np.random.PCG64(ss))
    ora.reset(NumpyDraws(ora.gen))
    acts = np.random.default_rng(1 + rank).integers(0, 4, (K, b))
    m = dict(episodes=0.0, return_sum=0.0, length_sum=0.0, env_steps=0.0)
    for k in range(K):
        el = ora.elapsed.copy() + 1
        o, r, d, tr = ora.step_seeded(acts[k])
        done = d | tr
        m["episodes"] += float(done.sum())
        m["return_sum"] += float(r.astype(np.float64).sum())
        m["length_sum"] += float(el[done].sum())
        m["env_steps"] += float(b)
    return m, o


def _worker(rank, world, port, out):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        m, _ = run_shard(rank, world)
        t = shard.max_over_ranks(1.0 + rank)
        tot = shard.allreduce_metrics(m)
        if rank == 0:
            np.save(out, np.array([t] + [tot[k] for k in shard.METRIC_KEYS]))
    finally:
        dist.destroy_process_group()


def test_shard_plan():
    assert [shard.shard_size(10, 3, r, strong=True) for r in range(3)] == [4, 3, 3]
    assert [shard.shard_offset(10, 3, r, strong=True) for r in range(3)] == [0, 4, 7]
    assert shard.shard_size(1 << 20, 8, 5) == 1 << 20 and shard.shard_offset(1 << 20, 8, 5) == 5 << 20
    # shard g's seed sequence is SeedSequence(seed).spawn(G)[g] (the reference's own spawning scheme)
    kids = np.random.SeedSequence(7).spawn(4)
    for g in range(4):
        assert np.array_equal(shard.shard_seed_sequence(7, g).generate_state(4), kids[g].generate_state(4))


def test_shards_are_independent_reference_envs():
    """Shard g equals the reference env of B/G envs seeded with its own spawned sequence, whatever the
    other shards do (no cross-shard stream)."""
    m0, o0 = run_shard(0, 2)
    ora = FourRoomsOracle(B // 2, grid_z=1, obs_type="hansen", time_limit=T)
    ora.gen = np.random.Generator(np.random.PCG64(np.random.SeedSequence(0).spawn(2)[0]))
    ora.reset(NumpyDraws(ora.gen))
    acts = np.random.default_rng(1).integers(0, 4, (K, B // 2))
    for k in range(K):
        o = ora.step_seeded(acts[k])[0]
    assert np.array_equal(o, o0)


@pytest.mark.timeout(240)
def test_gloo_world2_metrics_reduce(tmp_path):
    import torch.multiprocessing as mp
    out = str(tmp_path / "m.npy")
    mp.spawn(_worker, args=(2, _free_port(), out), nprocs=2, join=True)
    got = np.load(out)
    assert got[0] == 2.0  # MAX over ranks of the timed region
    serial = [run_shard(r, 2)[0] for r in range(2)]
    want = [sum(s[k] for s in serial) for k in shard.METRIC_KEYS]
    assert np.allclose(got[1:], want, rtol=0, atol=1e-9)
    assert got[4] == B * K and got[1] > 0
