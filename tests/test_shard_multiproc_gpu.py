"""The device shard path with two processes (VERDICT r2 "missing" #4): two ranks in a world-size-2 `gloo` group, each
stepping ITS FourRooms shard through the HIP kernels on cuda:0 (gym_po_amd.shard: the plan, the spawned seeding and
the two end-of-run collectives bench.py runs), then the all-reduced episode statistics against the serial oracle run
of both shards (tests/test_shard_gloo.run_shard) and each rank's last observations against its oracle shard.

The workers are spawned (fresh interpreters); the parent must not have initialised the GPU before it spawns them, so
conftest.py runs this module first and the test refuses to run in a process where torch already initialised HIP.
"""
import os

import numpy as np
import pytest

from gym_po_amd import shard
from test_shard_gloo import B, K, T, _free_port, run_shard

pytestmark = [pytest.mark.gpu, pytest.mark.gpu_first]


def _worker(rank, world, port, out):
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from gym_po_amd import MultistoryFourRoomsEnv
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        b = shard.shard_size(B, world, rank, strong=True)
        env = MultistoryFourRoomsEnv(b, grid_z=1, obs_type="hansen", time_limit=T, device=dev)
        shard.seed_shard(env, 0, rank, world)
        env.reset()
        acts = torch.as_tensor(np.random.default_rng(1 + rank).integers(0, 4, (K, b)), dtype=torch.int32, device=dev)
        obs = env.rollout(acts)[0]
        torch.cuda.synchronize(dev)
        tot = shard.allreduce_metrics(env.metrics())  # gloo on CPU tensors: the same code path as bench.py
        np.save(f"{out}.obs{rank}.npy", obs[-1].cpu().numpy())
        if rank == 0:
            np.save(out, np.array([tot[k] for k in shard.METRIC_KEYS]))
        env.close()
    finally:
        dist.destroy_process_group()


# Passed on the MI355X pool (profiles/r03_gpu_test_multiproc_shards.txt); GP_MULTIPROC_TEST=0 skips it.
@pytest.mark.skipif(os.environ.get("GP_MULTIPROC_TEST") == "0", reason="disabled: GP_MULTIPROC_TEST=0")
@pytest.mark.timeout(300)
def test_two_processes_device_shards_gloo(tmp_path):
    import torch
    from gym_po_amd import _lib
    # torch's own flag, and whether this process has loaded the native library (whose first handle initialises HIP
    # outside torch): either means the GPU may be initialised here, and spawning from it is not allowed
    if torch.cuda.is_initialized() or _lib._lib is not None:
        pytest.skip("this process may already have initialised the GPU: spawning from it is not allowed here")
    import torch.multiprocessing as mp
    out = str(tmp_path / "m.npy")
    mp.spawn(_worker, args=(2, _free_port(), out), nprocs=2, join=True)
    got = np.load(out)
    serial = [run_shard(r, 2) for r in range(2)]
    want = [sum(s[0][k] for s in serial) for k in shard.METRIC_KEYS]
    assert np.allclose(got, want, rtol=0, atol=1e-6), (got, want)
    for r in range(2):
        np.testing.assert_array_equal(np.load(f"{out}.obs{r}.npy").astype(np.int64),
                                      np.asarray(serial[r][1]).astype(np.int64), err_msg=f"rank {r}")
