"""GPU side of the shard path: a device shard seeded through gym_po_amd.shard equals the oracle env with
the spawned seed sequence, and the on-device episode statistics (what bench.py all-reduces) equal the
ones recomputed from the oracle trajectory."""
import numpy as np
import pytest

from gym_po_amd import shard
from test_shard_gloo import B, K, run_shard

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("rank", [0, 1])
def test_device_shard_matches_oracle_shard(rank, gpu_device):
    import torch
    from gym_po_amd import MultistoryFourRoomsEnv
    b = shard.shard_size(B, 2, rank, strong=True)
    env = MultistoryFourRoomsEnv(b, grid_z=1, obs_type="hansen", time_limit=30, device=gpu_device)
    shard.seed_shard(env, 0, rank, 2)
    env.reset()
    acts = torch.as_tensor(np.random.default_rng(1 + rank).integers(0, 4, (K, b)), dtype=torch.int32,
                           device=gpu_device)
    obs, rew, term, trunc = env.rollout(acts)
    m_want, o_want = run_shard(rank, 2)
    assert np.array_equal(obs[-1].cpu().numpy(), o_want.astype(np.int32))
    m = env.metrics()
    for k in shard.METRIC_KEYS:
        assert m[k] == m_want[k], k
    assert shard.allreduce_metrics(m, gpu_device) == m  # no process group: identity
