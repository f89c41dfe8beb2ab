"""Agent-facing interop: the step outputs are torch-ROCm tensors on the env's
device, exported zero-copy over DLPack to any DLPack consumer."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_outputs_export_zero_copy_over_dlpack(gpu_device):
    import torch
    from torch.utils.dlpack import from_dlpack, to_dlpack
    from gym_po_amd import MultistoryFourRoomsEnv
    B = 4096
    env = MultistoryFourRoomsEnv(B, grid_z=1, obs_type="hansen", device=gpu_device)
    obs, _ = env.reset(seed=0)
    o, r, d, t, _ = env.step(np.zeros(B, np.int64))
    for x in (obs, o, r, d, t):
        assert x.is_cuda
        y = from_dlpack(to_dlpack(x))             # capsule round trip
        z = torch.from_dlpack(x)                  # __dlpack__ protocol
        assert y.data_ptr() == x.data_ptr() == z.data_ptr()
        assert torch.equal(y, x) and torch.equal(z, x)
