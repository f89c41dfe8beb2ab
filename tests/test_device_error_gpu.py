"""Device-side failures of the persistent numpy-mode kernels are reported, never silent.

The fused rollout and the reset resolver wait on other blocks' tagged granules / flags. If the grid
were not co-resident (e.g. another persistent launch holding the CUs) a wait could never finish: it
then gives up after GridCtl's spin limit, sets the device error flag, and every other wave gives up
as soon as it sees the flag, so the launch still drains. The host reports the flag as GP_E_DEVICE
(GymPoError) from check(), metrics() and rng_state; reseeding clears it.

The test forces the failure deterministically with two diagnostic knobs read at env creation
(gp_debug_set): fault_block (that block never publishes) and spin_limit (a short wait limit).
"""
import pytest

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("kernel", ["wgrid", "fused", "two_kernel"])
def test_spin_timeout_raises_instead_of_silent_results(kernel, gpu_device):
    """wgrid: the windowed rollout's granule all-gather; fused: the older fused kernel's; two_kernel: the
    reset resolver's per-block flags."""
    import torch
    from gym_po_amd import MultistoryFourRoomsEnv
    from gym_po_amd._lib import GymPoError, debug_knobs
    B = 2048 * 8
    knobs = dict(disable_fused=kernel == "two_kernel", no_wgrid=kernel != "wgrid")
    with debug_knobs(**knobs):
        env_ok = MultistoryFourRoomsEnv(B, grid_z=1, obs_type="hansen", device=gpu_device)
    with debug_knobs(**knobs, spin_limit=4000, fault_block=1):
        env = MultistoryFourRoomsEnv(B, grid_z=1, obs_type="hansen", device=gpu_device)
    assert (env.query("fused_blocks") > 0) == (kernel != "two_kernel")
    assert env.query("wgrid") == (kernel == "wgrid")
    env.reset(seed=3)
    acts = torch.randint(0, 4, (6, B), dtype=torch.int32, device=gpu_device)
    env.rollout(acts)  # asynchronous: returns; the failure is on the device
    with pytest.raises(GymPoError, match="device error"):
        env.check()
    with pytest.raises(GymPoError, match="device error"):
        env.metrics()
    with pytest.raises(GymPoError, match="device error"):
        _ = env.rng_state
    env.seed(5)  # a new stream position clears the flag
    env.check()
    # the healthy handle on the same device is unaffected
    env_ok.reset(seed=3)
    env_ok.rollout(acts)
    env_ok.check()
    assert env_ok.metrics()["env_steps"] == 6 * B
