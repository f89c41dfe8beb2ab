"""A prepared rollout (gp_plan_run) launches on its env's device, not on the caller's current one (ADVICE r3:
gp_plan_run sets the env's device like every other entry point), and every C-ABI call gives the caller its current
device back (a scoped guard, so torch allocations on plain "cuda" stay on device 0). Needs two GPUs;
skipped with one."""
import pytest

pytestmark = pytest.mark.gpu


def test_rollout_plan_on_a_non_current_device():
    import torch
    from gym_po_amd import MultistoryFourRoomsEnv
    if torch.cuda.device_count() < 2:
        pytest.skip("one GPU visible")
    torch.cuda.set_device(0)
    B, K = 4096, 12
    e1 = MultistoryFourRoomsEnv(B, grid_z=1, obs_type="hansen", device="cuda:1")
    e2 = MultistoryFourRoomsEnv(B, grid_z=1, obs_type="hansen", device="cuda:1")
    e1.reset(seed=3)
    e2.reset(seed=3)
    acts = torch.randint(0, 4, (K, B), device="cuda:1", dtype=torch.int32)
    run, (obs, rew, term, trunc) = e1.rollout_plan(acts)
    assert torch.cuda.current_device() == 0
    run()
    assert torch.cuda.current_device() == 0
    for k in range(K):
        o, r, d, t, _ = e2.step(acts[k])
        assert torch.cuda.current_device() == 0
        assert torch.equal(obs[k], o) and torch.equal(rew[k], r) and torch.equal(term[k].bool(), d.bool())
    assert e1.rng_state == e2.rng_state
    e1.metrics()
    assert torch.cuda.current_device() == 0
