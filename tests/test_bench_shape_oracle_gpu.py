"""The bench's own workload stepped beside the oracle.

bench.py times config 3 -- one handle of 4096 envs x 8 agents x 64 beams, team
reward, respawn on, max_steps 2000, per-env auto-reset (MEV_AUTO_RESET), the
fused k_step with its XCD-aware block -> env order -- with device-resident
actions.  Here the same handle runs 200 steps and 16 of its envs, spread over
the whole batch, are stepped beside the C restatement (oracle/marl_oracle.c,
pinned to the reference's goldens), bit for bit on every output and on the full
state.  The envs' step counters are staggered close to max_steps so that
truncations and the auto-resets after them (reference env.py:147-161 reset()
then step()) fall inside the window, as they do in a long bench run."""
import numpy as np
import pytest

import oracle_replay as R

pytestmark = pytest.mark.gpu

E, N, RAYS, T, MAXS = 4096, 8, 64, 200, 2000
META = dict(rays=RAYS, obs_dim=31 + RAYS, num_lanes=3, n_agents=N, use_team=True, respawn=True, max_steps=MAXS, traffic=False,
            density=0.5, reward=[10.0, 1.0, -0.01, -10.0, -5.0, 10.0, -0.02, 0.2])


@pytest.mark.parametrize("split", [0, 3])
def test_bench_workload_sampled_envs_match_oracle(mev, split):
    """split 0: the bench's automatic choice (one wave per env); 3: the early split
    (a car wave and a LiDAR wave per env, the LiDAR's road march started after the
    kinematics, respawned egos re-marched)."""
    import torch

    h = mev.Handle(num_envs=E, num_agents=N, lidar_rays=RAYS, use_team_reward=1, respawn_enabled=1,
                   max_steps=MAXS, seed=0, device=0)
    h.set_step_split(split)
    assert h.step_kernel() == 2, "the bench size runs the fused k_step"
    assert h.step_split() == (2 if split == 3 else 0)
    torch.cuda.set_device(0)
    stream = torch.cuda.current_stream(0)
    h.set_stream(stream.cuda_stream)
    h.reset()
    rng = np.random.default_rng(11)
    # a first stretch of steps moves the envs off their spawn points (every env differs after it)
    warm = torch.Generator(device="cuda:0").manual_seed(5)
    for _ in range(40):
        h.step(torch.rand((E, N, 2), device="cuda:0", generator=warm) * 2 - 1, auto_reset=True, device=True)
    st = h.get_state()
    # staggered step counters: envs truncate (then auto-reset) at different steps of the window
    st["step_count"][:] = MAXS - rng.integers(1, T, E)
    h.set_state(st)
    st = h.get_state()
    sample = np.sort(rng.choice(E, 16, replace=False))
    sample[0], sample[-1] = 0, E - 1  # both ends of the batch (first and last workgroups)
    oracles = {int(e): R.oracle_from_device_state(META, st, int(e)) for e in sample}
    obs0 = h.observations()
    for e, o in oracles.items():
        assert np.array_equal(obs0[e].view(np.uint32), o.observe().view(np.uint32)), f"env {e}: obs after set_state"
    out = {k: torch.zeros_like(torch.as_tensor(v), device="cuda:0") for k, v in h.alloc_outputs().items()}
    idx = torch.as_tensor(sample, device="cuda:0")
    ended = {e: False for e in oracles}
    resets = 0
    for t in range(T):
        a = rng.uniform(-1, 1, (E, N, 2)).astype(np.float32)
        h.step(torch.from_numpy(a).to("cuda:0"), auto_reset=True, out=out, device=True)
        got = {k: v.index_select(0, idx).cpu().numpy() for k, v in out.items()}
        st_t = h.get_state() if t % 20 == 19 or t == T - 1 else None
        for j, (e, o) in enumerate(oracles.items()):
            if ended[e]:  # the device auto-reset this env before stepping it: reset() then step()
                o.reset([int(r) for r in st["route"][e]])
                resets += 1
            r = o.step(a[e])
            R.check_step(f"env {e} step {t + 1}", got, j, r)
            ended[e] = bool(r["terminated"] or r["truncated"])
            if st_t is not None:
                R.check_state(f"env {e} step {t + 1}", st_t, e, o)
    assert resets >= len(oracles) // 2, f"only {resets} auto-resets in the window"
    h.close()


def test_config2_full_size_sampled_envs_match_oracle(mev):
    """BASELINE config 2 at its full size: 4096 envs x 1 agent x 64 beams on the automatic early split
    (four envs per workgroup: a car wave and a LiDAR wave marching their four egos' beams from the
    poses after the kinematics), auto-reset, 300 steps; 16 sampled envs stepped beside the oracle,
    every output every step and the state every 20 steps, with truncations and auto-resets in the window."""
    import torch

    E2, T2 = 4096, 300
    meta = dict(META, n_agents=1, use_team=False)
    h = mev.Handle(num_envs=E2, num_agents=1, lidar_rays=RAYS, respawn_enabled=1, max_steps=MAXS, seed=0, device=0)
    assert h.step_kernel() == 2 and h.step_split() == 2 and h.step_pack() == 4, "config 2 runs the early split"
    torch.cuda.set_device(0)
    h.set_stream(torch.cuda.current_stream(0).cuda_stream)
    h.reset()
    rng = np.random.default_rng(17)
    warm = torch.Generator(device="cuda:0").manual_seed(6)
    for _ in range(40):
        h.step(torch.rand((E2, 1, 2), device="cuda:0", generator=warm) * 2 - 1, auto_reset=True, device=True)
    st = h.get_state()
    st["step_count"][:] = MAXS - rng.integers(1, T2, E2)
    h.set_state(st)
    st = h.get_state()
    sample = np.sort(rng.choice(E2, 16, replace=False))
    sample[0], sample[-1] = 0, E2 - 1
    oracles = {int(e): R.oracle_from_device_state(meta, st, int(e)) for e in sample}
    obs0 = h.observations()
    for e, o in oracles.items():
        assert np.array_equal(obs0[e].view(np.uint32), o.observe().view(np.uint32)), f"env {e}: obs after set_state"
    out = {k: torch.zeros_like(torch.as_tensor(v), device="cuda:0") for k, v in h.alloc_outputs().items()}
    idx = torch.as_tensor(sample, device="cuda:0")
    ended = {e: False for e in oracles}
    resets = 0
    for t in range(T2):
        a = rng.uniform(-1, 1, (E2, 1, 2)).astype(np.float32)
        h.step(torch.from_numpy(a).to("cuda:0"), auto_reset=True, out=out, device=True)
        got = {k: v.index_select(0, idx).cpu().numpy() for k, v in out.items()}
        st_t = h.get_state() if t % 20 == 19 or t == T2 - 1 else None
        for j, (e, o) in enumerate(oracles.items()):
            if ended[e]:
                o.reset([int(r) for r in st["route"][e]])
                resets += 1
            r = o.step(a[e])
            R.check_step(f"env {e} step {t + 1}", got, j, r)
            ended[e] = bool(r["terminated"] or r["truncated"])
            if st_t is not None:
                R.check_state(f"env {e} step {t + 1}", st_t, e, o)
    assert resets >= len(oracles) // 2, f"only {resets} auto-resets in the window"
    h.close()

