"""BASELINE config 4 at its full size beside the oracle.

One handle of 4096 envs x 1 ego x 64 beams with traffic at density 0.5 -- the shape
tools/bench_sweep.py times -- on the automatic traffic early split with the NPC-aware
deal, per-env auto-reset and the device's own Philox spawns.  Each step's spawn draw
of an env is recomputed on the host from the same counter (the kernel's Philox
restated in Python: philox() below, mev_kernels.hip npc_phase) and fed to the oracle
as that env's spawn_route, so 16 sampled envs -- spread over the deal's NPC classes
and over the batch -- are stepped beside the C restatement (oracle/marl_oracle.c,
pinned to the reference's goldens): every output every step, the full ego / NPC state
every 20 steps, bit for bit.  Step counters are staggered near max_steps so that
truncations and the auto-resets after them fall inside the window."""
import ctypes

import numpy as np
import pytest

import oracle_replay as R

pytestmark = pytest.mark.gpu

N, RAYS, T, MAXS, DENSITY, SEED, DT = 1, 64, 300, 2000, 0.5, 3, 1.0 / 60.0
META = dict(rays=RAYS, obs_dim=31 + RAYS, num_lanes=3, n_agents=N, use_team=False, respawn=True, max_steps=MAXS,
            traffic=True, density=DENSITY, reward=[10.0, 1.0, -0.01, -10.0, -5.0, 10.0, -0.02, 0.2])
M32 = 0xFFFFFFFF


def philox(c0, c1, c2, seed):
    """mev_kernels.hip philox(): 10 rounds over (c0, c1, c2, 0x9e3779b9) with key seed; (r0, r1)."""
    k0, k1 = seed & M32, (seed >> 32) & M32
    x0, x1, x2, x3 = c0 & M32, c1 & M32, c2 & M32, 0x9E3779B9
    for _ in range(10):
        p0, p1 = 0xD2511F53 * x0, 0xCD9E8D57 * x2
        y0 = (p1 >> 32) ^ x1 ^ k0
        y2 = (p0 >> 32) ^ x3 ^ k1
        x1, x3, x0, x2 = p1 & M32, p0 & M32, y0, y2
        k0, k1 = (k0 + 0x9E3779B9) & M32, (k1 + 0xBB67AE85) & M32
    return x0, x1


def spawn_draw(ctr, e, prob, nroutes):
    """The traffic-route index env e's step with rng counter ctr spawns on, or -1 (npc_phase:
    u01(a0) < spawn_prob, then a1 scaled to the route count)."""
    a0, a1 = philox(ctr & M32, ctr >> 32, e, SEED)
    u = np.float32(a0 >> 8) * np.float32(2.0 ** -24)
    return int((a1 * nroutes) >> 32) if u < prob else -1


@pytest.mark.parametrize("E", [4096, 8192])
def test_config4_full_size_sampled_envs_match_oracle(mev, E):
    """E = 8192: the traffic early split over two residency rounds of workgroups (automatic
    since round 6), the deal's later workgroups starting while earlier ones have appended."""
    import torch

    libm = ctypes.CDLL("libm.so.6")
    libm.expf.restype, libm.expf.argtypes = ctypes.c_float, [ctypes.c_float]
    # mev_step: spawn_prob = 1.0f - expf(-traffic_density * dt), in f32
    prob = np.float32(np.float32(1.0) - np.float32(libm.expf(float(-np.float32(DENSITY) * np.float32(DT)))))
    h = mev.Handle(num_envs=E, num_agents=N, lidar_rays=RAYS, traffic_flow=1, traffic_density=DENSITY,
                   max_steps=MAXS, seed=SEED, device=0)
    assert h.step_kernel() == 2 and h.step_split() == 2, "config 4 runs the fused traffic early split"
    troutes = [int(r) for r in h.default_traffic_routes()]
    torch.cuda.set_device(0)
    h.set_stream(torch.cuda.current_stream(0).cuda_stream)
    h.reset()
    warm = torch.Generator(device="cuda:0").manual_seed(9)
    for _ in range(240):  # fleets build up (density 0.5: 0.8 % spawn chance per step)
        h.step(torch.rand((E, N, 2), device="cuda:0", generator=warm) * 2 - 1, auto_reset=True, device=True)
    rng = np.random.default_rng(21)
    st = h.get_state()
    st["step_count"][:] = MAXS - rng.integers(1, T, E)
    h.set_state(st)
    st = h.get_state()
    # the counter the next step takes (every mev_step takes one value; SnapHeader: magic, version, E, N,
    # K, D, R, nfields, then rng_counter as u64)
    snap = h.snapshot()
    ctr = int(np.frombuffer(snap[32:40].tobytes(), np.uint64)[0])
    assert ctr >= 241
    # 16 envs over the NPC classes (the deal's 0..6, 7+) and the batch's ends
    cnt = st["npc_count"].astype(int)
    order = np.argsort(cnt, kind="stable")
    sample = sorted(set([0, E - 1] + [int(order[int(q * (E - 1))]) for q in np.linspace(0, 1, 14)]))
    assert len(set(np.minimum(cnt[sample], 7).tolist())) >= 3, cnt[sample]
    oracles = {e: R.oracle_from_device_state(META, st, e, troutes) for e in sample}
    obs0 = h.observations()
    for e, o in oracles.items():
        assert np.array_equal(obs0[e].view(np.uint32), o.observe().view(np.uint32)), f"env {e}: obs after set_state"
    out = {k: torch.zeros_like(torch.as_tensor(v), device="cuda:0") for k, v in h.alloc_outputs().items()}
    idx = torch.as_tensor(sample, device="cuda:0")
    ended = {e: False for e in oracles}
    resets = spawns = 0
    for t in range(T):
        a = rng.uniform(-1, 1, (E, N, 2)).astype(np.float32)
        h.step(torch.from_numpy(a).to("cuda:0"), auto_reset=True, out=out, device=True)
        got = {k: v.index_select(0, idx).cpu().numpy() for k, v in out.items()}
        st_t = h.get_state() if t % 20 == 19 or t == T - 1 else None
        for j, (e, o) in enumerate(oracles.items()):
            if ended[e]:  # the device auto-reset this env before stepping it: reset() then step()
                o.reset([int(r) for r in st["route"][e]])
                resets += 1
            sp = spawn_draw(ctr, e, prob, len(troutes))
            spawns += sp >= 0
            r = o.step(a[e], DT, sp)
            R.check_step(f"env {e} step {t + 1}", got, j, r)
            ended[e] = bool(r["terminated"] or r["truncated"])
            if st_t is not None:
                R.check_state(f"env {e} step {t + 1}", st_t, e, o)
        ctr += 1
    assert resets >= len(oracles) // 2, f"only {resets} auto-resets in the window"
    assert spawns >= 10, f"only {spawns} spawn draws in the window"
    h.close()
