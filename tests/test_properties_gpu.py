"""Full-size (BASELINE config 3: 4096 envs x 8 agents x 64 beams) properties of
the device path that do not need an oracle: determinism, env independence
(a permutation of envs permutes every output), batched == single-env,
auto-reset/truncation semantics and output invariants."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

E, N, R = 4096, 8, 64


def _handle(mev, **kw):
    cfg = dict(num_envs=E, num_agents=N, lidar_rays=R, use_team_reward=1)
    cfg.update(kw)
    return mev.Handle(**cfg)


def _warm_state(mev, steps=60, seed=0, **kw):
    """A diverse state: run random actions from reset."""
    h = _handle(mev, **kw)
    rng = np.random.default_rng(seed)
    for _ in range(steps):
        h.step(rng.uniform(-1, 1, (E, h.N, 2)).astype(np.float32))
    st = h.get_state()
    h.close()
    return st


def test_determinism_full_size(mev):
    st = _warm_state(mev)
    rng = np.random.default_rng(1)
    acts = rng.uniform(-1, 1, (10, E, N, 2)).astype(np.float32)
    outs = []
    for _ in range(2):
        h = _handle(mev)
        h.set_state(st)
        o = [h.step(a) for a in acts]
        outs.append((o, h.get_state()))
        h.close()
    for a, b in zip(outs[0][0], outs[1][0]):
        for k in a:
            assert np.array_equal(a[k], b[k]), k
    for k in outs[0][1]:
        assert np.array_equal(outs[0][1][k], outs[1][1][k]), k


@pytest.mark.parametrize("rays", [64, 128])
def test_fused_and_two_kernel_paths_agree_full_size(mev, rays):
    """The fused k_step (default at this size; at 128 beams it runs the env's
    LiDAR as two pools of 4 agents) and k_cars + k_lidar produce identical
    outputs and state, step after step, with auto-reset on."""
    st = _warm_state(mev, seed=6, lidar_rays=rays)
    rng = np.random.default_rng(7)
    acts = rng.uniform(-1, 1, (16, E, N, 2)).astype(np.float32)
    hs = []
    for kernel in (1, 2):
        h = _handle(mev, max_steps=70, lidar_rays=rays)  # some envs truncate and auto-reset inside the window
        h.set_step_kernel(kernel)
        assert h.step_kernel() == kernel
        h.set_state(st)
        hs.append(h)
    for a in acts:
        o1 = hs[0].step(a, auto_reset=True)
        o2 = hs[1].step(a, auto_reset=True)
        for k in o1:
            assert np.array_equal(o1[k], o2[k]), k
    s1, s2 = hs[0].get_state(), hs[1].get_state()
    for k in s1:
        assert np.array_equal(s1[k], s2[k]), k
    for h in hs:
        h.close()


@pytest.mark.parametrize("n,rays,pack", [(8, 64, 1), (4, 128, 1), (2, 64, 1), (1, 64, 2), (2, 64, 4), (1, 64, 8)])
def test_early_split_agrees_full_size(mev, n, rays, pack):
    """The early split (mev_set_step_split(3): a car wave and a LiDAR wave per env,
    the LiDAR's road march started right after the kinematics, respawned egos'
    beams marched again after the car part) == one wave per env == k_cars +
    k_lidar, bit for bit, step after step, with auto-reset and respawns in the
    window (4096 envs; 8 x 64 is the bench's config 3; with `pack` envs per workgroup
    the LiDAR wave serves all their agents, e.g. config 2 at 2 envs)."""
    st = _warm_state(mev, seed=8, num_agents=n, lidar_rays=rays)
    rng = np.random.default_rng(9)
    hs = []
    for kernel, split, pk in ((1, 0, 1), (2, 1, 1), (2, 3, pack)):
        h = _handle(mev, num_agents=n, lidar_rays=rays, max_steps=70)
        h.set_step_kernel(kernel)
        h.set_step_pack(pk)
        h.set_step_split(split)
        h.set_state(st)
        hs.append(h)
    assert hs[2].step_split() == 2 and hs[1].step_split() == 0
    assert hs[2].step_pack() == pack
    respawns = 0
    for t in range(120):
        a = rng.uniform(-1, 1, (E, n, 2)).astype(np.float32)
        o = [h.step(a, auto_reset=True) for h in hs]
        for k in o[0]:
            assert np.array_equal(o[0][k], o[1][k]), (t, k)
            assert np.array_equal(o[0][k], o[2][k]), (t, k)
        respawns += int(np.isin(o[2]["status"], (3, 4, 5)).sum())
    s = [h.get_state() for h in hs]
    for k in s[0]:
        assert np.array_equal(s[0][k], s[2][k]), k
    assert respawns > 100, respawns  # crashed egos respawn: the LiDAR wave's re-march ran
    for h in hs:
        h.close()


@pytest.mark.parametrize("pack", [2, 4, 8])
def test_packed_waves_agree_full_size(mev, pack):
    """Config 2 shape (4096 envs x 1 agent x 64 beams) and 4096 x 2 agents:
    2, 4 or 8 envs per fused k_step wave (8 x 2 agents: reduced to 4) == one env per wave == k_cars + k_lidar,
    bit for bit, step after step with auto-reset on."""
    for n in (1, 2):
        cfg = dict(num_envs=E, num_agents=n, lidar_rays=64, use_team_reward=1, max_steps=90, seed=5)
        hs = [mev.Handle(**cfg) for _ in range(4)]
        hs[0].set_step_kernel(1)
        hs[1].set_step_kernel(2)
        hs[1].set_step_pack(1)
        hs[2].set_step_kernel(2)
        hs[2].set_step_pack(pack)
        hs[2].set_step_split(1)
        hs[3].set_step_kernel(2)
        hs[3].set_step_pack(pack)
        hs[3].set_step_split(2)  # two waves per workgroup
        assert hs[2].step_pack() == min(pack, 8 // n) and hs[1].step_pack() == 1
        assert hs[3].step_split() and not hs[2].step_split()
        rng = np.random.default_rng(13)
        for t in range(120):
            a = rng.uniform(-1, 1, (E, n, 2)).astype(np.float32)
            o = [h.step(a, auto_reset=True) for h in hs]
            for k in o[0]:
                assert np.array_equal(o[0][k], o[1][k]), (n, t, k)
                assert np.array_equal(o[0][k], o[2][k]), (n, t, k)
                assert np.array_equal(o[0][k], o[3][k]), (n, t, k)
        s = [h.get_state() for h in hs]
        for k in s[0]:
            assert np.array_equal(s[0][k], s[2][k]), (n, k)
            assert np.array_equal(s[0][k], s[3][k]), (n, k)
        for h in hs:
            h.close()


def test_fused_and_two_kernel_paths_agree_traffic_full_size(mev):
    """Config 4 shape (4096 envs x 1 ego x 64 beams, traffic at density 0.5 with
    the Philox spawn stream, 32 NPC slots): the fused k_step (NPC phase, car
    part and LiDAR in one wave) and k_cars + k_lidar agree bit for bit, step
    after step, with auto-reset on; the NPC fleets (counts and every NPC
    field) too.  A third handle runs the traffic early split (two car waves and
    one LiDAR wave per workgroup, the NPC-aware deal over 2-env workgroups)."""
    cfg = dict(num_envs=E, num_agents=1, lidar_rays=64, traffic_flow=1, traffic_density=0.5, max_npcs=32,
               max_steps=300, seed=11)
    hs = [mev.Handle(**cfg) for _ in range(3)]
    for h, kernel in zip(hs, (1, 2, 2)):
        h.set_step_kernel(kernel)
    hs[1].set_step_split(1)  # one wave per env (the automatic choice here is the early split)
    assert hs[2].step_split() == 2 and hs[1].step_split() == 0
    rng = np.random.default_rng(12)
    most = 0
    for t in range(400):
        a = rng.uniform(-1, 1, (E, 1, 2)).astype(np.float32)
        o1 = hs[0].step(a, auto_reset=True)
        o2 = hs[1].step(a, auto_reset=True)
        o3 = hs[2].step(a, auto_reset=True)
        for k in o1:
            assert np.array_equal(o1[k], o2[k]), (t, k)
            assert np.array_equal(o1[k], o3[k]), (t, k, "split")
        if t % 50 == 49 or t == 399:
            s1, s2, s3 = hs[0].get_state(), hs[1].get_state(), hs[2].get_state()
            for k in s1:
                assert np.array_equal(s1[k], s2[k]), (t, k)
                assert np.array_equal(s1[k], s3[k]), (t, k, "split")
            most = max(most, int(s1["npc_count"].max()))
    assert most >= 4  # busy intersections were exercised
    for h in hs:
        h.close()


def test_env_deal_exact_beyond_residency(mev):
    """The fused traffic kernel's NPC-aware env deal is scheduling only: with
    16384 envs (four residency rounds of 4 waves per SIMD, so workgroups start
    while earlier ones of the same step have already appended to the next
    step's orders) the deal and the identity order agree bit for bit, every
    output each step and the whole state (NPC fleets included) every 25 steps,
    with auto-resets and busy intersections.  A third handle deals 4-env
    workgroups of the traffic early split (switched on after 40 steps of the
    one-env kernel; the deal then restarts from the identity order)."""
    E4 = 16384
    cfg = dict(num_envs=E4, num_agents=1, lidar_rays=64, traffic_flow=1, traffic_density=2.0, max_npcs=32,
               max_steps=90, seed=21)
    hs = [mev.Handle(**cfg) for _ in range(3)]
    hs[1].set_env_deal(False)
    hs[0].set_step_split(3)  # the deal on the early split (not automatic beyond 4096 envs)
    hs[1].set_step_split(1)  # the identity order on the one-wave-per-env kernel
    hs[2].set_step_split(1)  # the deal on the one-wave kernel, then (below) on the early split
    for h in hs:
        assert h.step_kernel() == 2
    assert hs[0].step_split() == 2 and hs[1].step_split() == 0 and hs[2].step_split() == 0
    rng = np.random.default_rng(22)
    most = 0
    for t in range(150):
        if t == 40:
            hs[2].set_step_split(3)
            assert hs[2].step_split() == 2
        a = rng.uniform(-1, 1, (E4, 1, 2)).astype(np.float32)
        o1 = hs[0].step(a, auto_reset=True)
        o2 = hs[1].step(a, auto_reset=True)
        o3 = hs[2].step(a, auto_reset=True)
        for k in o1:
            assert np.array_equal(o1[k], o2[k]), (t, k)
            assert np.array_equal(o1[k], o3[k]), (t, k, "split")
        if t % 25 == 24:
            s1, s2, s3 = hs[0].get_state(), hs[1].get_state(), hs[2].get_state()
            for k in s1:
                assert np.array_equal(s1[k], s2[k]), (t, k)
                assert np.array_equal(s1[k], s3[k]), (t, k, "split")
            most = max(most, int(s1["npc_count"].max()))
    assert most >= 5  # the deal sorted envs over several NPC classes
    for h in hs:
        h.close()


def test_step_kernel_selection(mev):
    h = _handle(mev)
    assert h.step_kernel() == 2  # automatic: fused at 4096 envs
    h.set_step_kernel(1)
    assert h.step_kernel() == 1
    with pytest.raises(mev.MevError):
        h.set_step_kernel(3)
    h.set_step_kernel(2)
    h.configure_traffic(1, 0.5)  # the fused kernel runs the NPC phase too
    assert h.step_kernel() == 2
    h.set_step_kernel(0)
    # automatic: 8 egos + 64 NPC slots need more than a wave's 10 KB LDS share
    assert h.step_kernel() == 1
    h.set_step_kernel(2)
    assert h.step_kernel() == 2
    h.close()
    small = _handle(mev, num_envs=64)
    assert small.step_kernel() == 2  # automatic: the 8-slot fused kernel at every batch size (8 agents x 64 beams)
    small.set_step_kernel(1)
    assert small.step_kernel() == 1
    small.close()
    big = mev.Handle(num_envs=64, num_agents=12, lidar_rays=64)
    assert big.step_kernel() == 1  # automatic: finer LiDAR waves for small batches of larger envs
    big.close()
    tiny = mev.Handle(num_envs=1, num_agents=1, lidar_rays=16)
    assert tiny.step_kernel() == 2  # automatic: one agent's beams fit one LiDAR wave, one launch
    tiny.close()
    # config 4 shape (1 ego, traffic, 32 NPC slots): fused automatically, as the traffic early
    # split (two car waves + a LiDAR wave per workgroup) where E is a multiple of 16
    t = mev.Handle(num_envs=4096, num_agents=1, lidar_rays=64, traffic_flow=1, traffic_density=0.5, max_npcs=32)
    assert t.step_kernel() == 2 and t.step_split() == 2
    t.set_step_split(1)
    assert t.step_split() == 0
    t.close()
    for e_ in (4088, 1000):  # (not a multiple of 16: one wave per env)
        t = mev.Handle(num_envs=e_, num_agents=1, lidar_rays=64, traffic_flow=1, traffic_density=0.5, max_npcs=32)
        assert t.step_split() == 0, e_
        t.close()


def test_env_permutation_equivariance(mev):
    st = _warm_state(mev, seed=2)
    rng = np.random.default_rng(3)
    perm = rng.permutation(E)
    acts = rng.uniform(-1, 1, (8, E, N, 2)).astype(np.float32)
    h1, h2 = _handle(mev), _handle(mev)
    h1.set_state(st)
    h2.set_state({k: v[perm] for k, v in st.items()})
    for a in acts:
        o1 = h1.step(a)
        o2 = h2.step(a[perm])
        for k in o1:
            assert np.array_equal(o1[k][perm], o2[k]), k
    h1.close()
    h2.close()


def test_batched_equals_single_env(mev):
    st = _warm_state(mev, seed=4)
    rng = np.random.default_rng(5)
    acts = rng.uniform(-1, 1, (6, E, N, 2)).astype(np.float32)
    hb = _handle(mev)
    hb.set_state(st)
    picks = [0, 1, 777, 4095]
    singles = []
    for e in picks:
        hs = mev.Handle(num_envs=1, num_agents=N, lidar_rays=R, use_team_reward=1)
        hs.set_state({k: v[e:e + 1] for k, v in st.items()})
        singles.append(hs)
    for a in acts:
        ob = hb.step(a)
        for e, hs in zip(picks, singles):
            os_ = hs.step(a[e:e + 1])
            for k in ob:
                assert np.array_equal(ob[k][e:e + 1], os_[k]), (e, k)
    for hs in singles:
        hs.close()
    hb.close()


def test_truncation_and_auto_reset(mev):
    h = _handle(mev, max_steps=30)
    rng = np.random.default_rng(6)
    st0 = h.get_state()
    for t in range(30):
        o = h.step(rng.uniform(-1, 1, (E, N, 2)).astype(np.float32), auto_reset=True)
    assert o["truncated"].all() and (o["step"] == 30).all()
    o = h.step(np.zeros((E, N, 2), np.float32), auto_reset=True)
    assert (o["step"] == 1).all() and not o["truncated"].any()
    st = h.get_state()
    # the step after an auto-reset starts from the spawn poses
    assert np.array_equal(st["spawn_x"], st0["spawn_x"])
    h.close()


def test_output_invariants(mev):
    h = _handle(mev)
    rng = np.random.default_rng(7)
    for t in range(120):
        o = h.step(rng.uniform(-1, 1, (E, N, 2)).astype(np.float32), auto_reset=True)
    obs = o["obs"]
    assert np.isfinite(obs).all()
    lid = obs[..., 31:]
    assert (lid >= 0).all() and (lid <= 1.0000001).all()
    # LiDAR distances are multiples of the 4 px step (or max_dist)
    d = np.rint(lid * 250.0)
    assert (np.isclose(lid * 250.0, d, atol=1e-3)).all()
    assert ((d % 4 == 0) | (d == 250)).all()
    assert set(np.unique(o["status"]).tolist()) <= {0, 2, 3, 4, 5}
    assert np.array_equal(o["done"] == 1, o["status"] != 0)
    assert (o["agents_alive"] == N).all()
    h.close()


def test_traffic_full_size_philox_spawns(mev):
    h = mev.Handle(num_envs=E, num_agents=1, lidar_rays=R, traffic_flow=1, traffic_density=0.5, max_npcs=32)
    rng = np.random.default_rng(8)
    counts = []
    for t in range(240):
        h.step(rng.uniform(-1, 1, (E, 1, 2)).astype(np.float32), auto_reset=True)
        if t % 40 == 39:
            counts.append(h.get_state()["npc_count"].copy())
    c = np.stack(counts)
    assert c.max() <= 32 and c.mean() > 0.3
    # spawn attempts follow p = 1 - exp(-0.5/60) per env-step: after 240 steps about
    # 240 * 0.00830 ~ 2 attempts per env, most of them accepted
    assert 0.5 < c[-1].mean() < 3.0
    assert h.npc_overflow() == 0
    h.close()
