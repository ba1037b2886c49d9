"""The persistent step server (k_serve, mev_set_serve, include/marlenv.h): host-mode
steps of small handles answered by a resident kernel through a mailbox in pinned
memory.  Every output and the state must equal the launched step's bit for bit --
including across idle exits and relaunches, other calls that stop the server in the
middle of a run (get_state, device-mode steps, reset) and recorded NPC spawns.  The
single env of the reference's env.py (cpp/bindings.cpp:53-55) is the case it is for."""
import time

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SHAPES = [
    dict(num_envs=1, num_agents=1, lidar_rays=16),
    dict(num_envs=1, num_agents=8, lidar_rays=64, use_team_reward=1),
    dict(num_envs=16, num_agents=4, lidar_rays=96),
    dict(num_envs=1, num_agents=1, lidar_rays=64, traffic_flow=1, traffic_density=0.5, max_npcs=32),
    dict(num_envs=4, num_agents=1, lidar_rays=32, traffic_flow=1, traffic_density=3.0, max_npcs=32),
    # env.py's traffic env: 64 NPC slots (the dynamic layout), 96 beams, the reference's 127-float rows
    dict(num_envs=1, num_agents=1, lidar_rays=96, traffic_flow=1, traffic_density=2.0, max_npcs=64, obs_dim=127),
]
IDS = ["cfg1", "cfg3_one_env", "e16_n4_r96", "cfg4_one_env", "traffic_e4", "envpy_traffic_k64"]


def _pair(mev, cfg):
    a = mev.Handle(seed=7, **cfg)
    b = mev.Handle(seed=7, **cfg)
    b.set_serve(0)
    return a, b


def _same(oa, ob, what):
    for k in oa:
        assert np.array_equal(oa[k], ob[k]), (what, k)


@pytest.mark.parametrize("cfg", SHAPES, ids=IDS)
def test_served_steps_equal_launched_steps(mev, cfg):
    a, b = _pair(mev, cfg)
    E, N = a.E, a.N
    rng = np.random.default_rng(3)
    a.reset()
    b.reset()
    T = 240
    acts = rng.uniform(-1, 1, (T, E, N, 2)).astype(np.float32)
    traffic = bool(cfg.get("traffic_flow"))
    for t in range(T):
        spawn = None
        if traffic and 60 <= t < 90:  # recorded spawns (the replay channel) for a while
            spawn = rng.integers(-1, 4, E).astype(np.int32)
        oa = a.step(acts[t], auto_reset=True, spawn_route=spawn)
        ob = b.step(acts[t], auto_reset=True, spawn_route=spawn)
        _same(oa, ob, t)
        if t == 100:
            time.sleep(0.2)  # longer than the server's idle limit: it leaves, the next step relaunches
        if t == 150:
            sa, sb = a.get_state(), b.get_state()  # stops the server
            for k in sa:
                assert np.array_equal(sa[k], sb[k]), k
    st = a.serve_stats()
    assert st["steps"] == T, st
    assert st["launches"] >= 3, st  # first step, after the idle pause, after get_state
    assert b.serve_stats()["steps"] == 0
    sa, sb = a.get_state(), b.get_state()
    for k in sa:
        assert np.array_equal(sa[k], sb[k]), k
    a.close()
    b.close()


def test_serve_interleaved_with_device_steps_and_resets(mev):
    import torch
    cfg = dict(num_envs=2, num_agents=2, lidar_rays=32)
    a, b = _pair(mev, cfg)
    E, N = a.E, a.N
    torch.cuda.set_device(0)
    rng = np.random.default_rng(5)
    a.reset()
    b.reset()
    dev_out = {k: torch.as_tensor(v).cuda() for k, v in a.alloc_outputs().items()}
    for t in range(120):
        act = rng.uniform(-1, 1, (E, N, 2)).astype(np.float32)
        if t % 7 == 3:  # a device-mode step between served host steps
            ta = torch.as_tensor(act).cuda()
            a.step(ta.data_ptr(), out={k: v.data_ptr() for k, v in dev_out.items()}, auto_reset=True, device=True)
            torch.cuda.synchronize()
            oa = {k: v.cpu().numpy() for k, v in dev_out.items()}
        else:
            oa = a.step(act, auto_reset=True)
        ob = b.step(act, auto_reset=True)
        _same(oa, ob, t)
        if t == 60:
            a.reset()
            b.reset()
    assert a.serve_stats()["steps"] > 90
    a.close()
    b.close()


def test_serve_off_and_on(mev):
    a = mev.Handle(num_envs=1, num_agents=1, lidar_rays=16)
    a.reset()
    act = np.zeros((1, 1, 2), np.float32)
    a.step(act)
    assert a.serve_stats()["running"]
    a.set_serve(0)
    assert not a.serve_stats()["running"]
    a.step(act)
    assert a.serve_stats()["steps"] == 1
    a.set_serve(1)
    a.step(act)
    assert a.serve_stats()["steps"] == 2
    with pytest.raises(Exception):
        a.set_serve(2)
    a.close()


def test_large_handles_are_not_served(mev):
    a = mev.Handle(num_envs=128, num_agents=1, lidar_rays=16)  # more than 64 workgroups
    a.reset()
    a.step(np.zeros((128, 1, 2), np.float32))
    assert a.serve_stats()["steps"] == 0
    a.close()


def test_torch_work_runs_beside_a_resident_server(mev):
    import torch
    a = mev.Handle(num_envs=1, num_agents=1, lidar_rays=16)
    a.reset()
    act = np.zeros((1, 1, 2), np.float32)
    a.step(act)
    assert a.serve_stats()["running"]
    x = torch.ones(4096, device="cuda")
    (x * 2).sum().item()  # (the first torch kernels may take longer than the server's idle limit)
    a.step(act)
    n0 = a.serve_stats()["launches"]
    t0 = time.perf_counter()
    for _ in range(50):
        a.step(act)
        (x * 2).sum().item()  # torch's stream, synchronised every call, while the server stays resident
    dt = (time.perf_counter() - t0) / 50
    assert dt < 0.005, dt  # nothing waits for the server's idle exit
    # it stayed resident (a rare host hiccup longer than the adaptive idle limit
    # only costs a relaunch)
    assert a.serve_stats()["launches"] - n0 <= 3
    a.set_stream(torch.cuda.current_stream().cuda_stream)  # a shared stream: launched steps only
    a.step(act)
    assert not a.serve_stats()["running"]
    assert a.serve_stats()["steps"] == 52
    a.close()


def test_device_wide_sync_between_served_steps():
    """An RL loop that calls torch.cuda.synchronize() (a device-wide wait, which also
    waits for a resident server's idle exit) between env.py steps: the adaptive idle
    limit (<= 2 ms, then launched steps after repeated idle exits) keeps each step
    well under 2 ms; without the synchronisation the same env is served."""
    import torch

    import pkgload
    pkgload.load()
    from marl_traffic_intersection_amd import env as envmod
    env = envmod.IntersectionEnv({"num_agents": 1})
    act = np.zeros((1, 2), np.float32)
    x = torch.ones(1024, device="cuda")
    (x * 2).sum().item()
    for _ in range(20):
        env.step(act)
    h = env.env._sync()
    s0 = h.serve_stats()
    t0 = time.perf_counter()
    n = 300
    for _ in range(n):
        env.step(act)
        torch.cuda.synchronize()
    per_step = (time.perf_counter() - t0) / n
    assert per_step < 0.002, per_step
    s1 = h.serve_stats()
    # (most of these steps ran launched: the server kept leaving before the next post)
    assert s1["steps"] - s0["steps"] < n
    # without device-wide waits, served again once the pause is over
    for _ in range(1100):
        env.step(act)
    s2 = h.serve_stats()
    t0 = time.perf_counter()
    for _ in range(200):
        env.step(act)
    served_dt = (time.perf_counter() - t0) / 200
    s3 = h.serve_stats()
    assert s3["steps"] - s2["steps"] >= 190, (s2, s3)
    assert served_dt < 0.001, served_dt
    env.close()


@pytest.mark.parametrize("traffic", [False, True], ids=["egos", "traffic"])
def test_env_py_through_the_server(traffic):
    """The drop-in env.py (one env per call) with its handle served and not served:
    the same observations, rewards, flags, info and traffic cars at every step."""
    import pkgload
    pkgload.load()
    from marl_traffic_intersection_amd import env as envmod
    cfg = {"num_agents": 1 if traffic else 3, "traffic_flow": traffic, "traffic_density": 2.0}
    envs = [envmod.IntersectionEnv(dict(cfg)) for _ in range(2)]
    rng = np.random.default_rng(11)
    n = 1 if traffic else 3
    first = rng.uniform(-1, 1, (n, 2)).astype(np.float32)
    for e in envs:
        e.step(first)
    envs[1].env._sync().set_serve(0)
    for t in range(150):
        act = rng.uniform(-1, 1, (n, 2)).astype(np.float32)
        ra, rb = envs[0].step(act), envs[1].step(act)
        assert np.array_equal(ra[0], rb[0]), t
        assert np.array_equal(np.asarray(ra[1]), np.asarray(rb[1])), t
        assert ra[2:4] == rb[2:4] and ra[4] == rb[4], t
        if traffic and t % 10 == 0:
            ca, cb = envs[0].traffic_cars, envs[1].traffic_cars
            assert [(c.state.x, c.state.y, c.state.heading, c.path_index) for c in ca] == \
                   [(c.state.x, c.state.y, c.state.heading, c.path_index) for c in cb], t
        if ra[2] or ra[3]:
            envs[0].reset()
            envs[1].reset()
    assert envs[0].env._sync().serve_stats()["steps"] > 100
    assert envs[1].env._sync().serve_stats()["steps"] == 1  # (its first step, before set_serve(0))
    for e in envs:
        e.close()


def test_several_served_handles_at_once(mev):
    """Four single-env handles stepped round-robin (a process running several env.py envs)
    against four launched twins: the first two get resident servers (the per-process cap)."""
    served = [mev.Handle(seed=s, num_envs=1, num_agents=2, lidar_rays=32) for s in range(4)]
    launched = [mev.Handle(seed=s, num_envs=1, num_agents=2, lidar_rays=32) for s in range(4)]
    for h in launched:
        h.set_serve(0)
    for h in served + launched:
        h.reset()
    rng = np.random.default_rng(9)
    s0 = None
    for t in range(110):
        if t == 10:  # (after the first rounds: kernel code loading may outlast an idle limit)
            t0 = time.perf_counter()
            s0 = [h.serve_stats()["steps"] for h in served]
        for i in range(4):
            act = rng.uniform(-1, 1, (1, 2, 2)).astype(np.float32)
            _same(served[i].step(act, auto_reset=True), launched[i].step(act, auto_reset=True), (t, i))
    # nothing waits for a server's idle exit: each server has a hardware queue of its own
    # (sharing one, each launched step would wait for the idle exit behind a resident server)
    assert time.perf_counter() - t0 < 2.0
    d = [h.serve_stats()["steps"] - a for h, a in zip(served, s0)]
    # two resident servers per process at most: the two handles that stepped first keep
    # their slots (across idle exits) and are served (almost) throughout
    assert d[0] >= 95 and d[1] >= 95 and sum(d[2:]) == 0, d
    for h in served + launched:
        h.close()


def test_resident_servers_are_capped(mev):
    """More single-env handles than the per-process cap of resident servers: the rest step
    launched, every handle stays exact, and nobody waits behind another handle's server."""
    hs = [mev.Handle(seed=s, num_envs=1, num_agents=1, lidar_rays=16) for s in range(6)]
    twins = [mev.Handle(seed=s, num_envs=1, num_agents=1, lidar_rays=16) for s in range(6)]
    for h in twins:
        h.set_serve(0)
    for h in hs + twins:
        h.reset()
    rng = np.random.default_rng(4)
    s0 = None
    for t in range(110):
        if t == 10:  # (after the first rounds: kernel code loading may outlast an idle limit)
            t0 = time.perf_counter()
            s0 = [h.serve_stats()["steps"] for h in hs]
        for i in range(6):
            act = rng.uniform(-1, 1, (1, 1, 2)).astype(np.float32)
            _same(hs[i].step(act, auto_reset=True), twins[i].step(act, auto_reset=True), (t, i))
    assert time.perf_counter() - t0 < 2.0
    d = [h.serve_stats()["steps"] - a for h, a in zip(hs, s0)]
    # kMaxResidentServers: handles 0 and 1 (the first to step) served throughout, the
    # others launched -- slot ownership does not move with idle exits
    assert d[0] >= 95 and d[1] >= 95 and sum(d[2:]) == 0, d
    for h in hs + twins:
        h.close()


def test_server_slots_follow_their_owners(mev):
    """Slot ownership (marlenv.h, mev_set_serve): the first two handles to step own the
    two server slots; a third is launched while they keep stepping; it takes a slot
    once an owner turns serving off, or has made no host step for 50 ms -- and every
    step stays exact against launched twins."""
    hs = [mev.Handle(seed=s, num_envs=1, num_agents=1, lidar_rays=16) for s in range(3)]
    tw = [mev.Handle(seed=s, num_envs=1, num_agents=1, lidar_rays=16) for s in range(3)]
    for h in tw:
        h.set_serve(0)
    for h in hs + tw:
        h.reset()
    rng = np.random.default_rng(11)

    def rounds(k, who):
        s0 = [h.serve_stats()["steps"] for h in hs]
        for _ in range(k):
            for i in who:
                act = rng.uniform(-1, 1, (1, 1, 2)).astype(np.float32)
                _same(hs[i].step(act, auto_reset=True), tw[i].step(act, auto_reset=True), i)
        return [h.serve_stats()["steps"] - a for h, a in zip(hs, s0)]

    d = rounds(40, [0, 1, 2])
    assert d[0] >= 35 and d[1] >= 35 and d[2] == 0, d
    hs[1].set_serve(0)  # handle 1 gives its slot up: handle 2's next step takes it
    d = rounds(40, [0, 1, 2])
    assert d[0] >= 35 and d[1] == 0 and d[2] >= 35, d
    hs[1].set_serve(1)  # handle 1 wants one again: both slots are owned and stepping
    d = rounds(40, [0, 1, 2])
    assert d[1] == 0, d
    d = rounds(40, [1, 2])  # handle 0 goes quiet, but only for a few ms: it keeps its slot
    assert d[1] == 0, d
    time.sleep(0.12)  # handle 0 silent for > 50 ms: handle 1 may take its slot
    d = rounds(40, [1, 2])
    assert d[1] >= 35 and d[2] >= 35, d
    for h in hs + tw:
        h.close()


def test_get_state_partial_fields(mev):
    """mev_get_state stages through pinned memory (one copy per SoA block): any subset of
    fields reads the same values as the full call."""
    import ctypes
    from marl_traffic_intersection_amd import _capi
    h = mev.Handle(num_envs=5, num_agents=3, lidar_rays=16, traffic_flow=1, traffic_density=4.0, max_npcs=32)
    h.reset()
    rng = np.random.default_rng(2)
    for _ in range(60):
        h.step(rng.uniform(-1, 1, (5, 3, 2)).astype(np.float32), auto_reset=True)
    full = h.get_state()
    for pick in (["heading"], ["intention", "npc_route"], ["npc_alive", "step_count"], ["alive", "npc_count", "y"]):
        st = _capi.MevState()
        got = {}
        for name, dt, per in _capi.STATE_FIELDS:
            if name in pick:
                got[name] = np.full(h._shape(per), 77, dt)
                setattr(st, name, got[name].ctypes.data)
        _capi._check(h._lib.mev_get_state(h._h, ctypes.byref(st)))
        for k, v in got.items():
            assert np.array_equal(v, full[k]), (pick, k)
    assert full["npc_count"].sum() > 0
    h.close()
