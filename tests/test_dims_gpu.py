"""Per-car sizes (reference Car::length / Car::width, cpp/Car.h:19-20, read-write through
cpp/bindings.cpp:24-25) on the device: the C ABI's bookkeeping around them (mev_set_car_dims).
Their arithmetic is pinned elsewhere: the dims_* / path_* goldens recorded from the reference
(tests/test_parity_gpu.py, both kernel paths) and randomized sizes against the oracle
(tests/test_gpu_vs_oracle.py dims_*)."""
import numpy as np
import pytest

import golden_replay as G

pytestmark = pytest.mark.gpu


def _default(a):
    d = np.empty_like(a)
    d[...] = (54.0, 24.0)
    return d


def _handle(mev, **kw):
    cfg = dict(num_envs=6, num_agents=4, lidar_rays=32, max_npcs=8)
    cfg.update(kw)
    return mev.Handle(**cfg)


def test_dims_flag_roundtrip_and_validation(mev):
    h = _handle(mev)
    ego, npc = h.car_dims()
    assert (ego == (54.0, 24.0)).all() and (npc == (54.0, 24.0)).all() and not h.car_dims_active()
    k_fixed = h.step_kernel(), h.step_pack(), h.step_split()
    ego2 = ego.copy()
    ego2[2, 1] = (80.0, 31.5)
    h.set_car_dims(ego2, None)  # NPC sizes unchanged
    assert h.car_dims_active()
    e3, n3 = h.car_dims()
    assert G.bits_equal(e3, ego2) and G.bits_equal(n3, npc)
    assert h.step_pack() == 1 and h.step_split() == 0  # the runtime-layout kernels
    npc2 = npc.copy()
    npc2[0, 3] = (10.0, 70.0)
    h.set_car_dims(None, npc2)
    assert G.bits_equal(h.car_dims()[1], npc2) and G.bits_equal(h.car_dims()[0], ego2)
    h.set_car_dims(ego, npc)  # all back at 54 x 24: the compile-time kernels again
    assert not h.car_dims_active()
    assert (h.step_kernel(), h.step_pack(), h.step_split()) == k_fixed
    for bad in (np.nan, np.inf, 2.0e4):
        b = ego.copy()
        b[0, 0, 0] = bad
        with pytest.raises(mev.MevError):
            h.set_car_dims(b, None)
    assert not h.car_dims_active()
    h.close()


@pytest.mark.parametrize("traffic", [False, True])
def test_dims_reset_gives_default_size(mev, traffic):
    """A reset makes new Cars (IntersectionEnv::reset + add_car_with_route): egos of the default size;
    the auto-reset of a step too (its env only).  A respawn keeps the size (Car::respawn)."""
    h = _handle(mev, traffic_flow=int(traffic), max_steps=5, num_agents=1 if traffic else 4)
    ego = np.empty((h.E, h.N, 2), np.float32)
    ego[...] = (90.0, 40.0)
    h.set_car_dims(ego, None)
    h.reset(env_mask=np.array([1, 0, 1, 0, 0, 0], np.uint8))
    e2, _ = h.car_dims()
    assert (e2[[0, 2]] == (54.0, 24.0)).all() and (e2[[1, 3, 4, 5]] == (90.0, 40.0)).all()
    h.set_car_dims(ego, None)
    acts = np.zeros((h.E, h.N, 2), np.float32)
    for t in range(6):  # max_steps 5: every env truncates at step 5, auto-resets at step 6
        h.step(acts, auto_reset=True)
        if t < 5:
            assert (h.car_dims()[0] == (90.0, 40.0)).all(), t
    assert (h.car_dims()[0] == (54.0, 24.0)).all()
    h.close()


def test_dims_snapshot_restore(mev):
    h = _handle(mev, traffic_flow=1, num_agents=2)
    rng = np.random.default_rng(3)
    ego = rng.uniform(20, 100, (h.E, h.N, 2)).astype(np.float32)
    npc = rng.uniform(20, 100, (h.E, h.K, 2)).astype(np.float32)
    h.set_car_dims(ego, npc)
    snap = h.snapshot()
    h.set_car_dims(_default(ego), _default(npc))
    assert not h.car_dims_active()
    h.restore(snap)
    assert h.car_dims_active()
    e2, n2 = h.car_dims()
    assert G.bits_equal(e2, ego) and G.bits_equal(n2, npc)
    # masked restore: only env 1 takes the snapshot's sizes; the flag covers both
    h.set_car_dims(_default(ego), _default(npc))
    mask = np.zeros(h.E, np.uint8)
    mask[1] = 1
    h.restore(snap, env_mask=mask)
    e3, _ = h.car_dims()
    assert h.car_dims_active() and G.bits_equal(e3[1], ego[1]) and (e3[0] == (54.0, 24.0)).all()
    h.close()


def test_restore_checks_route_table(mev):
    """A snapshot names routes by id: it restores only into a handle whose route table begins with
    the same routes (restoring custom-route ids into a handle without them read past
    the end of its tables)."""
    a = _handle(mev)
    path, _, _ = a.route_info(a.route_id(0, 12 + 3))
    bent = path.copy()
    bent[40:120, 0] += 5.0
    r = a.add_route(bent, 0)
    st = a.get_state()
    st["route"][0, 0] = r
    a.set_state(st)
    snap = a.snapshot()
    b = _handle(mev)  # no custom route
    with pytest.raises(mev.MevError):
        b.restore(snap)
    c = _handle(mev)  # another custom route under the same id
    other = path.copy()
    other[40:120, 1] += 5.0
    assert c.add_route(other, 0) == r
    with pytest.raises(mev.MevError):
        c.restore(snap)
    d = _handle(mev)  # the same route, then one more: restores
    assert d.add_route(bent, 0) == r
    d.add_route(other, 0)
    d.restore(snap)
    assert int(d.get_state()["route"][0, 0]) == r
    for x in (a, b, c, d):
        x.close()


def test_add_route_grows_tables_geometrically(mev):
    """mev_add_route fills spare table capacity (doubling when full): many routes, every one intact."""
    h = _handle(mev, num_envs=2)
    base, _, _ = h.route_info(h.route_id(1, 12 + 7))
    ids = []
    for k in range(40):
        p = base.copy()
        p[50:110, 0] += 0.25 * (k + 1)
        ids.append((h.add_route(p, k % 3), p, k % 3))
    for r, p, it in ids:
        got, intent, spawn = h.route_info(r)
        assert G.bits_equal(got, p) and intent == it and tuple(spawn[:2]) == tuple(p[0])
    st = h.get_state()
    st["route"][1, 2] = ids[-1][0]
    h.set_state(st)
    h.step(np.zeros((h.E, h.N, 2), np.float32))
    assert int(h.get_state()["route"][1, 2]) == ids[-1][0]
    h.close()


def test_beam_angles(mev):
    """Lidar::rel_angles writes (cpp/bindings.cpp:92): any finite list with |angle| <= 1000 rad is
    taken (lists the per-box beam culling cannot model -- uneven, descending -- run without it;
    their simulation is pinned in test_gpu_vs_oracle.py rel_*), non-finite ones are refused;
    a handle whose rays are the first 32 of the reference's 96-beam list casts exactly those beams."""
    h = _handle(mev, lidar_rays=32, lidar_fov_deg=360.0)
    f32 = np.float32
    start, stepd = f32(-360.0) * f32(0.5), f32(360.0) / f32(95)
    rel96 = np.array([(start + f32(i) * stepd) * f32(np.pi) / f32(180.0) for i in range(96)], np.float32)
    h.set_beam_angles(rel96[:32])
    assert G.bits_equal(h.beam_angles(), rel96[:32])
    uneven = rel96[:32].copy()
    uneven[7] += 0.01
    for ok in (uneven, rel96[:32][::-1].copy(), np.full(32, 0.5, np.float32)):
        h.set_beam_angles(ok)
        assert G.bits_equal(h.beam_angles(), ok)
    bad = rel96[:32].copy()
    bad[3] = np.inf
    with pytest.raises(mev.MevError):
        h.set_beam_angles(bad)
    bad[3] = 1001.0
    with pytest.raises(mev.MevError):
        h.set_beam_angles(bad)
    assert G.bits_equal(h.beam_angles(), np.full(32, 0.5, np.float32))
    h.close()
