"""Error behaviour of the C ABI (negative MEV_E* codes + mev_last_error, never an
exception across the boundary), mirrored by the Python binding as MevError /
IndexRangeError (IndexError, like the reference's std::out_of_range)."""
import ctypes

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("cfg", [
    dict(num_envs=0), dict(num_agents=0), dict(num_agents=65), dict(num_lanes=0), dict(num_lanes=9),
    dict(lidar_rays=0), dict(lidar_rays=1025), dict(lidar_step=0.0), dict(lidar_max_dist=-1.0),
    dict(max_npcs=65), dict(obs_dim=20), dict(device=99),
])
def test_invalid_configs_are_rejected(mev, cfg):
    with pytest.raises(mev.MevError) as ei:
        mev.Handle(**cfg)
    assert str(ei.value)


def test_out_of_range_routes_raise_index_error(mev):
    h = mev.Handle(num_envs=2, num_agents=2, lidar_rays=16)
    P = h.num_points
    with pytest.raises(IndexError):
        h.route_id(P, 0)
    with pytest.raises(IndexError):
        h.route_info(P * P)
    with pytest.raises(IndexError):
        h.set_ego_routes(np.full((2, 2), P * P, np.int32))
    with pytest.raises(IndexError):
        h.set_traffic_routes([-1])
    with pytest.raises(IndexError):
        h.set_reset_routes([P * P + 5])
    st = h.get_state()
    st["npc_count"][:] = 99
    with pytest.raises(IndexError):
        h.set_state(st)
    h.close()


def test_wrong_action_shape_is_rejected_before_the_device(mev):
    h = mev.Handle(num_envs=3, num_agents=2, lidar_rays=16)
    with pytest.raises(ValueError):
        h.step(np.zeros((3, 3, 2), np.float32))
    h.close()


def test_handle_survives_errors(mev):
    h = mev.Handle(num_envs=4, num_agents=2, lidar_rays=16)
    with pytest.raises(IndexError):
        h.route_info(-1)
    o = h.step(np.zeros((4, 2, 2), np.float32))
    assert o["step"].tolist() == [1, 1, 1, 1]
    h.close()


def test_large_batch_allocates_and_steps(mev):
    """One handle of 131072 envs x 8 agents (a quarter of cfg5's node-wide batch on one GPU)."""
    E = 131072
    h = mev.Handle(num_envs=E, num_agents=8, lidar_rays=64, use_team_reward=1)
    rng = np.random.default_rng(0)
    for _ in range(3):
        o = h.step(rng.uniform(-1, 1, (E, 8, 2)).astype(np.float32), auto_reset=True)
    assert np.isfinite(o["obs"]).all() and (o["step"] == 3).all()
    h.close()


def test_add_route_validates_and_extends_the_id_range(mev):
    """mev_add_route (a written Car.path): bad paths and intents are refused with
    nothing added; a good one gets id P*P and becomes a valid ego / traffic / reset
    route, read back by mev_route_info exactly (spawn = its first point)."""
    h = mev.Handle(num_envs=2, num_agents=2, lidar_rays=16)
    P = h.num_points
    path = h.route_info(h.route_id(0, 13))[0] + np.float32(3.0)
    bad = path.copy()
    bad[7, 1] = np.nan
    with pytest.raises(mev.MevError):
        h.add_route(bad, 0)
    with pytest.raises(mev.MevError):
        h.add_route(path, 3)
    for n in (0, 1, 4097):  # 2 .. 4096 points (the Python layer refuses, and the C ABI)
        with pytest.raises(ValueError):
            h.add_route(np.resize(path, (n, 2)), 0)
        raw = np.resize(path, (max(n, 1), 2))
        assert h._lib.mev_add_route_n(h._h, raw.ctypes.data_as(ctypes.POINTER(ctypes.c_float)), n, 0,
                                      ctypes.byref(ctypes.c_int32())) == -1  # MEV_E_INVALID
    with pytest.raises(IndexError):
        h.route_info(P * P)
    r = h.add_route(path, 1)
    assert r == P * P
    got, intent, spawn = h.route_info(r)
    assert (got.view(np.uint32) == path.view(np.uint32)).all() and intent == 1
    assert spawn[0] == path[0, 0] and spawn[1] == path[0, 1]
    h.set_ego_routes(np.full((2, 2), r, np.int32))
    h.set_traffic_routes([r, h.route_id(1, 14)])
    h.set_reset_routes([r])
    h.reset()
    h.step(np.zeros((2, 2, 2), np.float32))
    st = h.get_state()
    assert (st["route"] == r).all() and st["x"][0, 0] == path[0, 0]
    with pytest.raises(IndexError):
        h.route_info(r + 1)
    assert h.route_len(r) == 160 and h.route_len(0) == 160
    # a 37-point path: read back padded with its last point, its length kept
    r2 = h.add_route(path[:37], 2)
    got, intent, _ = h.route_info(r2)
    assert r2 == r + 1 and intent == 2 and h.route_len(r2) == 37
    assert (got[:37].view(np.uint32) == path[:37].view(np.uint32)).all()
    assert (got[37:].view(np.uint32) == path[36].view(np.uint32)).all()
    h.close()


def test_snapshot_format_1_is_refused_by_name(mev):
    """A format-1 snapshot (before per-car sizes and the route hash) is refused with its own
    message, and the handle is left as it was."""
    h = mev.Handle(num_envs=2, num_agents=2, lidar_rays=16)
    h.reset()
    snap = h.snapshot()
    old = snap.copy()
    old[4:8] = np.frombuffer(np.uint32(1).tobytes(), np.uint8)  # SnapHeader::version
    with pytest.raises(mev.MevError, match="format 1"):
        h.restore(old)
    h.restore(snap)  # the current format still restores
    h.close()
