"""Host-side pieces of the drop-in API (no GPU): lane names, reward mapping,
Lidar defaults and the host Car helpers against the reference's recorded
trajectories (tests/golden, generated from the real reference)."""
import math

import numpy as np
import pytest

import golden_replay as G
import pkgload

M = pkgload.load()
from marl_traffic_intersection_amd import cpp_backend, utils, vec_env  # noqa: E402


def test_point_index_roundtrip():
    for L in (1, 2, 3, 4):
        for i in range(8 * L):
            assert utils.point_index(utils.point_name(i, L), L) == i
    assert utils.point_index("IN_13", 3) == -1
    assert utils.point_index("OUT_0", 3) == -1
    assert utils.point_index("MID_1", 3) == -1
    assert utils.point_index("garbage", 3) == -1


def test_default_routes_match_golden_meta():
    meta = G.load("n12_r96_policy")["meta"]
    assert [list(r) for r in utils.default_routes(3)] == meta["ego_routes"]
    meta2 = G.load("lanes2_policy")["meta"]
    assert [list(r) for r in utils.default_routes(2)] == meta2["traffic_routes"]


def test_lane_layout_python_canvas():
    lay = utils.build_lane_layout(3)
    assert lay["points"]["IN_1"] == (450 - 21.0, 30)
    assert lay["points"]["OUT_7"] == (450 - 21.0, 870) and lay["points"]["IN_7"] == (450 + 21.0, 870)
    assert lay["dir_of"]["IN_4"] == "E" and lay["idx_of"]["IN_6"] == 2
    assert len(lay["points"]) == 24


def test_reward_vector_mapping():
    assert vec_env.reward_vector(None) == [10.0, 1.0, -0.01, -10.0, -5.0, 10.0, -0.02, 0.2]
    v = vec_env.reward_vector({"success_reward": 3.0, "team_alpha": 0.5})
    assert v[5] == 3.0 and v[7] == 0.5 and v[0] == 10.0
    with pytest.raises(ValueError):
        vec_env.reward_vector([1.0, 2.0])


def test_reward_config_fields_and_write_through():
    rc = cpp_backend.RewardConfig()
    assert rc.as_list() == pytest.approx([10.0, 1.0, -0.01, -10.0, -5.0, 10.0, -0.02, 0.2])
    with pytest.raises(AttributeError):
        rc.not_a_field = 1.0

    class Owner:
        _reward_dirty = False

    o = Owner()
    object.__setattr__(rc, "_owner", o)
    rc.k_succ = 7
    assert o._reward_dirty and rc.k_succ == 7.0


def test_lidar_defaults_match_reference_ctor():
    """Lidar() (reference cpp/Lidar.cpp:4-14): 72 rays over 360 deg, float32 arithmetic."""
    l_ = cpp_backend.Lidar()
    assert (l_.rays, l_.fov_deg, l_.max_dist, l_.step_size) == (72, 360.0, 250.0, 4.0)
    assert len(l_.distances) == 72 and all(d == 250.0 for d in l_.distances)
    f = np.float32
    start, step = f(-360.0) * f(0.5), f(360.0) / f(71)
    for i in (0, 1, 35, 71):
        want = f(f(start + f(i) * step) * f(math.pi)) / f(180.0)
        assert np.float32(l_.rel_angles[i]) == want
    assert l_.normalized() == [1.0] * 72


def _kin(f):
    return [float(x) for x in f[:6]]


@pytest.mark.parametrize("name", ["n12_r96_policy", "unclipped_x3", "dt_1_30_custom_reward", "cfg1_r16_random"])
def test_car_update_matches_reference_trajectory(name):
    """Car.update (host helper) reproduces every recorded pose of every car that
    stayed alive through a step, bit for bit."""
    g = G.load(name)
    dt = float(g["meta"]["dt"])
    prev = g["init_ego_f"]
    prev_alive = g["init_ego_i"][:, 0]
    checked = 0
    for t in range(len(g["actions"])):
        cur = g["ego_f"][t]
        for i in range(cur.shape[0]):
            if not prev_alive[i] or g["status"][t, i] != 0 or g["flags"][t, 1]:
                continue
            c = cpp_backend.Car()
            c.state = cpp_backend.State(*prev[i, :4])
            c.acc, c.steering_angle = float(prev[i, 4]), float(prev[i, 5])
            c.update(float(g["actions"][t, i, 0]), float(g["actions"][t, i, 1]), dt)
            got = np.array([c.state.x, c.state.y, c.state.v, c.state.heading, c.acc, c.steering_angle], np.float32)
            assert G.bits_equal(got, cur[i, :6]), (name, t, i, got, cur[i, :6])
            checked += 1
        prev, prev_alive = cur, g["ego_i"][t][:, 0]
    assert checked > 100


def test_car_check_collision_cases():
    def car(x, y, h, L=54.0, W=24.0):
        c = cpp_backend.Car()
        c.state = cpp_backend.State(x, y, 0.0, h)
        c.length, c.width = L, W
        return c

    a = car(100, 100, 0.0)
    assert a.check_collision(car(140, 100, 0.0))        # overlapping along the length
    assert not a.check_collision(car(155, 100, 0.0))    # 55 px apart > 54 px length
    assert a.check_collision(car(100, 120, 0.0))        # 20 px lateral < 24 px width
    assert not a.check_collision(car(100, 125, 0.0))
    assert a.check_collision(car(100, 135, math.pi / 2))  # crossing: its length spans 108..162
    assert not a.check_collision(car(100, 150, math.pi / 2, L=20.0))
    assert not a.check_collision(car(150, 140, math.pi / 4))
    # symmetric
    b = car(130, 110, 0.7)
    assert a.check_collision(b) == b.check_collision(a)


def test_backend_classes_shape():
    r = cpp_backend.StepResult()
    assert r.obs.shape == (0, 127) and r.step == 0 and not r.terminated
    s = cpp_backend.EnvState()
    assert s.next_agent_id == 1 and s.cars == [] and s.step_count == 0
    c = cpp_backend.Car()
    assert (c.length, c.width, c.alive, c.intention, c.path_index) == (54.0, 24.0, True, 0, 0)


def test_render_masks_match_reference_geometry():
    """The debug renderer's road and line masks equal the reference's rasters
    (tests/golden/static_lanes*.npz, recorded from RoadGeometry / LineMask)."""
    from marl_traffic_intersection_amd import render
    for L in (2, 3):
        g = np.load(f"{G.GOLDEN_DIR}/static_lanes{L}.npz")["grid"]
        assert np.array_equal(render.road_mask(L), (g & 1).astype(bool))
        assert np.array_equal(render.line_mask(L), (g & 4).astype(bool))


def test_lidars_setter_groups_cars_by_configuration():
    """IntersectionEnv.lidars (cpp/bindings.cpp:68, per-car Lidar objects): one configuration
    for every car keeps one handle; different ones become a per-car configuration (one device
    handle per distinct key when the env is stepped); cars added later get
    add_car_with_route's own 96-ray Lidar; reset() goes back to that default.  Host logic
    only -- no handle is created here."""
    env = cpp_backend.IntersectionEnv(3)
    env.reset()
    for s, e in [("IN_1", "OUT_4"), ("IN_4", "OUT_7"), ("IN_7", "OUT_10")]:
        env.add_car_with_route(s, e)
    env.lidars = [cpp_backend.Lidar(64, 360.0, 250.0, 4.0)] * 3  # one configuration: uniform
    assert env._lidar == (64, 360.0, 250.0, 4.0)
    short = cpp_backend.Lidar()  # 72 offsets, 48 rays: the first 48 offsets are the beams
    short.rays, short.max_dist = 48, 200.0
    env.lidars = [cpp_backend.Lidar(96), short, cpp_backend.Lidar(128, 270.0)]
    kind, keys = env._lidar
    assert kind == "per_car" and len(keys) == 3
    assert keys[0] == cpp_backend._default_key((96, 360.0, 250.0, 4.0))
    assert keys[1][0] == 48 and len(keys[1][4]) == 72 and keys[1][2] == 200.0
    assert keys[1][4][:48] == tuple(np.asarray(cpp_backend._rel_angles(72, 360.0), np.float32).tolist())[:48]
    env.add_car_with_route("IN_10", "OUT_1")  # a new car: its own 96-ray Lidar
    assert len(env._lidar[1]) == 4 and env._lidar[1][3] == cpp_backend._default_key(cpp_backend.DEFAULT_LIDAR)
    with pytest.raises(ValueError, match="one per car"):
        env.lidars = [short, cpp_backend.Lidar(96)]  # two configurations for four cars
    bad = cpp_backend.Lidar()
    bad.rays = 100  # more rays than offsets: the reference would read past rel_angles
    with pytest.raises(ValueError, match="rel_angles"):
        env.lidars = [bad] * 4
    env.reset()
    assert env._lidar == cpp_backend.DEFAULT_LIDAR
