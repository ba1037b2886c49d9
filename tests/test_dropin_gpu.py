"""The drop-in APIs on the GPU: env.py's IntersectionEnv and cpp_backend's
MARLEnv-equivalent replay reference recordings (tests/golden) bit for bit;
VecIntersectionEnv (torch and numpy) replays them across many envs at once."""
import numpy as np
import pytest

import golden_replay as G
import pkgload

pytestmark = pytest.mark.gpu

M = pkgload.load()
from marl_traffic_intersection_amd import cpp_backend, env as env_mod, vec_env  # noqa: E402

STATUS = ("ALIVE", "DEAD", "SUCCESS", "CRASH_WALL", "CRASH_LINE", "CRASH_CAR")


def _check_step(tag, g, t, obs, rew, term, trunc, info):
    assert G.bits_equal(np.asarray(obs, np.float32), g["obs"][t]), f"{tag} step {t + 1}: obs"
    assert G.bits_equal(np.asarray(rew, np.float32), g["rew"][t]), f"{tag} step {t + 1}: rewards"
    f = g["flags"][t]
    assert (int(term), int(trunc), info["agents_alive"], info["step"]) == tuple(int(x) for x in f), tag
    assert info["status"] == [STATUS[s] for s in g["status"][t]], tag
    assert info["done"] == [int(d) for d in g["done"][t]], tag


@pytest.mark.parametrize("name", ["n12_r96_policy", "n16_r96_ties"])
def test_env_py_replays_reference(name):
    g = G.load(name)
    meta = g["meta"]
    e = env_mod.IntersectionEnv({"num_agents": meta["n_agents"], "num_lanes": meta["num_lanes"],
                                 "use_team_reward": meta["use_team"], "respawn_enabled": meta["respawn"],
                                 "max_steps": meta["max_steps"]})
    obs, info = e.reset()
    assert info == {} and obs.shape == (meta["n_agents"], 127)
    assert G.bits_equal(obs, g["init_obs"])
    for t in range(len(g["actions"])):
        obs, rew, term, trunc, info = e.step(g["actions"][t])
        _check_step(name, g, t, obs, rew, term, trunc, info)
        assert sorted(info["collisions"]) == list(range(1, meta["n_agents"] + 1))
    # cars view == recorded state
    cars = e.env.cars
    for i, c in enumerate(cars):
        assert np.float32(c.state.x) == g["ego_f"][-1, i, 0] and c.path_index == g["ego_i"][-1, i, 2]
    e.close()


def test_env_py_reset_restarts_episode():
    g = G.load("n12_r96_policy")
    e = env_mod.IntersectionEnv({"num_agents": 12})
    for t in range(20):
        e.step(g["actions"][t])
    obs, _ = e.reset()
    assert G.bits_equal(obs, g["init_obs"])
    obs, rew, term, trunc, info = e.step(g["actions"][0])
    _check_step("after reset", g, 0, obs, rew, term, trunc, info)
    e.close()


def test_env_py_custom_reward_and_dt():
    g = G.load("dt_1_30_custom_reward")
    meta = g["meta"]
    keys = ["progress_scale", "stuck_speed_threshold", "stuck_penalty", "crash_vehicle_penalty",
            "crash_object_penalty", "success_reward", "action_smoothness_scale", "team_alpha"]
    e = env_mod.IntersectionEnv({"num_agents": meta["n_agents"], "num_lanes": meta["num_lanes"],
                                 "use_team_reward": meta["use_team"], "ego_routes": meta["ego_routes"],
                                 "reward_config": dict(zip(keys, meta["reward"]))})
    e.env.lidars = [cpp_backend.Lidar(meta["rays"])] * meta["n_agents"]
    obs, _ = e.reset()
    e.env.lidars = [cpp_backend.Lidar(meta["rays"])] * meta["n_agents"]
    obs = e.env.get_observations()
    assert G.bits_equal(obs, g["init_obs"])
    for t in range(len(g["actions"])):
        obs, rew, term, trunc, info = e.step(g["actions"][t], dt=meta["dt"])
        _check_step("custom", g, t, obs, rew, term, trunc, info)
    e.close()


@pytest.mark.parametrize("name", ["cfg2_r64_route03", "lanes2_policy", "cfg3_team_policy"])
def test_cpp_backend_replays_reference(name):
    """MARLEnv-style use: reset, add_car_with_route, per-car Lidar objects, step(throttles, steerings)."""
    g = G.load(name)
    meta = g["meta"]
    env = cpp_backend.IntersectionEnv(meta["num_lanes"])
    env.configure(meta["use_team"], meta["respawn"], meta["max_steps"])
    env.reset()
    for s, t in meta["ego_routes"]:
        env.add_car_with_route(s, t)
    env.lidars = [cpp_backend.Lidar(meta["rays"]) for _ in meta["ego_routes"]]
    assert G.bits_equal(env.get_observations(), g["init_obs"])
    for t in range(len(g["actions"])):
        a = g["actions"][t]
        res = env.step(a[:, 0].tolist(), a[:, 1].tolist(), meta["dt"])
        info = dict(agents_alive=res.agents_alive, step=res.step, status=res.status, done=res.done)
        _check_step(name, g, t, res.obs, res.rewards, res.terminated, res.truncated, info)
        assert res.agent_ids == list(range(1, len(meta["ego_routes"]) + 1))
    lid = env.lidars
    obs = env.get_observations()
    assert np.array_equal(np.float32(lid[0].normalized()), obs[0, 31:31 + meta["rays"]])
    env.close()


def test_cpp_backend_unknown_lanes():
    env = cpp_backend.IntersectionEnv(3)
    env.reset()
    env.add_car_with_route("IN_99", "OUT_1")  # unknown start: ignored (IntersectionEnv.cpp:80-82)
    with pytest.raises(IndexError):
        env.add_car_with_route("IN_1", "OUT_99")
    env.add_car_with_route("IN_1", "OUT_4")
    assert len(env.cars) == 1 and env.get_observations().shape == (1, 127)
    env.close()


def test_cpp_backend_state_roundtrip():
    """get_state/set_state: dynamics continue exactly; LiDAR switches to the
    72-ray Lidar() defaults like the reference (IntersectionEnv.cpp:406-416)."""
    g = G.load("n12_r96_policy")
    env = cpp_backend.IntersectionEnv(3)
    env.reset()
    for s, t in g["meta"]["ego_routes"]:
        env.add_car_with_route(s, t)
    for t in range(40):
        a = g["actions"][t]
        env.step(a[:, 0], a[:, 1])
    snap = env.get_state()
    assert snap.step_count == 40 and len(snap.cars) == 12 and snap.next_agent_id == 13
    other = cpp_backend.IntersectionEnv(3)
    other.set_state(snap)
    obs = other.get_observations()
    assert (obs[:, 31 + 72:] == 0).all() and (obs[:, 31:31 + 72] == 1.0).all()
    assert other.lidars[0].rays == 72
    for t in range(40, 100):
        a = g["actions"][t]
        r1 = env.step(a[:, 0], a[:, 1])
        r2 = other.step(a[:, 0], a[:, 1])
        assert r1.status == r2.status and r1.step == r2.step
        assert G.bits_equal(r1.obs[:, :31], r2.obs[:, :31])
    c1, c2 = env.cars, other.cars
    for a_, b_ in zip(c1, c2):
        assert (a_.state.x, a_.state.y, a_.state.heading, a_.path_index) == (b_.state.x, b_.state.y,
                                                                             b_.state.heading, b_.path_index)
    env.close()
    other.close()


def test_cpp_backend_add_car_mid_episode_keeps_state():
    g = G.load("n12_r96_policy")
    env = cpp_backend.IntersectionEnv(3)
    env.reset()
    for s, t in g["meta"]["ego_routes"][:4]:
        env.add_car_with_route(s, t)
    for t in range(30):
        env.step(g["actions"][t, :4, 0], g["actions"][t, :4, 1])
    before = env.cars
    env.add_car_with_route("IN_5", "OUT_11")
    after = env.cars
    assert len(after) == 5 and env.step_count == 30
    for a_, b_ in zip(before, after[:4]):
        assert (a_.state.x, a_.state.v, a_.path_index) == (b_.state.x, b_.state.v, b_.path_index)
    assert (after[4].state.x, after[4].state.y) == (after[4].spawn_state.x, after[4].spawn_state.y)
    env.close()


def test_env_py_traffic_mode():
    e = env_mod.IntersectionEnv({"traffic_flow": True, "traffic_density": 5.0, "num_agents": 4})
    obs, info = e.reset()
    assert e.num_agents == 1 and obs.shape == (127,)
    seen = 0
    for t in range(600):
        obs, rew, term, trunc, info = e.step([0.3, 0.0])
        assert obs.shape == (127,) and isinstance(rew, float) and isinstance(info["rewards"], float)
        seen = max(seen, len(e.traffic_cars))
        if term or trunc:
            e.reset()
    assert seen > 0
    e.close()


@pytest.mark.parametrize("backend", ["torch", "numpy"])
def test_vec_env_replays_reference_in_every_env(backend):
    import torch
    g = G.load("n12_r96_policy")
    E = 96
    v = vec_env.VecIntersectionEnv(E, num_agents=12, lidar_rays=96, backend=backend, auto_reset=True)
    obs = v.reset()
    obs = obs.cpu().numpy() if backend == "torch" else obs
    for e in (0, E - 1):
        assert G.bits_equal(obs[e], g["init_obs"])
    for t in range(len(g["actions"])):
        a = np.broadcast_to(g["actions"][t], (E, 12, 2)).copy()
        if backend == "torch":
            a = torch.from_numpy(a).cuda()
        obs, rew, term, trunc, info = v.step(a)
        if backend == "torch":
            obs, rew, term = obs.cpu().numpy(), rew.cpu().numpy(), term.cpu().numpy()
        if t % 50 == 49 or t == 0:
            assert all(G.bits_equal(obs[e], g["obs"][t]) for e in range(E)), t
            assert all(G.bits_equal(rew[e], g["rew"][t]) for e in range(E)), t
    v.close()


def test_rgb_array_render():
    from marl_traffic_intersection_amd import render
    e = env_mod.IntersectionEnv({"num_agents": 4, "render_mode": "rgb_array", "show_lidar": True})
    for _ in range(5):
        e.step(np.zeros((4, 2), np.float32))
    frame = e.render()
    assert frame.shape == (750, 750, 3) and frame.dtype == np.uint8
    for i in range(4):  # four 54x24 cars, coloured by agent index (Renderer.cpp:597-599)
        col = np.array(render._rgba8(render.AGENT_COLORS[i])[:3], np.uint8)
        assert (frame == col).all(-1).sum() > 300, i  # (semi-transparent hit rays are drawn over the cars)
    assert (frame == np.array(render.HIT, np.uint8)).all(-1).any()
    e.close()


@pytest.mark.parametrize("name", ["set_state_72_team", "set_state_72_n3"])
def test_cpp_backend_set_state_replays_reference(name):
    """The reference's set_state path (IntersectionEnv.cpp:404-416): a state taken
    from a running env, set into a fresh one, then stepped -- every LiDAR is then a
    default Lidar() of 72 rays (Lidar.h:11, Lidar.cpp:4-14).  Golden recorded from
    the reference itself (tests/golden/gen_golden.py gen_set_state): the full
    obs[127] (72 beams + 24 zeros), rewards, status and flags, bit for bit."""
    g = G.load(name)
    meta = g["meta"]
    assert meta["set_state"] and meta["rays"] == 72
    src = cpp_backend.IntersectionEnv(meta["num_lanes"])
    src.reset()
    for s, t in meta["ego_routes"]:
        src.add_car_with_route(s, t)
    snap = src.get_state()  # cars that carry their routes; the golden state goes into them
    f, i = g["init_ego_f"], g["init_ego_i"]
    for k, c in enumerate(snap.cars):
        v = [float(x) for x in f[k]]
        c.state.x, c.state.y, c.state.v, c.state.heading, c.acc, c.steering_angle = v[0:6]
        c.spawn_state.x, c.spawn_state.y, c.spawn_state.v, c.spawn_state.heading = v[6:10]
        c.prev_dist_to_goal, c.prev_action = v[10], (v[11], v[12])
        c.alive, c.intention, c.path_index = bool(i[k, 0]), int(i[k, 1]), int(i[k, 2])
    snap.step_count = int(meta["init_step"])
    src.close()
    env = cpp_backend.IntersectionEnv(meta["num_lanes"])
    env.configure(meta["use_team"], meta["respawn"], meta["max_steps"])
    env.set_state(snap)
    assert env.lidars[0].rays == 72
    assert G.bits_equal(env.get_observations(), g["init_obs"])  # 72 x 1.0, then zeros
    for t in range(len(g["actions"])):
        a = g["actions"][t]
        res = env.step(a[:, 0].tolist(), a[:, 1].tolist(), meta["dt"])
        info = dict(agents_alive=res.agents_alive, step=res.step, status=res.status, done=res.done)
        _check_step(name, g, t, res.obs, res.rewards, res.terminated, res.truncated, info)
    env.close()


def test_cpp_backend_cars_setter_and_written_path():
    """IntersectionEnv.cars / traffic_cars are read-write and Car.path is a plain
    read-write vector in the reference (cpp/bindings.cpp:29,66-67): writing the cars
    back unchanged leaves the run bit-identical to an untouched twin; a bent
    160-point path becomes a route of the env's own (mev_add_route), is read back
    as written, survives get_state/set_state into a fresh env and steers the car
    (its route-following features differ from the twin's from then on)."""
    g = G.load("n12_r96_policy")
    envs = [cpp_backend.IntersectionEnv(3) for _ in range(3)]
    for env in envs:
        env.reset()
        for s, t in g["meta"]["ego_routes"][:3]:
            env.add_car_with_route(s, t)
        for t in range(10):
            env.step(g["actions"][t, :3, 0], g["actions"][t, :3, 1])
    same, bent, twin = envs
    same.cars = same.cars  # written back unchanged
    cars = bent.cars
    p = np.asarray(cars[1].path, np.float64)
    d = np.gradient(p, axis=0)
    nrm = np.stack([-d[:, 1], d[:, 0]], 1) / np.maximum(np.hypot(d[:, 0], d[:, 1]), 1e-9)[:, None]
    new_path = (p + nrm * (8.0 * np.sin(np.pi * np.arange(len(p)) / (len(p) - 1)))[:, None]).astype(np.float32)
    cars[1].path = [tuple(map(float, q)) for q in new_path]
    bent.cars = cars
    assert G.bits_equal(np.asarray(bent.cars[1].path, np.float32), new_path)
    assert bent.cars[0].path == twin.cars[0].path
    differs = False
    for t in range(10, 60):
        a = g["actions"][t, :3]
        r0, r1, r2 = (e.step(a[:, 0], a[:, 1]) for e in (same, bent, twin))
        assert G.bits_equal(r0.obs, r2.obs) and G.bits_equal(r0.rewards, r2.rewards), t
        differs |= not G.bits_equal(r1.obs[1], r2.obs[1])
    assert differs
    snap = bent.get_state()
    other = cpp_backend.IntersectionEnv(3)
    other.set_state(snap)
    assert G.bits_equal(np.asarray(other.cars[1].path, np.float32), new_path)
    c0 = other.cars[0].path
    for bad in (c0[:1], c0 * 26):  # 1 and 4160 points (2 .. 4096 are taken)
        with pytest.raises(ValueError):
            c = other.cars
            c[0].path = bad
            other.cars = c
    for env in envs + [other]:
        env.close()


@pytest.mark.parametrize("name", ["dims_cfg3_policy", "dims_respawn_off", "path_bent_egos", "path_short_egos",
                                  "path_long_egos"])
def test_cpp_backend_written_cars_replay_reference(name):
    """MARLEnv-style writes through the read-write cars vector (cpp/bindings.cpp:24-25,29,66):
    Car.length / Car.width and Car.path set on the cars add_car_with_route made, then the
    recorded steps -- every output bit-exact against the reference, which recorded the same
    writes (tests/golden/gen_golden.py gen_dims / gen_paths)."""
    g = G.load(name)
    meta = g["meta"]
    env = cpp_backend.IntersectionEnv(meta["num_lanes"])
    env.configure(meta["use_team"], meta["respawn"], meta["max_steps"])
    env.reset()
    for s, t in meta["ego_routes"]:
        env.add_car_with_route(s, t)
    env.lidars = [cpp_backend.Lidar(meta["rays"]) for _ in meta["ego_routes"]]
    cars = env.cars
    f = g["init_ego_f"]
    eps = meta.get("ego_paths") or [-1] * len(cars)
    for k, c in enumerate(cars):
        c.length, c.width = float(f[k, 13]), float(f[k, 14])
        if eps[k] >= 0:
            c.path = [tuple(map(float, q)) for q in G.custom_paths(g)[eps[k]]]
    env.cars = cars
    back = env.cars
    assert [(c.length, c.width) for c in back] == [(float(x), float(y)) for x, y in f[:, 13:15]]
    assert G.bits_equal(env.get_observations(), g["init_obs"])
    for t in range(len(g["actions"])):
        a = g["actions"][t]
        res = env.step(a[:, 0].tolist(), a[:, 1].tolist(), meta["dt"])
        info = dict(agents_alive=res.agents_alive, step=res.step, status=res.status, done=res.done)
        _check_step(name, g, t, res.obs, res.rewards, res.terminated, res.truncated, info)
    # the sizes survive get_state / set_state into a fresh env (EnvState copies the Cars)
    other = cpp_backend.IntersectionEnv(meta["num_lanes"])
    other.set_state(env.get_state())
    assert [(c.length, c.width) for c in other.cars] == [(c.length, c.width) for c in env.cars]
    env.close()
    other.close()


@pytest.mark.parametrize("name", ["path_past_end_npc", "path_long_npc"])
def test_cpp_backend_written_traffic_cars_replay_reference(name):
    """NPCs written through the read-write traffic_cars vector (cpp/bindings.cpp:29-30,67) with
    Car.path set to paths of the caller's own: cuts of traffic routes with path_index past the
    cut's end (the reference's ghost scan is then empty, TrafficFlow.cpp:88-89) and paths of
    200-480 points -- every recorded output bit-exact against the reference (gen_golden.py
    gen_paths_past_end / gen_paths_long)."""
    g = G.load(name)
    meta = g["meta"]
    L = meta["num_lanes"]
    P = 8 * L
    env = cpp_backend.IntersectionEnv(L)
    env.configure(meta["use_team"], meta["respawn"], meta["max_steps"])
    env.configure_traffic(meta["traffic"], meta["density"])
    env.configure_routes([tuple(r) for r in meta["traffic_routes"]])
    env.reset()
    for s, t in meta["ego_routes"]:
        env.add_car_with_route(s, t)
    env.lidars = [cpp_backend.Lidar(meta["rays"]) for _ in meta["ego_routes"]]
    cps = G.custom_paths(g)
    cars = env.cars
    for k, c in enumerate(cars):
        if meta["ego_paths"][k] >= 0:
            c.path = [tuple(map(float, q)) for q in cps[meta["ego_paths"][k]]]
    env.cars = cars
    npcs = []
    for f, i in zip(g["init_npc_f"], g["init_npc_i"]):
        c = cpp_backend.Car()
        c.state = cpp_backend.State(*map(float, f[:4]))
        c.acc, c.steering_angle = float(f[4]), float(f[5])
        c.alive, c.intention, c.path_index = bool(i[0]), int(i[1]), int(i[2])
        if int(i[3]) >= 1000:
            c.path = [tuple(map(float, q)) for q in cps[int(i[3]) - 1000]]
        else:
            s, t = meta["traffic_routes"][int(i[3])]
            c._route = G.point_index(s, L) * P + G.point_index(t, L)
        npcs.append(c)
    env.traffic_cars = npcs
    past = [c.path_index >= len(c.path) for c in env.traffic_cars if len(c.path)]
    if name == "path_past_end_npc":
        assert sum(past) >= 3, past
    assert G.bits_equal(env.get_observations()[:, :31], g["init_obs"][:, :31])
    for t in range(len(g["actions"])):
        a = g["actions"][t]
        res = env.step(a[:, 0].tolist(), a[:, 1].tolist(), meta["dt"])
        info = dict(agents_alive=res.agents_alive, step=res.step, status=res.status, done=res.done)
        _check_step(name, g, t, res.obs, res.rewards, res.terminated, res.truncated, info)
    env.close()


def test_cpp_backend_traffic_without_egos_replays_reference():
    """An env with traffic and no egos (reset, traffic_cars written, no add_car_with_route): step()
    counts, truncates and runs the traffic (IntersectionEnv.cpp:133-142) -- the step flags and every
    NPC's state bit-exact against the reference (gen_golden.py gen_no_ego); then egos added to the
    running episode find the NPCs and the step count where the steps left them."""
    g = G.load("traffic_no_ego")
    meta = g["meta"]
    L = meta["num_lanes"]
    P = 8 * L
    env = cpp_backend.IntersectionEnv(L)
    env.configure(meta["use_team"], meta["respawn"], meta["max_steps"])
    env.configure_traffic(meta["traffic"], meta["density"])
    env.configure_routes([tuple(r) for r in meta["traffic_routes"]])
    env.reset()
    npcs = []
    for f, i in zip(g["init_npc_f"], g["init_npc_i"]):
        c = cpp_backend.Car()
        c.state = cpp_backend.State(*map(float, f[:4]))
        c.acc, c.steering_angle = float(f[4]), float(f[5])
        c.alive, c.intention, c.path_index = bool(i[0]), int(i[1]), int(i[2])
        s, t = meta["traffic_routes"][int(i[3])]
        c._route = G.point_index(s, L) * P + G.point_index(t, L)
        npcs.append(c)
    env.traffic_cars = npcs
    assert env.cars == [] and env.get_observations().shape == (0, 127) and len(env.traffic_cars) == len(npcs)
    for t in range(len(g["actions"])):
        res = env.step([], [], meta["dt"])
        f = g["flags"][t]
        assert (int(res.terminated), int(res.truncated), res.agents_alive, res.step) == tuple(int(x) for x in f), t
        assert res.obs.shape == (0, 127) and len(res.rewards) == 0 and res.status == [] and res.agent_ids == []
        tc = env.traffic_cars
        k = int(g["npc_count"][t])
        assert len(tc) == k, (t, len(tc), k)
        got = np.array([[c.state.x, c.state.y, c.state.v, c.state.heading, c.acc, c.steering_angle] for c in tc],
                       np.float32).reshape(k, 6)
        assert G.bits_equal(got, g["npc_f"][t, :k, :6]), t
        assert [c.path_index for c in tc] == g["npc_i"][t, :k, 2].tolist(), t
        if t == 40:
            snap = env.get_state()
    assert env.step_count == len(g["actions"])
    # egos join the running episode: NPCs and the step count carry over (add_car_with_route, :78-131)
    other = cpp_backend.IntersectionEnv(L)
    other.configure(meta["use_team"], meta["respawn"], meta["max_steps"])
    other.configure_traffic(meta["traffic"], meta["density"])
    other.configure_routes([tuple(r) for r in meta["traffic_routes"]])
    other.set_state(snap)
    assert other.cars == [] and other.step_count == 41 and len(other.traffic_cars) == int(g["npc_count"][40])
    other.add_car_with_route("IN_1", "OUT_4")
    assert len(other.cars) == 1 and other.step_count == 41
    assert [(c.state.x, c.path_index) for c in other.traffic_cars] == [(c.state.x, c.path_index) for c in snap.traffic_cars]
    res = other.step([0.5], [0.0], meta["dt"])
    assert res.step == 42 and len(res.rewards) == 1 and res.obs.shape == (1, 127)
    env.reset()  # the no-ego handle starts over: no traffic, step 0
    assert env.traffic_cars == [] and env.step_count == 0
    assert env.step([], []).step == 1
    env.close()
    other.close()


@pytest.mark.parametrize("name", ["lidar_mixed_n4", "lidar_mixed_npc"])
def test_cpp_backend_per_car_lidars_replay_reference(name):
    """Per-car LiDAR objects written through IntersectionEnv.lidars (cpp/bindings.cpp:68,85-92):
    Lidar() as constructed (72 rays), Lidar() with fewer rays than its offsets, a 128-ray
    270-degree fan with its offsets written, a short-range 32-ray Lidar among NPCs -- every
    recorded output bit-exact against the reference (gen_golden.py gen_lidars), one device
    handle per configuration behind the drop-in.  Before the first step only the heads are
    compared: the reference's LiDAR block then shows the written Lidar's own distances."""
    g = G.load(name)
    meta = g["meta"]
    L = meta["num_lanes"]
    env = cpp_backend.IntersectionEnv(L)
    env.configure(meta["use_team"], meta["respawn"], meta["max_steps"])
    env.configure_traffic(meta["traffic"], meta["density"])
    env.configure_routes([tuple(r) for r in meta["traffic_routes"]])
    env.reset()
    for s, t in meta["ego_routes"]:
        env.add_car_with_route(s, t)
    lids = []
    for k, cl in enumerate(meta["car_lidars"]):
        if not cl:
            lids.append(cpp_backend.Lidar(96))  # add_car_with_route's own
            continue
        rays, fov, maxd, stp, nrel = cl
        l_ = cpp_backend.Lidar()  # 72 rays, members written as a MARLEnv user would
        l_.rays, l_.fov_deg, l_.max_dist, l_.step_size = rays, fov, maxd, stp
        if nrel >= 0:
            l_.rel_angles = g["car_rel"][k, :nrel].tolist()
        lids.append(l_)
    env.lidars = lids
    if len(g["init_npc_f"]):
        P = 8 * L
        npcs = []
        for f, i in zip(g["init_npc_f"], g["init_npc_i"]):
            c = cpp_backend.Car()
            c.state = cpp_backend.State(*map(float, f[:4]))
            c.acc, c.steering_angle = float(f[4]), float(f[5])
            c.length, c.width = float(f[13]), float(f[14])
            c.alive, c.intention, c.path_index = bool(i[0]), int(i[1]), int(i[2])
            s, t = meta["traffic_routes"][int(i[3])]
            c._route = G.point_index(s, L) * P + G.point_index(t, L)  # (its lane route: Car.path left empty)
            npcs.append(c)
        env.traffic_cars = npcs
    assert G.bits_equal(env.get_observations()[:, :31], g["init_obs"][:, :31])
    got = env.lidars
    assert [(l_.rays, l_.max_dist, l_.step_size) for l_ in got] == [(l_.rays, l_.max_dist, l_.step_size) for l_ in lids]
    for t in range(len(g["actions"])):
        a = g["actions"][t]
        res = env.step(a[:, 0].tolist(), a[:, 1].tolist(), meta["dt"])
        info = dict(agents_alive=res.agents_alive, step=res.step, status=res.status, done=res.done)
        _check_step(name, g, t, res.obs, res.rewards, res.terminated, res.truncated, info)
    # the Lidars read back carry the reference's distances of the last step
    last = g["obs"][-1]
    for k, l_ in enumerate(env.lidars):
        if last[k].any():  # (a dead car's row is zero)
            n_ = min(l_.rays, 96)
            assert G.bits_equal(np.asarray(l_.normalized(), np.float32)[:n_], last[k, 31:31 + n_]), k
    env.close()
