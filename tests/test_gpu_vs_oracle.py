"""Device path vs the C restatement (oracle/marl_oracle.c, itself pinned to the
reference by tests/test_oracle.py) on randomized inputs the golden set does not
cover: random poses/speeds/controls/path indices for every ego, random NPC
fleets placed on their routes, random (partly unclipped) actions and random
spawn decisions, many envs per handle.  Bit-exact on every output and on the
full state after every step."""
import zlib

import numpy as np
import pytest

import golden_replay as G
from conftest import STEP_KERNELS, use_step_kernel
import oracle_replay as R

pytestmark = pytest.mark.gpu

ROUTES3 = [(1, 4), (2, 8), (3, 12), (4, 7), (5, 11), (6, 3), (7, 10), (8, 2), (9, 6), (10, 1), (11, 5), (12, 9)]
ROUTES2 = [(1, 3), (2, 6), (3, 5), (4, 8), (6, 2), (7, 1), (8, 4)]

CONFIGS = [
    dict(name="n8_r64_team", n=8, rays=64, use_team=True),
    dict(name="n1_r64", n=1, rays=64),
    dict(name="n3_r16_norespawn", n=3, rays=16, respawn=False, max_steps=40),
    dict(name="n12_r96_obs127", n=12, rays=96),
    dict(name="n8_r128", n=8, rays=128, use_team=True),
    dict(name="lanes2_n7", n=7, rays=64, lanes=2),
    dict(name="n5_r33_custom", n=5, rays=33, reward=[3.0, 0.5, -0.1, -2.0, -1.0, 4.0, -0.3, 0.7], dt=1 / 30),
    dict(name="traffic_n1", n=1, rays=64, traffic=True, density=0.5, spawn_p=0.15, npcs=6),
    dict(name="traffic_n3", n=3, rays=48, traffic=True, density=2.0, spawn_p=0.3, npcs=9),
    # dense fleets: the NPC controller's parallel rounds disagree now and then, so its
    # sequential fallback runs (npc_stats) and is checked here as well
    dict(name="traffic_dense", n=2, rays=32, traffic=True, density=5.0, spawn_p=0.6, npcs=24, npc_gap=30.0,
         expect_seq=True),
    # routes of the caller's own (a written Car.path, cpp/bindings.cpp:29 -> mev_add_route) beside lane routes,
    # for egos and NPCs (NPCs spawn on them too: their first point)
    dict(name="custom_routes_n6", n=6, rays=64, custom=True),
    dict(name="custom_routes_traffic", n=3, rays=48, traffic=True, density=1.0, spawn_p=0.3, npcs=8, custom=True),
    # written paths of fewer than 160 points (mev_add_route_n: rows padded with the last point, the SUCCESS
    # axis from the path's own last segment); egos may sit at path_index past their path's end
    dict(name="short_routes_n6", n=6, rays=64, use_team=True, custom="short"),
    dict(name="short_routes_traffic", n=1, rays=64, traffic=True, density=1.0, spawn_p=0.3, npcs=8, custom="short"),
    # written paths of more than 160 points (the table's rows re-laid out at the longest, rounded up to 16), and
    # NPCs whose path_index lies past their path's end (the reference's ghost scan is then empty)
    dict(name="long_routes_n6", n=6, rays=64, use_team=True, custom="long"),
    dict(name="long_routes_traffic", n=1, rays=64, traffic=True, density=1.0, spawn_p=0.3, npcs=8, custom="long"),
    dict(name="past_end_traffic", n=2, rays=48, traffic=True, density=1.0, spawn_p=0.3, npcs=10, custom="short",
         past=0.4),
    # per-car sizes (Car::length / Car::width, cpp/Car.h:19-20; mev_set_car_dims): egos and injected NPCs of
    # random sizes, spawned NPCs of the default one; the runtime-layout kernels run these handles
    dict(name="dims_n8_r64_team", n=8, rays=64, use_team=True, dims=True),
    dict(name="dims_n2_r16", n=2, rays=16, dims=True),
    dict(name="dims_traffic_n3", n=3, rays=48, traffic=True, density=2.0, spawn_p=0.3, npcs=9, dims=True),
    dict(name="dims_traffic_n1", n=1, rays=64, traffic=True, density=0.5, spawn_p=0.2, npcs=12, npc_gap=45.0,
         dims=True),
    # more than 16 neighbour candidates with exact distance ties (std::sort's order, IntersectionEnv.cpp:490):
    # every car on a 30-px lattice of the road cross, half the egos parked (v = 0, zero throttle every step:
    # they stay on their lattice points), so equal squared distances recur at every step
    dict(name="n24_lattice_ties", n=24, rays=64, use_team=True, lattice=30, frozen=0.5),
    dict(name="n40_lattice_ties", n=40, rays=32, lattice=30, frozen=0.6),
    dict(name="traffic_lattice_ties", n=3, rays=48, traffic=True, density=1.0, spawn_p=0.3, npcs=24, lattice=30,
         frozen=0.7),
    # written Lidar.rel_angles (cpp/bindings.cpp:91) that the LiDAR's per-box beam culling cannot model
    # (SimParams::beam_cull = 0: every beam against every candidate box): a reversed fan, uneven offsets,
    # a fan over three revolutions, one repeated angle
    dict(name="rel_reversed_n8", n=8, rays=32, rel="reversed"),
    dict(name="rel_uneven_n8", n=8, rays=24, use_team=True, rel="uneven"),
    dict(name="rel_wide_n6", n=6, rays=16, rel="wide"),
    dict(name="rel_constant_traffic", n=2, rays=8, traffic=True, density=2.0, spawn_p=0.3, npcs=9, rel="constant"),
]


def rel_list(kind, rays, rng):
    """Beam offsets (radians) of a written Lidar.rel_angles."""
    f32 = np.float32
    fan = np.array([(f32(-180.0) + f32(i) * (f32(360.0) / f32(rays - 1))) * f32(np.pi) / f32(180.0)
                    for i in range(rays)], np.float32)
    if kind == "reversed":
        return fan[::-1].copy()
    if kind == "uneven":
        return np.sort(rng.uniform(-np.pi, np.pi, rays)).astype(np.float32)
    if kind == "wide":
        return np.linspace(-3 * np.pi, 3 * np.pi, rays).astype(np.float32)
    return np.full(rays, 0.3, np.float32)


def lattice_points(rng, lanes, spacing, count):
    """count distinct points of a `spacing`-px lattice centred on the intersection, inside the road cross."""
    rw = 42 * lanes
    ks = np.arange(-(375 // spacing), 375 // spacing + 1)
    pts = [(375.0 + spacing * a, 375.0 + spacing * b) for a in ks for b in ks
           if (abs(spacing * a) < rw or abs(spacing * b) < rw) and 0 < 375 + spacing * a < 750 and 0 < 375 + spacing * b < 750]
    pick = rng.choice(len(pts), size=count, replace=False)
    return [pts[k] for k in pick]


def random_dims(rng, h):
    """Random (length, width) per ego and NPC slot: 12..130 x 8..70 px, some at the default 54 x 24."""
    ego = np.stack([rng.uniform(12, 130, (h.E, h.N)), rng.uniform(8, 70, (h.E, h.N))], -1).astype(np.float32)
    npc = np.stack([rng.uniform(12, 130, (h.E, h.K)), rng.uniform(8, 70, (h.E, h.K))], -1).astype(np.float32)
    ego[rng.uniform(size=(h.E, h.N)) < 0.25] = (54.0, 24.0)
    return ego, npc


def resample(p, n):
    """Polyline p at n points, uniform in the point index (linear interpolation in f64)."""
    p = np.asarray(p, np.float64)
    t = np.linspace(0.0, len(p) - 1.0, n)
    i0 = np.minimum(np.floor(t).astype(int), len(p) - 2)
    w = (t - i0)[:, None]
    return (p[i0] * (1.0 - w) + p[i0 + 1] * w).astype(np.float32)


def custom_routes(h, kind=True):
    """Four 160-point routes that no lane pair generates: three lane routes bent sideways by up to 9 px
    (a sine bump along the route's normal) and one straight diagonal across the whole intersection.
    "short": cut to 100, 40, 2 (the first point and point 60) and 75 points; "long": resampled at
    240, 500, 1000 and 333 points."""
    short = kind == "short"
    out = []
    for s, t, amp in ((1, 4, 9.0), (3, 12, -6.0), (7, 10, 5.0)):
        path, intent, _ = h.route_info(h.route_id(s - 1, 12 + t - 1))
        d = np.gradient(path.astype(np.float64), axis=0)
        nrm = np.stack([-d[:, 1], d[:, 0]], 1) / np.maximum(np.hypot(d[:, 0], d[:, 1]), 1e-9)[:, None]
        bump = amp * np.sin(np.pi * np.arange(160) / 159.0)
        out.append(((path + nrm * bump[:, None]).astype(np.float32), int(intent)))
    diag = np.stack([np.linspace(120.0, 640.0, 160), np.linspace(610.0, 140.0, 160)], 1).astype(np.float32)
    out.append((diag, 1))
    if short:
        out = [(out[0][0][:100], out[0][1]), (out[1][0][:40], out[1][1]),
               (out[2][0][[0, 60]], out[2][1]), (out[3][0][:75], out[3][1])]
    if kind == "long":
        out = [(resample(p_, m), it) for (p_, it), m in zip(out, (240, 500, 1000, 333))]
    return out


def _place_index(rng, n):
    """A path point to place a car at: the first 150 of a path of <= 160 points, anywhere on a longer one."""
    return int(rng.integers(0, n - 1 if n > 160 else min(150, n - 1)))


def _random_state(rng, h, n, npcs, lanes, routes_table, gap=60.0, extra=(), lattice=0, frozen=None, past=0.0):
    E = h.E
    st = h.get_state()
    ids = [h.route_id(s - 1, 4 * lanes + t - 1) for s, t in routes_table] + list(extra)
    nr = len(ids)
    ego_routes = np.zeros((E, n), np.int32)
    for e in range(E):
        for i in range(n):
            ego_routes[e, i] = ids[rng.integers(0, nr)]
    h.set_ego_routes(ego_routes)
    st["route"][:] = ego_routes
    rw = 42 * lanes
    for e in range(E):
        for i in range(n):
            path, intent, spawn = h.route_info(int(ego_routes[e, i]))
            if rng.uniform() < 0.7:  # near its route
                j = _place_index(rng, h.route_len(int(ego_routes[e, i])))
                x, y = path[j] + rng.normal(0, 4, 2)
                hd = np.arctan2(-(path[j + 1, 1] - path[j, 1]), path[j + 1, 0] - path[j, 0]) + rng.normal(0, 0.2)
                pidx = max(0, j - int(rng.integers(0, 5)))
            else:  # anywhere in the cross
                x, y = rng.uniform(375 - rw, 375 + rw), rng.uniform(0, 750)
                if rng.uniform() < 0.5:
                    x, y = y, x
                hd = rng.uniform(-np.pi, np.pi)
                pidx = int(rng.integers(0, 150))
            st["x"][e, i], st["y"][e, i] = x, y
            st["heading"][e, i] = hd
            st["v"][e, i] = rng.uniform(0, 8)
            st["acc"][e, i] = rng.uniform(-15, 15)
            st["steering"][e, i] = rng.uniform(-0.6, 0.6)
            st["prev_dist"][e, i] = rng.uniform(0, 700) if rng.uniform() < 0.8 else 0.0
            st["prev_a0"][e, i], st["prev_a1"][e, i] = rng.uniform(-1, 1, 2)
            st["spawn_x"][e, i], st["spawn_y"][e, i], st["spawn_heading"][e, i] = spawn
            st["spawn_v"][e, i] = 0.0
            st["path_index"][e, i] = pidx
            st["intention"][e, i] = intent
            st["alive"][e, i] = 0 if rng.uniform() < 0.05 else 1
    troutes = ids
    for e in range(E):
        k = int(rng.integers(0, npcs + 1)) if npcs else 0
        placed = []
        cnt = 0
        for _ in range(k * 10):
            if cnt >= k:
                break
            ri = int(rng.integers(0, len(troutes)))
            path, intent, spawn = h.route_info(troutes[ri])
            j = _place_index(rng, h.route_len(troutes[ri]))
            x, y = path[j]
            if any((x - a) ** 2 + (y - b) ** 2 < gap ** 2 for a, b in placed):
                continue
            placed.append((x, y))
            st["npc_x"][e, cnt], st["npc_y"][e, cnt] = x + rng.normal(0, 1), y + rng.normal(0, 1)
            st["npc_heading"][e, cnt] = np.arctan2(-(path[j + 1, 1] - path[j, 1]), path[j + 1, 0] - path[j, 0])
            st["npc_v"][e, cnt] = rng.uniform(0, 5)
            st["npc_acc"][e, cnt] = 0.0
            st["npc_steering"][e, cnt] = rng.uniform(-0.2, 0.2)
            st["npc_path_index"][e, cnt] = max(0, j - 1)
            if rng.uniform() < past:  # (a written path_index past the path's end)
                st["npc_path_index"][e, cnt] = h.route_len(troutes[ri]) + int(rng.integers(0, 20))
            st["npc_route"][e, cnt] = troutes[ri]
            st["npc_intention"][e, cnt] = intent
            st["npc_alive"][e, cnt] = 1
            cnt += 1
        st["npc_count"][e] = cnt
    if lattice:  # every car of the env on its own lattice point; parked egos stand still
        for e in range(E):
            k = int(st["npc_count"][e])
            pts = lattice_points(rng, lanes, lattice, n + k)
            for i in range(n):
                st["x"][e, i], st["y"][e, i] = pts[i]
                if frozen[e, i]:
                    st["v"][e, i] = 0.0
            for j in range(k):
                st["npc_x"][e, j], st["npc_y"][e, j] = pts[n + j]
    st["step_count"][:] = rng.integers(0, 5, E)
    h.set_state(st)
    return st, troutes


def _oracle_from_state(cfg, st, e, troutes, customs=(), dims=None, rel=None):
    n = cfg["n"]
    meta = dict(rays=cfg["rays"], num_lanes=cfg.get("lanes", 3), n_agents=n, use_team=cfg.get("use_team", False),
                respawn=cfg.get("respawn", True), max_steps=cfg.get("max_steps", 2000),
                traffic=cfg.get("traffic", False), density=cfg.get("density", 0.5),
                reward=cfg.get("reward", [10.0, 1.0, -0.01, -10.0, -5.0, 10.0, -0.02, 0.2]))
    o = R.make_oracle(meta)
    if rel is not None:
        o.set_rel_angles(rel)
    for path, intent in customs:
        o.add_route(path, intent)
    o.set_traffic_routes(troutes)
    cars = R.O.new_cars(n)
    m = {"x": "x", "y": "y", "v": "v", "h": "heading", "acc": "acc", "steer": "steering", "sx": "spawn_x",
         "sy": "spawn_y", "sv": "spawn_v", "sh": "spawn_heading", "prev_dist": "prev_dist", "pa0": "prev_a0",
         "pa1": "prev_a1", "path_index": "path_index", "route": "route", "intention": "intention", "alive": "alive"}
    for a, b in m.items():
        cars[a] = st[b][e]
    k = int(st["npc_count"][e])
    npcs = R.O.new_cars(k)
    mn = {"x": "npc_x", "y": "npc_y", "v": "npc_v", "h": "npc_heading", "acc": "npc_acc", "steer": "npc_steering",
          "path_index": "npc_path_index", "route": "npc_route", "intention": "npc_intention", "alive": "npc_alive"}
    for a, b in mn.items():
        npcs[a] = st[b][e, :k]
    if dims is not None:
        cars["len"], cars["wid"] = dims[0][e, :, 0], dims[0][e, :, 1]
        npcs["len"], npcs["wid"] = dims[1][e, :k, 0], dims[1][e, :k, 1]
    o.set_state(cars, npcs, int(st["step_count"][e]))
    return o


@pytest.mark.parametrize("kernel", STEP_KERNELS)
@pytest.mark.parametrize("cfg", CONFIGS, ids=[c["name"] for c in CONFIGS])
def test_random_states_match_oracle(mev, cfg, kernel):
    _random_states_vs_oracle(mev, cfg, kernel)


PACKED = [c for c in CONFIGS if c["n"] <= 4 and not c.get("traffic") and not c.get("dims")]


@pytest.mark.parametrize("pack", [2, 4, 8])
@pytest.mark.parametrize("cfg", PACKED, ids=[c["name"] for c in PACKED])
def test_random_states_match_oracle_packed_waves(mev, cfg, pack):
    """Several envs per fused k_step wave (mev_set_step_pack), each env from its
    own random state: every output and the state after every step bit-exact."""
    _random_states_vs_oracle(mev, cfg, 2, pack)


@pytest.mark.parametrize("pack", [1, 2, 4])
@pytest.mark.parametrize("cfg", [c for c in CONFIGS if not c.get("traffic") and not c.get("dims")],
                         ids=[c["name"] for c in CONFIGS if not c.get("traffic") and not c.get("dims")])
def test_random_states_match_oracle_early_split(mev, cfg, pack):
    """The early split (mev_set_step_split(3): the LiDAR wave computes the poses
    after Car::update itself and marches the road beside the car part), `pack`
    envs per workgroup, each env from its own random state: every output and the
    state after every step bit-exact against the oracle."""
    if pack > 1 and pack * cfg["n"] > 8:
        pytest.skip("fewer agent slots than the pack: the same run as a smaller pack")
    _random_states_vs_oracle(mev, cfg, 2, pack, split=3)


TRAFFIC_ONE_EGO = [c for c in CONFIGS if c.get("traffic") and c["n"] == 1 and not c.get("dims")]


@pytest.mark.parametrize("cfg", TRAFFIC_ONE_EGO, ids=[c["name"] for c in TRAFFIC_ONE_EGO])
def test_random_states_match_oracle_traffic_early_split(mev, cfg):
    """The traffic early split (mev_set_step_split(3), one ego and <= 32 NPC slots per
    env, E divisible by 16: two car waves -- NPC phase and car part of one env each
    -- and one LiDAR wave for their four egos per workgroup), 32 envs from random
    states: every output and the state after every step bit-exact."""
    _random_states_vs_oracle(mev, cfg, 2, 0, split=3, max_npcs=32, E=32)


def _random_states_vs_oracle(mev, cfg, kernel, pack=0, split=0, max_npcs=64, E=24):
    rng = np.random.default_rng(zlib.crc32(cfg["name"].encode()))
    T = 50
    n, lanes = cfg["n"], cfg.get("lanes", 3)
    R_ = cfg["rays"]
    D = 127 if R_ <= 96 else 31 + R_
    h = mev.Handle(num_envs=E, num_agents=n, num_lanes=lanes, lidar_rays=R_, obs_dim=D,
                   traffic_flow=int(cfg.get("traffic", False)), traffic_density=cfg.get("density", 0.5),
                   use_team_reward=int(cfg.get("use_team", False)), respawn_enabled=int(cfg.get("respawn", True)),
                   max_steps=cfg.get("max_steps", 2000), max_npcs=max_npcs,
                   reward=cfg.get("reward", [10.0, 1.0, -0.01, -10.0, -5.0, 10.0, -0.02, 0.2]))
    use_step_kernel(mev, h, kernel)
    if pack:
        h.set_step_pack(pack)
        assert h.step_pack() == (pack if pack * n <= 8 else max(1, 8 // n)), h.step_pack()
    if split:
        h.set_step_split(split)
        if cfg.get("traffic"):
            assert h.step_split() == 2, "traffic early split not selected"
        elif h.step_split() != 2:  # the early split needs the slots' beams in one 512-beam pool
            assert h.step_pack() * n * R_ > 512, (h.step_pack(), n, R_)
            pytest.skip("beams of the workgroup's slots exceed one LiDAR pool")
    rel = None
    if cfg.get("rel"):
        rel = rel_list(cfg["rel"], R_, rng)
        h.set_beam_angles(rel)
        assert G.bits_equal(h.beam_angles(), rel)
    table = ROUTES2 if lanes == 2 else ROUTES3
    customs = custom_routes(h, cfg["custom"]) if cfg.get("custom") else []
    extra = [h.add_route(path, intent) for path, intent in customs]
    P = 8 * lanes
    assert extra == list(range(P * P, P * P + len(customs)))
    for r, (path, intent) in zip(extra, customs):
        got = h.route_info(r)
        assert h.route_len(r) == len(path)
        assert G.bits_equal(got[0][: len(path)], path) and got[1] == intent and tuple(got[2][:2]) == tuple(path[0])
    frozen = rng.uniform(size=(E, n)) < cfg.get("frozen", 0.0)
    st, troutes = _random_state(rng, h, n, cfg.get("npcs", 0), lanes, table, cfg.get("npc_gap", 60.0), extra,
                                cfg.get("lattice", 0), frozen, cfg.get("past", 0.0))
    h.set_traffic_routes(troutes)
    dims = None
    if cfg.get("dims"):
        dims = random_dims(rng, h)
        h.set_car_dims(*dims)
        assert h.car_dims_active()
        assert all(G.bits_equal(a, b) for a, b in zip(h.car_dims(), dims))
    oracles = [_oracle_from_state(cfg, st, e, troutes, customs, dims, rel) for e in range(E)]
    obs0 = h.observations()
    for e in range(E):
        assert G.bits_equal(obs0[e], oracles[e].observe()), f"env {e}: observation after set_state"
    dt = cfg.get("dt", 1 / 60)
    out = h.alloc_outputs()
    for t in range(T):
        acts = rng.uniform(-1, 1, (E, n, 2)).astype(np.float32)
        acts[rng.uniform(size=(E, n)) < 0.1] *= 2.5  # unclipped inputs
        acts[..., 0][rng.uniform(size=(E, n)) < 0.1] = 0.0  # exact-zero throttle (friction branch)
        acts[..., 0][frozen] = 0.0  # parked egos (v = 0) stay on their lattice points
        spawn = None
        if cfg.get("traffic"):
            spawn = np.where(rng.uniform(size=E) < cfg["spawn_p"], rng.integers(0, len(troutes), E), -1).astype(np.int32)
        h.step(acts, dt, out=out, spawn_route=spawn)
        gst = h.get_state()
        cd = h.car_dims() if dims is not None else None
        for e in range(E):
            r = oracles[e].step(acts[e], dt, int(spawn[e]) if spawn is not None else -1)
            tag = f"{cfg['name']} env {e} step {t + 1}"
            assert G.bits_equal(out["obs"][e], r["obs"]), tag + ": obs"
            assert G.bits_equal(out["reward"][e], r["rew"]), tag + ": reward"
            assert G.bits_equal(out["status"][e], r["status"]) and G.bits_equal(out["done"][e], r["done"]), tag
            got = [int(out["terminated"][e]), int(out["truncated"][e]), int(out["agents_alive"][e]), int(out["step"][e])]
            assert got == [r["terminated"], r["truncated"], r["agents_alive"], r["step"]], tag + ": flags"
            egos, npcs, sc = oracles[e].get_state()
            assert G.bits_equal(gst["x"][e], egos["x"]) and G.bits_equal(gst["heading"][e], egos["h"]), tag + ": pose"
            assert G.bits_equal(gst["path_index"][e], egos["path_index"]), tag + ": path_index"
            assert int(gst["npc_count"][e]) == len(npcs), tag + ": npc count"
            k = len(npcs)
            if k:
                assert G.bits_equal(gst["npc_x"][e, :k], npcs["x"]) and G.bits_equal(gst["npc_v"][e, :k], npcs["v"]), tag
            if cd is not None:  # sizes move with their cars (NPC erase, spawns of the default size)
                assert G.bits_equal(cd[0][e, :, 0], egos["len"]) and G.bits_equal(cd[0][e, :, 1], egos["wid"]), tag
                assert G.bits_equal(cd[1][e, :k, 0], npcs["len"]) and G.bits_equal(cd[1][e, :k, 1], npcs["wid"]), tag
    if cfg.get("expect_seq"):
        assert h.npc_stats()[1] > 0, "the controller's sequential fallback never ran"
    h.close()
