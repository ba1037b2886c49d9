"""Generate the golden vectors in tests/golden/*.npz from the REAL reference.

TEST INFRASTRUCTURE.  Runs only in the build container, where /root/reference
exists and oracle/build_ref.sh has produced $MEV_REF_BUILD/libref_harness.so (the
unmodified reference simulator + our harness).  The .npz files it writes are
committed; the GPU box never needs the reference.

    python tests/golden/gen_golden.py            # (re)writes every scenario
    python tests/golden/gen_golden.py --check    # regenerates the deterministic scenarios into a
                                                 # temporary directory and compares them with the
                                                 # committed files, array by array, byte for byte
    python tests/golden/gen_golden.py NAME ...   # (re)writes the named scenarios only

Each scenario file holds the configuration (``meta`` JSON), the initial state
the device path is loaded with, the per-step inputs (actions, and for traffic
mode the route index of the NPC the reference's unseeded RNG spawned that step)
and the reference's per-step outputs: observations (N x 127), rewards, done,
status codes, (terminated, truncated, agents_alive, step) and the full ego/NPC
state after the step (incl. fields pybind does not expose).

Status codes: 0 ALIVE, 1 DEAD, 2 SUCCESS, 3 CRASH_WALL, 4 CRASH_LINE, 5 CRASH_CAR.
"""
from __future__ import annotations

import json
from typing import List
import math
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import refharness as R  # noqa: E402

OUT = os.path.dirname(os.path.abspath(__file__))
HERE = OUT

ROUTES3 = [("IN_1", "OUT_4"), ("IN_2", "OUT_8"), ("IN_3", "OUT_12"), ("IN_4", "OUT_7"),
           ("IN_5", "OUT_11"), ("IN_6", "OUT_3"), ("IN_7", "OUT_10"), ("IN_8", "OUT_2"),
           ("IN_9", "OUT_6"), ("IN_10", "OUT_1"), ("IN_11", "OUT_5"), ("IN_12", "OUT_9")]
ROUTES2 = [("IN_1", "OUT_3"), ("IN_2", "OUT_6"), ("IN_3", "OUT_5"), ("IN_4", "OUT_8"),
           ("IN_6", "OUT_2"), ("IN_7", "OUT_1"), ("IN_8", "OUT_4")]
DEFAULT_REWARD = [10.0, 1.0, -0.01, -10.0, -5.0, 10.0, -0.02, 0.2]


def policy(obs: np.ndarray, rng: np.random.Generator, target_v=3.5, noise=0.05) -> np.ndarray:
    """Route-following driver used to produce realistic action streams (the
    actions are stored; the device path never runs this)."""
    n = obs.shape[0]
    a = np.zeros((n, 2), np.float32)
    v = obs[:, 2] * 8.0
    th = obs[:, 5] * math.pi
    a[:, 1] = np.clip(2.0 * th, -1.0, 1.0)
    a[:, 0] = np.clip((target_v - v) * 0.5, -1.0, 1.0)
    a += rng.normal(0.0, noise, a.shape).astype(np.float32)
    return np.clip(a, -1.0, 1.0).astype(np.float32)


def run(name: str, *, n_agents: int, rays=96, use_team=False, respawn=True, max_steps=2000,
        traffic=False, density=0.5, lanes=3, ego_routes=None, reward=None, steps=200,
        act="random", seed=0, dt=1.0 / 60.0, act_scale=1.0, zero_throttle_p=0.0,
        inject=None, notes="", warmup=0, roundtrip=False, custom_paths=None, ego_paths=None, car_lidars=None):
    """custom_paths: C paths of the caller's own, [n][2] each, 2 <= n <= 4096 (Car.path writes;
    recorded padded with their last point, their lengths in custom_len); ego_paths: per ego
    the custom path written into its Car.path, or -1 (NPCs on custom path k, injected by
    `inject`, record route 1000 + k).  car_lidars: per ego None (add_car_with_route's own
    96-ray Lidar) or (rays, fov_deg, max_dist, step_size, rel_angles or None): the Lidar
    written into IntersectionEnv.lidars[k] (a Lidar() with those members assigned; None keeps
    Lidar()'s own 72 offsets, cpp/Lidar.cpp:4-14)."""
    routes = ROUTES3 if lanes == 3 else ROUTES2
    if ego_routes is None:
        ego_routes = [routes[i % len(routes)] for i in range(n_agents)]
    reward = list(DEFAULT_REWARD if reward is None else reward)
    env = R.RefEnv(num_lanes=lanes, use_team=use_team and not traffic, respawn=respawn, max_steps=max_steps,
                   traffic=traffic, density=density, routes=routes, reward=reward, rays=rays)
    env.reset()
    for i, (s, e) in enumerate(ego_routes):
        assert env.add_car(s, e, tag=routes.index((s, e)) if (s, e) in routes else -1) == 0
    cps = [] if custom_paths is None else [np.asarray(c, np.float32) for c in custom_paths]
    for c in cps:
        env.add_custom_path(c)
    for i, k in enumerate(ego_paths or []):
        if k >= 0:
            env.set_car_path(0, i, k)  # Car.path = ... (cpp/bindings.cpp:29)
    env.custom_paths = cps
    for k, cl in enumerate(car_lidars or []):
        if cl is not None:
            env.set_car_lidar(k, *cl)
    rng = np.random.default_rng(seed)
    if inject is not None:
        inject(env, rng)
    # unrecorded warm-up steps, then optionally IntersectionEnv::set_state(get_state())
    # (cpp/IntersectionEnv.cpp:394-416): the recorded part starts from that state, with
    # every LiDAR rebuilt as a default Lidar() of 72 rays (cpp/Lidar.h:11)
    wobs = env.obs()
    for t in range(warmup):
        wa = (rng.uniform(-1.0, 1.0, (env.n, 2)) * act_scale).astype(np.float32) if act == "random" \
            else policy(wobs, rng)
        wobs = env.step(wa, dt)["obs"]
    if roundtrip:
        env.state_roundtrip()
        rays = 72
    init_step = env.step_count
    n = env.n
    ef, ei = env.cars(0)
    nf, ni = env.cars(1)
    init_obs = env.obs()
    A, O, RW, D, ST, FL, SP, EF, EI, NC, LD = [], [], [], [], [], [], [], [], [], [], []
    NFl, NIl = [], []
    cur_obs = init_obs
    for t in range(steps):
        if act == "random":
            a = (rng.uniform(-1.0, 1.0, (n, 2)) * act_scale).astype(np.float32)
        else:
            a = policy(cur_obs, rng)
        if zero_throttle_p > 0:
            a[rng.uniform(size=n) < zero_throttle_p, 0] = 0.0
        r = env.step(a, dt)
        cur_obs = r["obs"]
        A.append(a)
        O.append(r["obs"])
        RW.append(r["rew"])
        D.append(r["done"].astype(np.uint8))
        ST.append(r["status"].astype(np.uint8))
        FL.append([r["terminated"], r["truncated"], r["agents_alive"], r["step"]])
        SP.append(r["spawned"])
        f, i = env.cars(0)
        EF.append(f)
        EI.append(i)
        f, i = env.cars(1)
        NC.append(len(f))
        NFl.append(f)
        NIl.append(i)
        if not car_lidars:
            LD.append(env.lidar())
    kmax = max([len(x) for x in NFl] + [1])
    npc_f = np.zeros((steps, kmax, R.NF), np.float32)
    npc_i = np.zeros((steps, kmax, R.NI), np.int32)
    for t in range(steps):
        npc_f[t, : NC[t]] = NFl[t]
        npc_i[t, : NC[t]] = NIl[t]
    meta = dict(name=name, num_lanes=lanes, n_agents=n, rays=rays, use_team=bool(use_team and not traffic),
                respawn=respawn, max_steps=max_steps, traffic=traffic, density=density,
                reward=reward, ego_routes=ego_routes, traffic_routes=routes, dt=dt, steps=steps,
                act=act, seed=seed, notes=notes, init_step=init_step, warmup=warmup, set_state=bool(roundtrip))
    if cps:
        meta["ego_paths"] = [int(k) for k in ego_paths or [-1] * n]
    if car_lidars:
        # per ego: [] (the default 96-ray Lidar) or [rays, fov_deg, max_dist, step_size, n_rel];
        # car_rel[k, :n_rel] = its rel_angles (n_rel = -1: Lidar()'s own 72)
        meta["car_lidars"] = [[] if cl is None else [int(cl[0]), float(cl[1]), float(cl[2]), float(cl[3]),
                                                      -1 if cl[4] is None else int(len(cl[4]))]
                              for cl in car_lidars]
    arrays = dict(
        meta=np.array(json.dumps(meta)),
        init_ego_f=ef, init_ego_i=ei, init_npc_f=nf.reshape(-1, R.NF), init_npc_i=ni.reshape(-1, R.NI),
        init_obs=init_obs, actions=np.asarray(A, np.float32), obs=np.asarray(O, np.float32),
        rew=np.asarray(RW, np.float32), done=np.asarray(D, np.uint8), status=np.asarray(ST, np.uint8),
        flags=np.asarray(FL, np.int32), spawned=np.asarray(SP, np.int32), ego_f=np.asarray(EF, np.float32),
        ego_i=np.asarray(EI, np.int32), npc_count=np.asarray(NC, np.int32), npc_f=npc_f, npc_i=npc_i,
    )
    if rays > 96:
        arrays["lidar"] = np.asarray(LD, np.float32)
    if cps:
        m = max([160] + [len(c) for c in cps])
        arrays["custom_paths"] = np.stack([np.concatenate([c, np.repeat(c[-1:], m - len(c), 0)])
                                           for c in cps]).astype(np.float32)
        if any(len(c) != 160 for c in cps):
            arrays["custom_len"] = np.array([len(c) for c in cps], np.int32)
    if car_lidars:
        m = max([len(cl[4]) for cl in car_lidars if cl is not None and cl[4] is not None] + [1])
        rel = np.zeros((n, m), np.float32)
        for k, cl in enumerate(car_lidars):
            if cl is not None and cl[4] is not None:
                rel[k, : len(cl[4])] = np.asarray(cl[4], np.float32)
        arrays["car_rel"] = rel
    path = os.path.join(OUT, f"{name}.npz")
    np.savez_compressed(path, **arrays)
    env.close()
    st = np.asarray(ST)
    hist = {int(c): int((st == c).sum()) for c in range(6)}
    print(f"{name:28s} n={n} R={rays} steps={steps} max_npc={max(NC) if NC else 0} "
          f"spawns={int((np.asarray(SP) >= 0).sum())} status={hist} -> {os.path.getsize(path)//1024} KB")


def inject_random_egos(env: R.RefEnv, rng: np.random.Generator):
    """Scatter the egos over the road area with random headings/speeds/controls."""
    f, i = env.cars(0)
    for k in range(len(f)):
        if rng.uniform() < 0.5:  # somewhere in the cross
            x, y = rng.uniform(249, 501), rng.uniform(0, 750)
            if rng.uniform() < 0.5:
                x, y = y, x
        else:  # near the box
            x, y = rng.uniform(230, 520, 2)
        f[k, 0], f[k, 1] = x, y
        f[k, 2] = rng.uniform(0, 8)
        f[k, 3] = rng.uniform(-math.pi, math.pi)
        f[k, 4] = rng.uniform(-15, 15)
        f[k, 5] = rng.uniform(-0.6, 0.6)
        f[k, 10] = rng.uniform(0, 600) if rng.uniform() < 0.8 else 0.0
        f[k, 11], f[k, 12] = rng.uniform(-1, 1, 2)
        i[k, 2] = int(rng.integers(0, 150))
        env.set_car(k, f[k], i[k])


def inject_dead(env: R.RefEnv, rng: np.random.Generator):
    inject_random_egos(env, rng)
    f, i = env.cars(0)
    for k in range(len(f)):
        if k % 3 == 1:
            i[k, 0] = 0
            env.set_car(k, f[k], i[k])


def inject_npcs(kcount: int, dims=None, custom=None):
    """dims: (length, width) per injected NPC, cycled (default 54 x 24); custom: inject
    NPC j on custom path custom[j] (>= 0) instead of a random traffic route."""
    def _inj(env: R.RefEnv, rng: np.random.Generator):
        """Place NPCs on points of random traffic routes (on their own path,
        path-aligned heading), at least 70 px apart and away from the ego."""
        ef, _ = env.cars(0)
        placed = [(float(ef[0, 0]), float(ef[0, 1]))] if len(ef) else []  # (an env may have no ego)
        e0 = len(placed)
        tries = 0
        while len(placed) < kcount + e0 and tries < 1000:
            tries += 1
            j = len(placed) - e0
            cj = custom[j] if custom is not None and j < len(custom) else -1
            route = int(rng.integers(0, 12))
            path = env.route_path(route) if cj < 0 else env.custom_paths[cj]
            idx = int(rng.integers(0, min(150, len(path) - 1)))
            x, y = float(path[idx, 0]), float(path[idx, 1])
            if placed and min((x - px) ** 2 + (y - py) ** 2 for px, py in placed) < 70.0 ** 2:
                continue
            dx, dy = path[idx + 1] - path[idx]
            f = np.zeros(R.NF, np.float32)
            f[0], f[1] = x + rng.normal(0, 1.0), y + rng.normal(0, 1.0)
            f[2] = rng.uniform(0, 5)
            f[3] = math.atan2(-dy, dx) + rng.normal(0, 0.05)
            f[6], f[7], f[9] = path[0, 0], path[0, 1], math.atan2(-(path[1, 1] - path[0, 1]), path[1, 0] - path[0, 0])
            f[13], f[14] = (54.0, 24.0) if dims is None else dims[j % len(dims)]
            i = np.array([1, 0, max(0, idx - 2), route], np.int32)
            assert env.add_npc(route, f, i) == 0
            if cj >= 0:  # Car.path = custom path cj (intention stays the route's, as a plain write)
                env.set_car_path(1, env.k - 1, cj)
            placed.append((x, y))
    return _inj


EGO_DIMS = [(80.0, 30.0), (40.0, 18.0), (54.0, 24.0), (70.0, 36.0), (30.0, 12.0), (110.0, 22.0), (60.0, 60.0),
            (20.0, 40.0)]
NPC_DIMS = [(90.0, 34.0), (36.0, 16.0), (54.0, 24.0), (66.0, 44.0), (120.0, 20.0)]


def with_ego_dims(inject=None, dims=EGO_DIMS):
    """Write Car.length / Car.width of every ego (cpp/bindings.cpp:24-25), after `inject`."""
    def _inj(env: R.RefEnv, rng: np.random.Generator):
        if inject is not None:
            inject(env, rng)
        f, i = env.cars(0)
        for k in range(len(f)):
            f[k, 13], f[k, 14] = dims[k % len(dims)]
            env.set_car(k, f[k], i[k])
    return _inj


def bent_path(env: R.RefEnv, route: int, amp: float, waves: float = 1.5) -> np.ndarray:
    """Traffic route `route`'s 160 points with a lateral sine offset (zero at both ends)."""
    p = env.route_path(route).astype(np.float64)
    t = np.linspace(0.0, 1.0, len(p))
    d = np.gradient(p, axis=0)
    nrm = np.stack([-d[:, 1], d[:, 0]], 1) / np.maximum(np.hypot(d[:, 0], d[:, 1]), 1e-9)[:, None]
    off = amp * np.sin(np.pi * t) * np.sin(2.0 * np.pi * waves * t)
    return (p + nrm * off[:, None]).astype(np.float32)


def diag_path(x0, y0, x1, y1, n=160) -> np.ndarray:
    t = np.linspace(0.0, 1.0, n, dtype=np.float64)
    return np.stack([x0 + (x1 - x0) * t, y0 + (y1 - y0) * t], 1).astype(np.float32)


def gen_static(lanes: int):
    """Route table and geometry of the reference for `lanes` lanes: every
    (start point, end point) pair's 160-point path, intent and spawn heading
    (cpp/RouteGen.cpp:7-205, cpp/IntersectionEnv.cpp:78-131), plus the road /
    yellow-line / line-mask predicates on the integer pixel grid and on random
    real-valued points."""
    nl = 4 * lanes
    names = [f"IN_{k}" for k in range(1, nl + 1)] + [f"OUT_{k}" for k in range(1, nl + 1)]
    pairs = [(s, e) for s in names for e in names]
    env = R.RefEnv(num_lanes=lanes, traffic=True, density=0.0, routes=pairs)
    env.reset()
    paths = np.stack([env.route_path(k) for k in range(len(pairs))])
    for k, (s_, e_) in enumerate(pairs):
        assert env.add_car(s_, e_, tag=k) == 0
    ef, ei = env.cars(0)
    grid = R.geometry_grid(lanes)
    rng = np.random.default_rng(lanes)
    pts = np.concatenate([rng.uniform(-120, 870, (30000, 2)), rng.uniform(150, 600, (30000, 2))]).astype(np.float32)
    road = np.array([R.lib().rh_is_on_road(lanes, float(x), float(y)) for x, y in pts], np.uint8)
    yel = np.array([R.lib().rh_hits_yellow_line(lanes, float(x), float(y)) for x, y in pts], np.uint8)
    env.close()
    np.savez_compressed(os.path.join(OUT, f"static_lanes{lanes}.npz"), names=np.array(names), paths=paths,
                        intent=ei[:, 1], spawn=ef[:, [0, 1, 3]], grid=grid, pts=pts, road=road, yellow=yel)
    print(f"static_lanes{lanes}: {len(pairs)} routes, grid on-road px={int((grid & 1).sum())}")


def gen_set_state():
    """set_state round trips (reference IntersectionEnv.cpp:404-416): 40 steps, then
    get_state/set_state, then 60 recorded steps with the 72-ray default LiDAR."""
    run("set_state_72_team", n_agents=8, rays=64, use_team=True, steps=60, act="policy", seed=20, warmup=40,
        roundtrip=True)
    run("set_state_72_n3", n_agents=3, rays=96, steps=60, act="random", seed=21, warmup=40, roundtrip=True)


def gen_dims():
    """Per-car sizes (Car::length / Car::width, cpp/Car.h:19-20, read-write through
    bindings.cpp:24-25): the status corners, the SAT and the LiDAR boxes of every car."""
    for c in range(4):
        run(f"dims_inject_egos_c{c}", n_agents=8, rays=64, steps=4, act="random", seed=400 + c,
            inject=with_ego_dims(inject_random_egos))
    run("dims_cfg3_policy", n_agents=8, rays=64, use_team=True, steps=300, act="policy", seed=410,
        inject=with_ego_dims())
    run("dims_respawn_off", n_agents=6, rays=96, respawn=False, steps=200, act="policy", seed=411,
        inject=with_ego_dims(dims=EGO_DIMS[::-1]))
    run("dims_npc_k7", n_agents=1, rays=64, traffic=True, density=0.0, steps=200, act="policy", seed=412,
        inject=with_ego_dims(inject_npcs(7, dims=NPC_DIMS), dims=[(90.0, 30.0)]))


def gen_dims_traffic():
    """Sized egos and NPCs with the reference's (unseeded) spawns: recorded and replayed."""
    run("dims_traffic_d5", n_agents=1, rays=64, traffic=True, density=5.0, steps=400, act="policy", seed=413,
        inject=with_ego_dims(inject_npcs(4, dims=NPC_DIMS), dims=[(70.0, 30.0)]))


def gen_paths():
    """Written Car.path (cpp/bindings.cpp:29; every function reads a car's path through it)."""
    env = R.RefEnv(num_lanes=3, traffic=True, density=0.0, routes=ROUTES3)
    bent = [bent_path(env, 0, 14.0), bent_path(env, 4, 10.0, 2.0), bent_path(env, 7, 12.0, 1.0)]
    env.close()
    run("path_bent_egos", n_agents=4, rays=64, use_team=True, steps=200, act="policy", seed=420,
        custom_paths=bent, ego_paths=[0, -1, 1, 2])
    # a diagonal route across the box for the ego (from its own spawn: the path is written after
    # add_car_with_route, so the car stays where that put it), an NPC on a bent traffic route
    env = R.RefEnv(num_lanes=3, traffic=True, density=0.0, routes=ROUTES3)
    p0 = env.route_path(5)
    diag = diag_path(float(p0[0, 0]), float(p0[0, 1]), 520.0, 520.0)
    bent_npc = bent_path(env, 9, 12.0)
    env.close()
    run("path_diag_npc", n_agents=1, rays=64, traffic=True, density=0.0, steps=200, act="policy", seed=421,
        ego_routes=[ROUTES3[5]], custom_paths=[diag, bent_npc], ego_paths=[0],
        inject=inject_npcs(3, custom=[1, -1, 1]))


def gen_paths_traffic():
    env = R.RefEnv(num_lanes=3, traffic=True, density=0.0, routes=ROUTES3)
    bent_npc = bent_path(env, 2, 10.0, 2.0)
    env.close()
    run("path_npc_d2", n_agents=1, rays=64, traffic=True, density=2.0, steps=300, act="policy", seed=422,
        custom_paths=[bent_npc], ego_paths=[-1], inject=inject_npcs(2, custom=[0, 0]))


def gen_paths_short():
    """Written Car.path of fewer than 160 points: every reader clamps to path.size()
    (Car.cpp:56, IntersectionEnv.cpp:16-17,177-182,446, TrafficFlow.cpp:55,89,262-263)."""
    env = R.RefEnv(num_lanes=3, traffic=True, density=0.0, routes=ROUTES3)
    r = [env.route_path(k) for k in range(12)]
    env.close()
    # ego k starts on ROUTES3[k]: a cut at 100 points (the last segment inside the turn), one at 40, and
    # a 2-point path from its start straight to point 60; ego 1 keeps its own route
    short = [r[0][:100], r[2][:40], np.stack([r[3][0], r[3][60]])]
    run("path_short_egos", n_agents=4, rays=64, use_team=True, steps=300, act="policy", seed=430,
        custom_paths=short, ego_paths=[0, -1, 1, 2])
    # traffic: the ego on a 120-point cut of its route; NPCs on 90- and 130-point cuts of traffic routes
    # (they arrive at path.back() inside the box and leave; the ghost scan runs into the path's end)
    env = R.RefEnv(num_lanes=3, traffic=True, density=0.0, routes=ROUTES3)
    p5, n9, n4 = env.route_path(5), env.route_path(9), env.route_path(4)
    env.close()
    run("path_short_npc", n_agents=1, rays=64, traffic=True, density=0.0, steps=300, act="policy", seed=431,
        ego_routes=[ROUTES3[5]], custom_paths=[p5[:120], n9[:90], n4[:130]], ego_paths=[0],
        inject=inject_npcs(4, custom=[1, 2, 1, 2]))


def resample(p: np.ndarray, n: int) -> np.ndarray:
    """Polyline p at n points, uniform in the point index (linear interpolation in f64)."""
    p = np.asarray(p, np.float64)
    t = np.linspace(0.0, len(p) - 1.0, n)
    i0 = np.minimum(np.floor(t).astype(int), len(p) - 2)
    w = (t - i0)[:, None]
    return (p[i0] * (1.0 - w) + p[i0 + 1] * w).astype(np.float32)


def gen_paths_long():
    """Written Car.path of more than 160 points (every reader bounds by path.size(): the window
    search Car.cpp:56, the look-ahead IntersectionEnv.cpp:446 / TrafficFlow.cpp:55, the ghost
    scan TrafficFlow.cpp:89, path.back() and the last segment IntersectionEnv.cpp:16-17,177-182)."""
    env = R.RefEnv(num_lanes=3, traffic=True, density=0.0, routes=ROUTES3)
    r = [env.route_path(k) for k in range(12)]
    env.close()
    # ego 0: its route at 400 points; ego 2: its route continued straight for 90 more points past
    # the exit (the goal off screen); ego 3: its route at 1000 points; ego 1 keeps its own route
    ext = np.concatenate([r[2], r[2][-1] + (r[2][-1] - r[2][-2]) * np.arange(1, 91, dtype=np.float32)[:, None]])
    run("path_long_egos", n_agents=4, rays=64, use_team=True, steps=300, act="policy", seed=432,
        custom_paths=[resample(r[0], 400), ext, resample(r[3], 1000)], ego_paths=[0, -1, 1, 2])
    # traffic: the ego on its route at 320 points, NPCs on traffic routes at 480 and 200 points
    env = R.RefEnv(num_lanes=3, traffic=True, density=0.0, routes=ROUTES3)
    p5, n9, n4 = env.route_path(5), env.route_path(9), env.route_path(4)
    env.close()
    run("path_long_npc", n_agents=1, rays=64, traffic=True, density=0.0, steps=300, act="policy", seed=433,
        ego_routes=[ROUTES3[5]], custom_paths=[resample(p5, 320), resample(n9, 480), resample(n4, 200)],
        ego_paths=[0], inject=inject_npcs(5, custom=[1, 2, 1, 2, -1]))


def inject_npcs_past_end(env: R.RefEnv, rng: np.random.Generator):
    """NPCs in the box whose path_index lies past the end of their Car.path (a plain write of
    path_index / path, cpp/bindings.cpp:29-30): update_path_index keeps it there (Car.cpp:56,
    an empty window), the look-ahead clamps to path.back() and the ghost scan is empty
    (TrafficFlow.cpp:88-89); beside them NPCs on their full routes."""
    # (traffic route, point of it the NPC stands on, custom path written into Car.path or -1, path_index)
    spec = [(9, 75, 0, 75), (4, 100, 1, 100), (7, 120, -1, 170), (2, 40, -1, 38), (0, 70, -1, 68),
            (10, 85, 0, 61), (11, 60, -1, 58)]
    for route, idx, cj, pidx in spec:
        path = env.route_path(route)
        dx, dy = path[idx + 1] - path[idx]
        f = np.zeros(R.NF, np.float32)
        f[0], f[1] = path[idx, 0] + rng.normal(0, 1.0), path[idx, 1] + rng.normal(0, 1.0)
        f[2] = rng.uniform(1, 5)
        f[3] = math.atan2(-dy, dx) + rng.normal(0, 0.05)
        f[6], f[7], f[9] = path[0, 0], path[0, 1], math.atan2(-(path[1, 1] - path[0, 1]), path[1, 0] - path[0, 0])
        f[13], f[14] = 54.0, 24.0
        assert env.add_npc(route, f, np.array([1, 0, pidx, route], np.int32)) == 0
        if cj >= 0:
            env.set_car_path(1, env.k - 1, cj)


def gen_paths_past_end():
    env = R.RefEnv(num_lanes=3, traffic=True, density=0.0, routes=ROUTES3)
    n9, n4 = env.route_path(9), env.route_path(4)
    env.close()
    run("path_past_end_npc", n_agents=1, rays=64, traffic=True, density=0.0, steps=200, act="policy", seed=434,
        custom_paths=[n9[:60], n4[:90]], ego_paths=[-1], inject=inject_npcs_past_end)


def gen_no_ego():
    """Traffic in an env without egos (reset, then traffic_cars written, no add_car_with_route):
    step() still counts, truncates and runs update_traffic_flow (IntersectionEnv.cpp:133-142)."""
    run("traffic_no_ego", n_agents=0, rays=64, traffic=True, density=0.0, steps=300, act="random", seed=435,
        ego_routes=[], max_steps=250, inject=inject_npcs(7))


def gen_no_ego_traffic():
    """The same with the reference's own spawns at density 5 (recorded, replayed)."""
    run("traffic_no_ego_d5", n_agents=0, rays=64, traffic=True, density=5.0, steps=400, act="random", seed=436,
        ego_routes=[])


def rel_angles(rays: int, fov: float) -> List[float]:
    """Lidar's beam offsets (cpp/Lidar.cpp:4-14, IntersectionEnv.cpp:118-126) in float32."""
    f32 = np.float32
    start = f32(-fov) * f32(0.5)
    step = f32(fov) / f32(rays - 1) if rays > 1 else f32(0.0)
    return [float((start + f32(i) * step) * f32(np.pi) / f32(180.0)) for i in range(rays)]


def gen_lidars():
    """Per-car LiDAR objects (IntersectionEnv.lidars is read-write, cpp/bindings.cpp:68, each
    Lidar's members too, :85-92): cars with different ray counts, ranges, steps and beam
    offsets in one env -- Lidar() as constructed (72 rays), Lidar() with fewer rays than its
    72 offsets (the first ones are used), offsets written for a 270-degree fan of 128 rays
    (the observation keeps 96), and NPCs in the beams."""
    run("lidar_mixed_n4", n_agents=4, rays=96, steps=200, act="policy", seed=430,
        car_lidars=[None, (72, 360.0, 250.0, 4.0, None), (48, 360.0, 200.0, 5.0, None),
                    (128, 270.0, 250.0, 4.0, rel_angles(128, 270.0))])
    run("lidar_mixed_npc", n_agents=2, rays=96, traffic=True, density=0.0, steps=200, act="policy", seed=431,
        car_lidars=[(32, 360.0, 150.0, 3.0, rel_angles(32, 360.0)), None], inject=inject_npcs(3))


def inject_npc_ring(kcount: int, spread: int = 300):
    """kcount NPCs around ego 0 at integer offsets in symmetric sets -- (a, b), (-a, b), (b, a),
    (-b, a) -- so that many of their distances to ego 0 are exactly equal: more than 16
    neighbour candidates with ties, where std::sort's order (IntersectionEnv.cpp:490) is not
    the push order.  At least 60 px apart, on screen; random traffic routes and speeds."""
    def _inj(env: R.RefEnv, rng: np.random.Generator):
        ef, _ = env.cars(0)
        x0, y0 = float(ef[0, 0]), float(ef[0, 1])
        placed = [(x0, y0)]
        tries = 0
        while len(placed) < kcount + 1 and tries < 4000:
            tries += 1
            a, b = int(rng.integers(40, spread)), int(rng.integers(0, spread))
            for dx, dy in ((a, b), (-a, b), (b, a), (-b, a)):
                if len(placed) >= kcount + 1:
                    break
                x, y = x0 + dx, y0 + dy
                if not (10 <= x <= 740 and 10 <= y <= 740):
                    continue
                if min((x - px) ** 2 + (y - py) ** 2 for px, py in placed) < 60.0 ** 2:
                    continue
                route = int(rng.integers(0, 12))
                path = env.route_path(route)
                f = np.zeros(R.NF, np.float32)
                f[0], f[1] = x, y
                f[2] = rng.uniform(0, 4)
                f[3] = rng.uniform(-math.pi, math.pi)
                f[6], f[7], f[9] = path[0, 0], path[0, 1], math.atan2(-(path[1, 1] - path[0, 1]), path[1, 0] - path[0, 0])
                f[13], f[14] = 54.0, 24.0
                i = np.array([1, 0, int(rng.integers(0, 100)), route], np.int32)
                assert env.add_npc(route, f, i) == 0
                placed.append((x, y))
    return _inj


def inject_ego_ring(env: R.RefEnv, rng: np.random.Generator):
    """Egos 1.. around ego 0 at integer offsets in symmetric sets (inject_npc_ring's layout):
    equal distances among more than 16 candidates."""
    f, i = env.cars(0)
    x0, y0 = float(f[0, 0]), float(f[0, 1])
    placed = [(x0, y0)]
    k = 1
    while k < len(f):
        a, b = int(rng.integers(40, 330)), int(rng.integers(0, 330))
        for dx, dy in ((a, b), (-a, b), (b, a), (-b, a)):
            if k >= len(f):
                break
            x, y = x0 + dx, y0 + dy
            if not (10 <= x <= 740 and 10 <= y <= 740):
                continue
            if min((x - px) ** 2 + (y - py) ** 2 for px, py in placed) < 60.0 ** 2:
                continue
            f[k, 0], f[k, 1] = x, y
            f[k, 2] = rng.uniform(0, 5)
            f[k, 3] = rng.uniform(-math.pi, math.pi)
            env.set_car(k, f[k], i[k])
            placed.append((x, y))
            k += 1


def gen_ties():
    """More than 16 neighbour candidates (IntersectionEnv.cpp:466-490): std::sort orders equal
    distances by its partitions.  N >= 18 egos share spawn points (two cars on one point are
    equidistant from every other) and symmetric spawn points tie too; rings of integer offsets
    tie by construction."""
    run("n18_team", n_agents=18, rays=96, use_team=True, steps=200, act="policy", seed=40)
    run("n24_team", n_agents=24, rays=64, use_team=True, steps=150, act="policy", seed=41)
    run("n32_r32", n_agents=32, rays=32, steps=60, act="policy", seed=42)
    run("n20_ring", n_agents=20, rays=64, steps=4, act="random", seed=43, inject=inject_ego_ring)
    run("ring_npc_k20", n_agents=1, rays=64, traffic=True, density=0.0, steps=150, act="policy", seed=44,
        inject=inject_npc_ring(20))
    run("ring_npc_k18_n4", n_agents=4, rays=64, traffic=True, density=0.0, steps=100, act="policy", seed=45,
        inject=inject_npc_ring(18))
    # the largest fleets a handle takes: 64 egos (mev_create's limit), and 1 ego among 48 NPCs of 64 slots
    run("n64_r16", n_agents=64, rays=16, steps=40, act="policy", seed=46)
    run("ring_npc_k48", n_agents=1, rays=32, traffic=True, density=0.0, steps=80, act="policy", seed=47,
        inject=inject_npc_ring(48, spread=340))


# (name prefix or scenario name, generator, deterministic).  Traffic with density > 0 draws
# its spawns from the reference's unseeded RNG (TrafficFlow.cpp:278,324): not reproducible.
def _core():
    gen_static(3)
    gen_static(2)
    # Config 1 shape: 1 env x 1 agent, 16 beams.
    run("cfg1_r16_random", n_agents=1, rays=16, steps=400, act="random", seed=0)
    run("cfg1_r16_policy", n_agents=1, rays=16, steps=300, act="policy", seed=1)
    # Config 2 shape, every route (straight / left / right), policy-driven to SUCCESS.
    for r in range(12):
        run(f"cfg2_r64_route{r:02d}", n_agents=1, rays=64, steps=160, act="policy", seed=10 + r,
            ego_routes=[ROUTES3[r]])
    # Config 3 shape: 8 agents, team reward, 64 beams.
    run("cfg3_team_random_s0", n_agents=8, rays=64, use_team=True, steps=300, act="random", seed=0)
    run("cfg3_team_random_s1", n_agents=8, rays=64, use_team=True, steps=300, act="random", seed=1)
    run("cfg3_team_policy", n_agents=8, rays=64, use_team=True, steps=400, act="policy", seed=2)
    # Native 127-D observation (96 beams), all 12 routes; 16 agents forces spawn ties.
    run("n12_r96_policy", n_agents=12, rays=96, steps=300, act="policy", seed=3)
    run("n16_r96_ties", n_agents=16, rays=96, steps=60, act="policy", seed=4)
    # Config 5 shape: 8 agents, 128 beams (obs truncates at 127; raw lidar stored).
    run("cfg5_r128_team", n_agents=8, rays=128, use_team=True, steps=150, act="random", seed=5)
    # respawn off / truncation / unclipped actions / exact-zero throttle / other dt.
    run("respawn_off_policy", n_agents=8, rays=64, respawn=False, steps=250, act="policy", seed=6)
    run("truncate_50", n_agents=2, rays=32, max_steps=50, steps=80, act="random", seed=7)
    run("unclipped_x3", n_agents=4, rays=64, steps=200, act="random", act_scale=3.0, seed=8)
    run("zero_throttle", n_agents=4, rays=64, steps=200, act="random", zero_throttle_p=0.5, seed=9)
    run("dt_1_30_custom_reward", n_agents=6, rays=48, use_team=True, steps=200, act="policy", seed=10,
        dt=1.0 / 30.0, reward=[5.0, 2.0, -0.05, -7.0, -3.0, 4.0, -0.1, 0.5])
    # 2-lane layout.
    run("lanes2_policy", n_agents=7, rays=64, lanes=2, steps=300, act="policy", seed=11)
    # State injection.
    for c in range(6):
        run(f"inject_egos_c{c}", n_agents=8, rays=64, steps=3, act="random", seed=100 + c, inject=inject_random_egos)
    run("inject_dead", n_agents=6, rays=64, steps=20, act="random", seed=200, inject=inject_dead)
    for k in (2, 5, 9):
        run(f"inject_npc_k{k}", n_agents=1, rays=64, traffic=True, density=0.0, steps=150, act="policy",
            seed=300 + k, inject=inject_npcs(k))
    gen_set_state()


def _traffic():
    # Traffic mode (config 4 shape) with recorded spawns.
    run("traffic_d05", n_agents=1, rays=64, traffic=True, density=0.5, steps=1500, act="policy", seed=12)
    run("traffic_d5", n_agents=1, rays=64, traffic=True, density=5.0, steps=800, act="policy", seed=13)
    run("traffic_d20", n_agents=1, rays=64, traffic=True, density=20.0, steps=500, act="policy", seed=14)
    run("traffic_d20_random", n_agents=1, rays=64, traffic=True, density=20.0, steps=400, act="random", seed=15)


GROUPS = [("core", _core, True), ("dims", gen_dims, True), ("paths", gen_paths, True), ("lidars", gen_lidars, True),
          ("paths_short", gen_paths_short, True), ("ties", gen_ties, True), ("paths_long", gen_paths_long, True),
          ("paths_past_end", gen_paths_past_end, True), ("no_ego", gen_no_ego, True),
          ("traffic", _traffic, False), ("dims_traffic", gen_dims_traffic, False),
          ("paths_traffic", gen_paths_traffic, False), ("no_ego_traffic", gen_no_ego_traffic, False)]


def check() -> int:
    """Regenerate every deterministic scenario into a temporary directory and compare each
    array of each file with the committed one, byte for byte.  Returns the mismatch count."""
    import tempfile
    global OUT
    bad = 0
    with tempfile.TemporaryDirectory() as tmp:
        OUT = tmp
        for _, gen, det in GROUPS:
            if det:
                gen()
        OUT = HERE
        for fn in sorted(os.listdir(tmp)):
            a = np.load(os.path.join(tmp, fn), allow_pickle=False)
            path = os.path.join(HERE, fn)
            if not os.path.exists(path):
                print(f"MISSING {fn}")
                bad += 1
                continue
            b = np.load(path, allow_pickle=False)
            diff = sorted(set(a.files) ^ set(b.files))
            diff += [k for k in sorted(set(a.files) & set(b.files))
                     if a[k].dtype != b[k].dtype or a[k].shape != b[k].shape or a[k].tobytes() != b[k].tobytes()]
            if diff:
                print(f"DIFFERS {fn}: {diff}")
                bad += 1
    print(f"gen_golden --check: {bad} file(s) differ")
    return bad


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "--check":
        sys.exit(1 if check() else 0)
    if len(sys.argv) > 1 and sys.argv[1] == "--set-state":  # only the set_state scenarios
        gen_set_state()
        return
    if len(sys.argv) > 1:  # groups by name
        for name, gen, _ in GROUPS:
            if name in sys.argv[1:]:
                gen()
        return
    for _, gen, _ in GROUPS:
        gen()


if __name__ == "__main__":
    main()
