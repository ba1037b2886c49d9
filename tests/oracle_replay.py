"""Replay golden scenarios through the C restatement (oracle/marl_oracle.c)."""
import os
import sys

import numpy as np

import golden_replay as G

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
import oracle as O  # noqa: E402


def state_from_records(f, i, routes):
    cars = O.new_cars(len(f))
    names = ["x", "y", "v", "h", "acc", "steer", "sx", "sy", "sv", "sh", "prev_dist", "pa0", "pa1"]
    for j, nm in enumerate(names):
        cars[nm] = f[:, j]
    cars["alive"] = i[:, 0]
    cars["intention"] = i[:, 1]
    cars["path_index"] = i[:, 2]
    cars["route"] = routes
    if f.shape[1] >= 15:  # the recorded Car::length / Car::width (ref_harness.cpp car_to_rec)
        cars["len"], cars["wid"] = f[:, 13], f[:, 14]
    return cars


def make_oracle(meta, lidar=None):
    """lidar: (rays, max_dist, step_size, rel_angles[:rays]) of a per-car LiDAR (None: meta's)."""
    R = int(meta["rays"]) if lidar is None else int(lidar[0])
    kw = {} if lidar is None else dict(max_dist=float(lidar[1]), step=float(lidar[2]), obs_dim=127)
    env = O.OracleEnv(num_lanes=int(meta["num_lanes"]), n_agents=int(meta["n_agents"]), rays=R,
                      obs_dim=kw.pop("obs_dim", int(meta.get("obs_dim", 127 if R <= 96 else 31 + R))),
                      use_team=bool(meta["use_team"]), respawn=bool(meta["respawn"]), max_steps=int(meta["max_steps"]),
                      traffic=bool(meta["traffic"]), density=float(meta["density"]), reward=meta["reward"], max_npcs=64,
                      **kw)
    if lidar is not None:
        env.set_rel_angles(np.asarray(lidar[3], np.float32))
    return env


def car_lidar_keys(d):
    """Per ego of a golden with per-car LiDAR objects (meta car_lidars, gen_golden.py gen_lidars):
    (rays, max_dist, step_size, rel_angles[:rays]); [] = add_car_with_route's 96-ray Lidar,
    n_rel -1 = Lidar()'s own 72 offsets (cpp/Lidar.cpp:4-14)."""
    def rel(rays, fov):
        f32 = np.float32
        st = f32(fov) / f32(rays - 1) if rays > 1 else f32(0.0)
        return [float((f32(-fov) * f32(0.5) + f32(i) * st) * f32(np.pi) / f32(180.0)) for i in range(rays)]
    keys = []
    for k, cl in enumerate(d["meta"]["car_lidars"]):
        if not cl:
            keys.append((96, 250.0, 4.0, tuple(rel(96, 360.0))))
            continue
        rays, _, maxd, stp, nrel = cl
        r = rel(72, 360.0) if nrel < 0 else d["car_rel"][k, :nrel].tolist()
        keys.append((int(rays), float(maxd), float(stp), tuple(np.asarray(r[:rays], np.float32).tolist())))
    return keys


def replay(name):
    """Every recorded output of golden `name` against the oracle.  Per-car LiDAR objects: one
    oracle per distinct configuration, all stepped alike, each car's row from its own (before
    the first step only the heads are compared: the reference's block then shows the written
    Lidar's stale distances, which no simulation state holds)."""
    d = G.load(name)
    meta = d["meta"]
    L = int(meta["num_lanes"])
    keys = car_lidar_keys(d) if "car_lidars" in meta else None
    uniq = list(dict.fromkeys(keys)) if keys else [None]
    envs = [make_oracle(meta, k) for k in uniq]
    row_of = np.array([uniq.index(k) for k in keys]) if keys else None
    env = envs[0]
    cids = G.custom_route_ids(env, d)
    for o in envs[1:]:
        G.custom_route_ids(o, d)
    tr = [env.route_id(G.point_index(s, L), G.point_index(e, L)) for s, e in meta["traffic_routes"]]
    ego_routes = G.ego_route_ids(env, d, L, cids)
    egos = state_from_records(d["init_ego_f"], d["init_ego_i"], ego_routes)
    k = len(d["init_npc_f"])
    npcs = state_from_records(d["init_npc_f"], d["init_npc_i"], G.npc_route_ids(d["init_npc_i"][:, 3], tr, cids)) \
        if k else []
    for o in envs:
        o.set_traffic_routes(tr)
        o.set_state(egos, npcs, int(meta.get("init_step", 0)))

    def stitch(rows):
        out = rows[0].copy()
        for g in range(1, len(rows)):
            out[row_of == g] = rows[g][row_of == g]
        return out
    errs = []
    if keys is None and not G.bits_equal(env.observe()[:, :127], d["init_obs"]):
        errs.append("initial obs")
    if keys is not None and not G.bits_equal(env.observe()[:, :31], d["init_obs"][:, :31]):
        errs.append("initial obs heads")
    for t in range(int(meta["steps"])):
        rs = [o.step(d["actions"][t], float(meta["dt"]), int(d["spawned"][t]) if meta["traffic"] else -1)
              for o in envs]
        r = rs[0]
        if keys is not None:
            r = dict(r, obs=stitch([q["obs"] for q in rs]))
            if any(not G.bits_equal(q["rew"], r["rew"]) for q in rs[1:]):
                errs.append(f"step {t + 1}: the per-LiDAR oracles diverged")
        if not G.bits_equal(r["obs"][:, :127], d["obs"][t]):
            errs.append(f"step {t + 1}: obs")
        if not G.bits_equal(r["rew"], d["rew"][t]):
            errs.append(f"step {t + 1}: reward")
        if not G.bits_equal(r["status"], d["status"][t]) or not G.bits_equal(r["done"], d["done"][t]):
            errs.append(f"step {t + 1}: status/done")
        if [r["terminated"], r["truncated"], r["agents_alive"], r["step"]] != [int(x) for x in d["flags"][t]]:
            errs.append(f"step {t + 1}: flags")
        if "lidar" in d and not G.bits_equal(r["obs"][:, 31:], d["lidar"][t] * np.float32(1.0 / 250.0)):
            errs.append(f"step {t + 1}: full lidar")
        egos, npcs, sc = env.get_state()
        ef = d["ego_f"][t]
        for j, nm in enumerate(["x", "y", "v", "h", "acc", "steer", "sx", "sy", "sv", "sh", "prev_dist", "pa0", "pa1"]):
            if not G.bits_equal(egos[nm], ef[:, j]):
                errs.append(f"step {t + 1}: ego {nm}")
        if len(npcs) != int(d["npc_count"][t]):
            errs.append(f"step {t + 1}: npc count")
        elif ef.shape[1] >= 15:  # car sizes move with their cars (NPC erase, resets)
            if not (G.bits_equal(egos["len"], ef[:, 13]) and G.bits_equal(egos["wid"], ef[:, 14])):
                errs.append(f"step {t + 1}: ego length / width")
            kc = int(d["npc_count"][t])
            if kc and not (G.bits_equal(npcs["len"], d["npc_f"][t, :kc, 13]) and
                           G.bits_equal(npcs["wid"], d["npc_f"][t, :kc, 14])):
                errs.append(f"step {t + 1}: npc length / width")
        if errs:
            break
    for o in envs:
        o.close()
    return errs


EGO_FIELDS = {"x": "x", "y": "y", "v": "v", "h": "heading", "acc": "acc", "steer": "steering", "sx": "spawn_x",
              "sy": "spawn_y", "sv": "spawn_v", "sh": "spawn_heading", "prev_dist": "prev_dist", "pa0": "prev_a0",
              "pa1": "prev_a1", "path_index": "path_index", "route": "route", "intention": "intention",
              "alive": "alive"}
NPC_FIELDS = {"x": "npc_x", "y": "npc_y", "v": "npc_v", "h": "npc_heading", "acc": "npc_acc",
              "steer": "npc_steering", "path_index": "npc_path_index", "route": "npc_route",
              "intention": "npc_intention", "alive": "npc_alive"}


def oracle_from_device_state(meta, st, e, traffic_routes=None, dims=None):
    """An oracle env holding env e of a device handle's state (mev_get_state arrays, every hidden
    Car field included): the reference's IntersectionEnv with its cars / traffic_cars / step_count
    set to the same values (cpp/IntersectionEnv.cpp:394-416, set_state)."""
    o = make_oracle(meta)
    if traffic_routes is not None:
        o.set_traffic_routes([int(r) for r in traffic_routes])
    n = int(meta["n_agents"])
    cars = O.new_cars(n)
    for a, b in EGO_FIELDS.items():
        cars[a] = st[b][e]
    k = int(st["npc_count"][e])
    npcs = O.new_cars(k)
    for a, b in NPC_FIELDS.items():
        npcs[a] = st[b][e, :k]
    if dims is not None:  # (ego [E][N][2], npc [E][K][2]) from Handle.car_dims()
        cars["len"], cars["wid"] = dims[0][e, :, 0], dims[0][e, :, 1]
        npcs["len"], npcs["wid"] = dims[1][e, :k, 0], dims[1][e, :k, 1]
    o.set_state(cars, npcs, int(st["step_count"][e]))
    return o


def check_step(tag, out, e, r):
    """Every output of env e of a device step (numpy dict) equals the oracle's step result r, bit for bit."""
    assert G.bits_equal(out["obs"][e], r["obs"]), tag + ": obs"
    assert G.bits_equal(out["reward"][e], r["rew"]), tag + ": reward"
    assert G.bits_equal(out["status"][e], r["status"]) and G.bits_equal(out["done"][e], r["done"]), tag + ": status"
    got = [int(out["terminated"][e]), int(out["truncated"][e]), int(out["agents_alive"][e]), int(out["step"][e])]
    assert got == [r["terminated"], r["truncated"], r["agents_alive"], r["step"]], tag + ": flags"


def check_state(tag, gst, e, o, dims=None):
    """The full ego / NPC state of env e (mev_get_state arrays) equals the oracle's, bit for bit
    (and the car sizes, dims = Handle.car_dims(), when given)."""
    egos, npcs, sc = o.get_state()
    if dims is not None:
        assert G.bits_equal(dims[0][e, :, 0], egos["len"]) and G.bits_equal(dims[0][e, :, 1], egos["wid"]), \
            f"{tag}: ego length / width"
        k_ = len(npcs)
        assert G.bits_equal(dims[1][e, :k_, 0], npcs["len"]) and G.bits_equal(dims[1][e, :k_, 1], npcs["wid"]), \
            f"{tag}: npc length / width"
    for a, b in EGO_FIELDS.items():
        if a in egos.dtype.names:
            assert G.bits_equal(gst[b][e], egos[a]), f"{tag}: ego {a}"
    assert int(gst["npc_count"][e]) == len(npcs), tag + ": npc count"
    k = len(npcs)
    for a, b in NPC_FIELDS.items():
        if k and a in npcs.dtype.names:
            assert G.bits_equal(gst[b][e, :k], npcs[a]), f"{tag}: npc {a}"
    assert int(gst["step_count"][e]) == int(sc), tag + ": step_count"
