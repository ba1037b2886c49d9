"""Replay a golden scenario (tests/golden/*.npz, produced from the REAL reference
by tests/golden/gen_golden.py) through the device path and compare every
output bit-for-bit.  Test infrastructure; no /root/reference access."""
from __future__ import annotations

import glob
import json
import os
from dataclasses import dataclass, field
from typing import List, Optional

import numpy as np

GOLDEN_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")

EGO_F = ["x", "y", "v", "heading", "acc", "steering", "spawn_x", "spawn_y", "spawn_v", "spawn_heading",
         "prev_dist", "prev_a0", "prev_a1"]
NPC_F = ["npc_x", "npc_y", "npc_v", "npc_heading", "npc_acc", "npc_steering"]


def scenario_names(prefix: str = "") -> List[str]:
    out = []
    for p in sorted(glob.glob(os.path.join(GOLDEN_DIR, "*.npz"))):
        n = os.path.basename(p)[:-4]
        if n.startswith("static_"):
            continue
        if n.startswith(prefix):
            out.append(n)
    return out


def load(name: str):
    z = np.load(os.path.join(GOLDEN_DIR, name + ".npz"), allow_pickle=False)
    d = {k: z[k] for k in z.files}
    d["meta"] = json.loads(str(d["meta"]))
    return d


def point_index(name: str, lanes: int) -> int:
    kind, k = name.split("_")
    k = int(k)
    return k - 1 if kind == "IN" else 4 * lanes + k - 1


def bits_equal(a, b) -> bool:
    a = np.ascontiguousarray(a)
    b = np.ascontiguousarray(b)
    if a.shape != b.shape:
        return False
    if a.dtype == np.float32:
        return np.array_equal(a.view(np.uint32), b.astype(np.float32).view(np.uint32))
    return np.array_equal(a, b)


@dataclass
class Report:
    name: str
    steps: int = 0
    mismatches: List[str] = field(default_factory=list)
    max_obs_diff: float = 0.0
    seq_turns: int = 0  # NPC turns the controller ran sequentially (handle-wide, npc_stats)

    @property
    def ok(self) -> bool:
        return not self.mismatches

    def add(self, msg: str):
        if len(self.mismatches) < 20:
            self.mismatches.append(msg)


DEFAULT_DIMS = (54.0, 24.0)  # Car::length / Car::width defaults (cpp/Car.h:19-20)


def custom_paths(d):
    """Scenario d's paths of the caller's own, each its own length: the file holds them padded
    to [C][160][2] with their point counts in custom_len (absent: all 160)."""
    if "custom_paths" not in d:
        return []
    cps = d["custom_paths"]
    lens = d["custom_len"] if "custom_len" in d else [len(cp) for cp in cps]
    return [cp[: int(n)] for cp, n in zip(cps, lens)]


def custom_route_ids(h, d):
    """Register scenario d's paths of the caller's own (Car.path writes) on handle / oracle h
    (add_route); their ids, in the scenario's order."""
    return [h.add_route(cp, 0) for cp in custom_paths(d)]


def ego_route_ids(h, d, L, cids):
    """Each ego's route id: its lane route, or the custom path written into its Car.path."""
    eps = d["meta"].get("ego_paths") or [-1] * int(d["meta"]["n_agents"])
    return [cids[k] if k >= 0 else h.route_id(point_index(s, L), point_index(e, L))
            for (s, e), k in zip(d["meta"]["ego_routes"], eps)]


def npc_route_ids(rec_routes, troutes, cids):
    """NPC route ids from the recorded route indexes (traffic route, or 1000 + custom path)."""
    return [cids[r - 1000] if r >= 1000 else troutes[r] for r in rec_routes]


def has_dims(d) -> bool:
    """Whether scenario d writes Car::length / Car::width (record columns 13, 14)."""
    f = [d["init_ego_f"], d["ego_f"].reshape(-1, d["ego_f"].shape[-1])]
    if len(d["init_npc_f"]):
        f.append(d["init_npc_f"])
    return any(a.shape[-1] >= 15 and (np.any(a[:, 13] != DEFAULT_DIMS[0]) or np.any(a[:, 14] != DEFAULT_DIMS[1]))
               for a in f)


def set_dims(h, data):
    """The scenarios' initial car sizes on envs 0..B-1 of handle h (mev_set_car_dims)."""
    ego = np.empty((h.E, h.N, 2), np.float32)
    npc = np.empty((h.E, h.K, 2), np.float32)
    ego[...] = DEFAULT_DIMS
    npc[...] = DEFAULT_DIMS
    for b, d in enumerate(data):
        ego[b] = d["init_ego_f"][:, 13:15]
        k = len(d["init_npc_f"])
        if k:
            npc[b, :k] = d["init_npc_f"][:, 13:15]
    h.set_car_dims(ego, npc)


def npc_slots(data) -> int:
    """NPC slots a handle needs for these scenarios: 32, or 64 past 32 NPCs (ring_npc_k48)."""
    k = max(max(len(d["init_npc_f"]), int(d["npc_count"].max()) if len(d["npc_count"]) else 0) for d in data)
    return 32 if k <= 32 else 64


# An env without egos (traffic_no_ego*: the reference steps its traffic with cars empty) runs on a handle
# with one ego slot holding a dead car far off the map, as cpp_backend does: a dead ego is skipped by every
# ego loop of IntersectionEnv::step, and the only reader of a dead ego, the NPC spawn test's distance to
# every ego (TrafficFlow.cpp:240-259), never reaches it there.
NO_EGO_XY = -1.0e5


def ego_slots(meta) -> int:
    return max(1, int(meta["n_agents"]))


def make_handle(mod, meta, num_envs: int, device: int = 0, max_npcs: int = 32):
    R = int(meta["rays"])
    return mod.Handle(num_envs=num_envs, num_agents=ego_slots(meta), num_lanes=int(meta["num_lanes"]),
                      lidar_rays=R, obs_dim=127 if R <= 96 else 31 + R, traffic_flow=int(meta["traffic"]),
                      traffic_density=float(meta["density"]), use_team_reward=int(meta["use_team"]),
                      respawn_enabled=int(meta["respawn"]), max_steps=int(meta["max_steps"]),
                      reward=meta["reward"], max_npcs=max_npcs, device=device)


def set_egos(st, b, d, routes):
    """Env b's egos in a mev_get_state dict at scenario d's initial state (routes: their ids);
    without egos, the placeholder slot (NO_EGO_XY)."""
    f, i = d["init_ego_f"], d["init_ego_i"]
    if len(f) == 0:
        for key in EGO_F:
            st[key][b] = 0.0
        st["x"][b], st["y"][b] = NO_EGO_XY, NO_EGO_XY
        st["spawn_x"][b], st["spawn_y"][b] = NO_EGO_XY, NO_EGO_XY
        st["alive"][b], st["intention"][b], st["path_index"][b], st["route"][b] = 0, 0, 0, routes
        return
    for j, key in enumerate(EGO_F):
        st[key][b] = f[:, j]
    st["alive"][b], st["intention"][b], st["path_index"][b], st["route"][b] = i[:, 0], i[:, 1], i[:, 2], routes


def single_env_handle(mod, d):
    """A one-env handle at golden scenario d's initial state (as replay() sets it up);
    returns (handle, spawn_route(t) for its steps)."""
    meta = d["meta"]
    L = int(meta["num_lanes"])
    h = make_handle(mod, meta, 1, max_npcs=npc_slots([d]))
    cids = custom_route_ids(h, d)
    troutes = [h.route_id(point_index(s, L), point_index(e, L)) for s, e in meta["traffic_routes"]]
    h.set_traffic_routes(troutes)
    ego_routes = np.array([(ego_route_ids(h, d, L, cids) + troutes)[: ego_slots(meta)]], np.int32)
    h.set_ego_routes(ego_routes)
    st = h.get_state()
    set_egos(st, 0, d, ego_routes[0])
    k = len(d["init_npc_f"])
    st["npc_count"][0] = k
    if k:
        nf, ni = d["init_npc_f"], d["init_npc_i"]
        for j, key in enumerate(NPC_F):
            st[key][0, :k] = nf[:, j]
        st["npc_alive"][0, :k], st["npc_intention"][0, :k], st["npc_path_index"][0, :k] = ni[:, 0], ni[:, 1], ni[:, 2]
        st["npc_route"][0, :k] = npc_route_ids(ni[:, 3], troutes, cids)
    st["step_count"][0] = int(meta.get("init_step", 0))
    h.set_state(st)
    if has_dims(d):
        set_dims(h, [d])
    spawn_of = (lambda t: np.array([d["spawned"][t]], np.int32)) if meta["traffic"] else (lambda t: None)
    return h, spawn_of


def replay(mod, names, steps: Optional[int] = None, stop_at_first=True, kernel: int = 0,
           pack: int = 0, split: int = 0) -> List[Report]:
    """Run the scenarios `names` (identical configs) as envs 0..B-1 of one handle
    (kernel: the step kernel path, 0 = automatic; None is returned when the
    requested path does not apply to the scenario's configuration)."""
    if isinstance(names, str):
        names = [names]
    data = [load(n) for n in names]
    meta = data[0]["meta"]
    for d in data[1:]:
        for k in ("num_lanes", "n_agents", "rays", "use_team", "respawn", "max_steps", "traffic", "density", "reward",
                  "dt", "traffic_routes"):
            assert d["meta"][k] == meta[k], f"scenario configs differ in {k}"
    B = len(data)
    L = int(meta["num_lanes"])
    h = make_handle(mod, meta, B, max_npcs=npc_slots(data))
    if kernel:
        try:
            h.set_step_kernel(kernel)
        except mod.MevError:
            h.close()
            return None
    if pack:
        h.set_step_pack(pack)  # envs per fused wave (scheduling only)
    if split:
        h.set_step_split(split)  # two waves per fused workgroup: 1 off, 2 on (scheduling only)
    # paths of the caller's own: each scenario's, registered in turn (ids per scenario)
    cids = [custom_route_ids(h, d) for d in data]
    troutes = [h.route_id(point_index(s, L), point_index(e, L)) for s, e in meta["traffic_routes"]]
    h.set_traffic_routes(troutes)
    n = int(meta["n_agents"])
    ego_routes = np.zeros((B, ego_slots(meta)), np.int32)
    for b, d in enumerate(data):
        ego_routes[b] = (ego_route_ids(h, d, L, cids[b]) + troutes)[: ego_slots(meta)]
    h.set_ego_routes(ego_routes)
    # initial state
    st = h.get_state()
    for b, d in enumerate(data):
        set_egos(st, b, d, ego_routes[b])
        k = len(d["init_npc_f"])
        st["npc_count"][b] = k
        if k:
            nf, ni = d["init_npc_f"], d["init_npc_i"]
            for j, key in enumerate(NPC_F):
                st[key][b, :k] = nf[:, j]
            st["npc_alive"][b, :k] = ni[:, 0]
            st["npc_intention"][b, :k] = ni[:, 1]
            st["npc_path_index"][b, :k] = ni[:, 2]
            st["npc_route"][b, :k] = npc_route_ids(ni[:, 3], troutes, cids[b])
        st["step_count"][b] = int(d["meta"].get("init_step", 0))  # set_state scenarios start mid-episode
    h.set_state(st)
    dims = any(has_dims(d) for d in data)
    if dims:
        set_dims(h, data)
    reports = [Report(nm) for nm in names]
    obs0 = h.observations()
    for b, d in enumerate(data):
        if not bits_equal(obs0[b, :n, :127], d["init_obs"]):
            reports[b].add("initial obs differ")
    T = min(int(meta["steps"]), steps or 10 ** 9)
    out = h.alloc_outputs()
    for t in range(T):
        acts = np.stack([d["actions"][t] for d in data])
        if n == 0:  # (the placeholder slot's action: a dead car reads none)
            acts = np.zeros((B, 1, 2), np.float32)
        spawn = None
        if meta["traffic"]:
            spawn = np.array([d["spawned"][t] for d in data], np.int32)
        h.step(acts, float(meta["dt"]), out=out, spawn_route=spawn)
        st = h.get_state()
        cd = h.car_dims() if dims else None
        for b, d in enumerate(data):
            rep = reports[b]
            if not rep.ok and stop_at_first:
                continue
            rep.steps = t + 1
            g_obs = d["obs"][t]
            my = out["obs"][b][:n]
            diff = float(np.max(np.abs(my[:, :127] - g_obs))) if my.size else 0.0
            rep.max_obs_diff = max(rep.max_obs_diff, diff)
            if not bits_equal(my[:, :127], g_obs):
                bad = np.argwhere(my[:, :127].view(np.uint32) != g_obs.view(np.uint32))
                rep.add(f"step {t + 1}: obs differ at {bad[:4].tolist()} (max |d|={diff:.3g})")
            if "lidar" in d and meta["rays"] > 96:
                if not bits_equal(my[:, 31:], d["lidar"][t] * np.float32(1.0 / 250.0)):
                    rep.add(f"step {t + 1}: full lidar differs")
            if not bits_equal(out["reward"][b][:n], d["rew"][t]):
                rep.add(f"step {t + 1}: reward {out['reward'][b].tolist()} vs {d['rew'][t].tolist()}")
            if not bits_equal(out["done"][b][:n], d["done"][t]):
                rep.add(f"step {t + 1}: done {out['done'][b].tolist()} vs {d['done'][t].tolist()}")
            if not bits_equal(out["status"][b][:n], d["status"][t]):
                rep.add(f"step {t + 1}: status {out['status'][b].tolist()} vs {d['status'][t].tolist()}")
            fl = d["flags"][t]
            got = [int(out["terminated"][b]), int(out["truncated"][b]), int(out["agents_alive"][b]),
                   int(out["step"][b])]
            if got != [int(x) for x in fl]:
                rep.add(f"step {t + 1}: flags {got} vs {fl.tolist()}")
            ef, ei = d["ego_f"][t], d["ego_i"][t]
            for j, key in enumerate(EGO_F):
                if not bits_equal(st[key][b][:n], ef[:, j]):
                    rep.add(f"step {t + 1}: ego {key} {st[key][b][:4]} vs {ef[:4, j]}")
            if not bits_equal(st["alive"][b][:n], ei[:, 0].astype(np.uint8)) or \
                    not bits_equal(st["intention"][b][:n], ei[:, 1]) or not bits_equal(st["path_index"][b][:n], ei[:, 2]):
                rep.add(f"step {t + 1}: ego alive/intention/path_index differ")
            kc = int(d["npc_count"][t])
            if int(st["npc_count"][b]) != kc:
                rep.add(f"step {t + 1}: npc count {int(st['npc_count'][b])} vs {kc}")
            elif kc:
                nf, ni = d["npc_f"][t, :kc], d["npc_i"][t, :kc]
                for j, key in enumerate(NPC_F):
                    if not bits_equal(st[key][b, :kc], nf[:, j]):
                        rep.add(f"step {t + 1}: {key} {st[key][b, :kc]} vs {nf[:, j]}")
                if not bits_equal(st["npc_path_index"][b, :kc], ni[:, 2]):
                    rep.add(f"step {t + 1}: npc path_index differ")
                if not bits_equal(st["npc_route"][b, :kc], np.array(npc_route_ids(ni[:, 3], troutes, cids[b]), np.int32)):
                    rep.add(f"step {t + 1}: npc route differ")
                if cd is not None and not bits_equal(cd[1][b, :kc], nf[:, 13:15]):
                    rep.add(f"step {t + 1}: npc length / width differ")
            if cd is not None and not bits_equal(cd[0][b][:n], ef[:, 13:15]):
                rep.add(f"step {t + 1}: ego length / width differ")
        if stop_at_first and all(not r.ok for r in reports):
            break
    seq = h.npc_stats()[1]
    for r in reports:
        r.seq_turns = seq
    h.close()
    return reports
