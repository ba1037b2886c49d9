"""Drop-in for the reference's backend module (reference cpp_backend.py:30-66,
which lazily imports the pybind11 module MARLEnv, cpp/bindings.cpp:11-95).

The classes keep MARLEnv's names, attributes and methods (State, Car,
RewardConfig, StepResult, EnvState, Lidar, IntersectionEnv), but the
simulation runs in libmarlenv_hip.so on the GPU: one IntersectionEnv here is a
device handle holding ONE env (E = 1) whose N = number of added cars.  There
is no CPU simulator behind these classes — without the HIP library and a GPU,
creating the environment raises.

Deviations from MARLEnv (all outside the hot path):
 * configure_routes validates lane names immediately (MARLEnv fails later,
   inside step, on an unknown end lane; an unknown start lane never spawns);
 * per-car LiDAR objects (IntersectionEnv.lidars, bindings.cpp:68,85-92) are simulated
   as in the reference, each car's rays / max_dist / step_size / rel_angles; cars of
   different configurations are stepped by one device handle per configuration, all
   fed the same calls (identical states and spawn streams), each car's observation row
   taken from the handle of its own configuration.  rel_angles may be any finite list
   (|angle| <= 1000 rad) with at least `rays` entries, and rays >= 1 (the reference
   reads past the end otherwise);
   `lidars` must hold one Lidar per car, or one configuration for all of them;
 * Car.path may be any path of 2 .. 4096 points (every path MARLEnv itself
   generates has 160, RouteGen.cpp:111-205); a path that is not a lane-layout route
   is appended to the device route table (mev_add_route_n); paths of fewer than 2 or
   more than 4096 points raise ValueError (the reference reads path[1] of any
   non-empty path);
 * Car.length / Car.width (bindings.cpp:24-25) are simulated per car, as in the
   reference (status corners, SAT collisions, LiDAR boxes; mev_set_car_dims), in
   |value| <= 1e4 px;
 * observations after set_state() / mid-episode add_car_with_route() carry a
   fresh LiDAR block (max range), exactly as after reset.
"""
from __future__ import annotations

import math
from typing import List, Optional, Sequence, Tuple

import numpy as np

from . import _capi
from .utils import point_index, point_name

STATUS = _capi.STATUS_NAMES
DEFAULT_LIDAR = (96, 360.0, 250.0, 4.0)  # IntersectionEnv.cpp:113-116
CTOR_LIDAR = (72, 360.0, 250.0, 4.0)     # Lidar() defaults, Lidar.h:11-14 (used by set_state)
OBS_W = 127


def has_cpp_backend() -> bool:
    """True when the gfx950 library is present (reference cpp_backend.py:38-39)."""
    return _capi.lib_available()


class State:
    """reference cpp/Car.h:9-14"""

    __slots__ = ("x", "y", "v", "heading")

    def __init__(self, x: float = 0.0, y: float = 0.0, v: float = 0.0, heading: float = 0.0):
        self.x, self.y, self.v, self.heading = float(x), float(y), float(v), float(heading)

    def __repr__(self):
        return f"State(x={self.x:.3f}, y={self.y:.3f}, v={self.v:.3f}, heading={self.heading:.4f})"


class Car:
    """reference cpp/Car.h:16-46 (bound fields + the hidden ones, for state round trips)."""

    def __init__(self):
        self.state = State()
        self.length = 54.0
        self.width = 24.0
        self.alive = True
        self.intention = 0
        self.path: List[Tuple[float, float]] = []
        self.path_index = 0
        self.acc = 0.0
        self.steering_angle = 0.0
        self.spawn_state = State()
        self.prev_dist_to_goal = 0.0
        self.prev_action = (0.0, 0.0)
        self._route = -1

    def update(self, throttle: float, steer_input: float, dt: float):
        """Car::update (cpp/Car.cpp:9-40), same float arithmetic (host C helper)."""
        k = _capi.car_update([self.state.x, self.state.y, self.state.v, self.state.heading, self.acc,
                              self.steering_angle], throttle, steer_input, dt)
        self.state.x, self.state.y, self.state.v, self.state.heading = (float(k[0]), float(k[1]), float(k[2]),
                                                                        float(k[3]))
        self.acc, self.steering_angle = float(k[4]), float(k[5])

    def check_collision(self, other: "Car") -> bool:
        """Car::check_collision (cpp/Car.cpp:117-141), SAT on the oriented boxes."""
        a = [self.state.x, self.state.y, self.state.heading, self.length, self.width]
        b = [other.state.x, other.state.y, other.state.heading, other.length, other.width]
        return _capi.car_check_collision(a, b)

    def __repr__(self):
        return f"Car({self.state!r}, alive={self.alive}, intention={self.intention}, path_index={self.path_index})"


class RewardConfig:
    """reference cpp/Reward.h:5-14; writes go straight to the owning environment
    (as MARLEnv's by-reference property does, which env.py:57-77 relies on)."""

    _FIELDS = ("k_prog", "v_min_ms", "k_stuck", "k_cv", "k_co", "k_succ", "k_sm", "alpha")

    def __init__(self):
        object.__setattr__(self, "_owner", None)
        for k, v in zip(self._FIELDS, (10.0, 1.0, -0.01, -10.0, -5.0, 10.0, -0.02, 0.2)):
            object.__setattr__(self, k, float(v))

    def __setattr__(self, name, value):
        if name not in self._FIELDS:
            raise AttributeError(name)
        object.__setattr__(self, name, float(value))
        if self._owner is not None:
            self._owner._reward_dirty = True

    def as_list(self) -> List[float]:
        return [getattr(self, k) for k in self._FIELDS]

    def __repr__(self):
        return "RewardConfig(" + ", ".join(f"{k}={getattr(self, k)}" for k in self._FIELDS) + ")"


class StepResult:
    """reference cpp/Reward.h:16-29 (obs / rewards are float32 numpy arrays)."""

    def __init__(self):
        self.obs = np.zeros((0, OBS_W), np.float32)
        self.rewards = np.zeros(0, np.float32)
        self.done: List[int] = []
        self.status: List[str] = []
        self.agent_ids: List[int] = []
        self.agents_alive = 0
        self.terminated = False
        self.truncated = False
        self.step = 0


class EnvState:
    """reference cpp/EnvState.h:9-15"""

    def __init__(self):
        self.cars: List[Car] = []
        self.traffic_cars: List[Car] = []
        self.agent_ids: List[int] = []
        self.next_agent_id = 1
        self.step_count = 0


class Lidar:
    """reference cpp/Lidar.h:8-27 (defaults of Lidar(): 72 rays, 360 deg, 250 px, 4 px)."""

    def __init__(self, rays: int = 72, fov_deg: float = 360.0, max_dist: float = 250.0, step_size: float = 4.0):
        self.rays = int(rays)
        self.fov_deg = float(fov_deg)
        self.max_dist = float(max_dist)
        self.step_size = float(step_size)
        self.distances = [self.max_dist] * self.rays
        self.rel_angles = _rel_angles(self.rays, self.fov_deg)

    def normalized(self) -> List[float]:
        """Lidar::normalized (cpp/Lidar.cpp:92-98): d * (1/max) in float32."""
        inv = np.float32(1.0) / np.float32(self.max_dist) if self.max_dist > 0 else np.float32(0.0)
        return (np.asarray(self.distances, np.float32) * inv).tolist()


def _lidar_key(l_: "Lidar") -> tuple:
    """A car's LiDAR as the simulation sees it: (rays, fov_deg, max_dist, step_size, rel_angles);
    rel_angles as float32 values, every entry (the reference keeps the whole list)."""
    rays = int(l_.rays)
    rel = tuple(np.asarray(l_.rel_angles, np.float32).reshape(-1).tolist())
    if rays < 1 or len(rel) < rays:
        raise ValueError(f"Lidar with {rays} rays and {len(rel)} rel_angles: need rays >= 1 and at least rays "
                         "offsets (the reference reads past the end of rel_angles otherwise)")
    return (rays, float(l_.fov_deg), float(l_.max_dist), float(l_.step_size), rel)


def _default_key(lidar) -> tuple:
    """The per-car key of a uniform (rays, fov, max, step) configuration."""
    return (int(lidar[0]), float(lidar[1]), float(lidar[2]), float(lidar[3]),
            tuple(np.asarray(_rel_angles(int(lidar[0]), float(lidar[1])), np.float32).tolist()))


class _LidarGroup:
    """One env as several device handles that differ only in their LiDAR (one per distinct
    per-car configuration, cpp_backend's per-car `lidars`): every call that changes the env
    goes to all of them in the same order, so their states -- and their spawn streams --
    stay identical; reads come from the first; car i's observation row from handle
    row_of[i]."""

    # every call that changes the env or how it is stepped (not set_beam_angles: each handle
    # keeps its own configuration); snapshot / restore and the gather have no per-car-LiDAR use
    _ALL = ("set_state", "set_car_dims", "set_traffic_routes", "set_ego_routes", "reset", "configure",
            "configure_traffic", "set_reward", "add_route", "set_reset_routes", "set_stream", "use_own_stream",
            "set_step_kernel", "set_step_pack", "set_step_split", "set_env_deal", "set_serve", "kernel_timing")
    _REFUSED = ("snapshot", "restore", "comm_init", "set_gather_format", "set_beam_angles")

    def __init__(self, handles, row_of):
        self._hs = list(handles)
        self._row_of = np.asarray(row_of)
        self._outs = None

    def __getattr__(self, name):
        if name in _LidarGroup._REFUSED:
            raise AttributeError(f"{name}: not available on an env whose cars have different LiDAR configurations")
        if name in _LidarGroup._ALL:
            def call(*a, **k):
                r = [getattr(h, name)(*a, **k) for h in self._hs]
                return r[0]
            return call
        return getattr(self._hs[0], name)

    def _stitch(self, obs0, others):
        for g, o in enumerate(others, start=1):
            m = self._row_of == g
            obs0[0, m] = o[0, m]
        return obs0

    def step(self, actions, dt=1.0 / 60.0, out=None):
        if self._outs is None:
            self._outs = [h.alloc_outputs() for h in self._hs[1:]]
        r = self._hs[0].step(actions, dt, out=out)
        for h, o in zip(self._hs[1:], self._outs):
            h.step(actions, dt, out=o)
        self._stitch(r["obs"], [o["obs"] for o in self._outs])
        return r

    def observations(self):
        return self._stitch(self._hs[0].observations().copy(), [h.observations() for h in self._hs[1:]])

    def close(self):
        for h in self._hs:
            h.close()


def _rel_angles(rays: int, fov: float) -> List[float]:
    """Beam offsets in float32 exactly as cpp/Lidar.cpp:4-14."""
    f32 = np.float32
    start = f32(-fov) * f32(0.5)
    step = f32(fov) / f32(rays - 1) if rays > 1 else f32(0.0)
    pi = f32(math.pi)
    return [float((start + f32(i) * step) * pi / f32(180.0)) for i in range(rays)]


class IntersectionEnv:
    """MARLEnv.IntersectionEnv (reference cpp/IntersectionEnv.h:23-105) on the GPU."""

    def __init__(self, num_lanes: int = 3, device: int = 0, max_npcs: int = 32):
        # max_npcs: NPC slots of the device handle.  32 (the C ABI's default) runs the compile-time
        # one-ego kernels; spawned traffic never exceeds 15 NPCs (profiles/r6_fleet_probe.txt), and a
        # written traffic_cars vector of more cars re-creates the handle at 64 slots (_apply_state).
        self.num_lanes = int(num_lanes)
        self._device = int(device)
        self._max_npcs = int(max_npcs)
        self._paths = {}  # route id -> its path points as (x, y) tuples (Car.path)
        self._route_ids = None  # path bytes (f32 [n, 2]) -> route id, built on first use
        self._custom: List[Tuple[np.ndarray, int]] = []  # Car.path routes of the caller's own, in id order
        self._use_team, self._respawn, self._max_steps = False, True, 2000
        self._traffic, self._density = False, 0.5
        self._reward = RewardConfig()
        object.__setattr__(self._reward, "_owner", self)
        self._reward_dirty = True
        self._lidar = DEFAULT_LIDAR
        self._h: Optional[_capi.Handle] = None
        self._out_h = None  # the handle step()'s buffers (_out, _act) belong to
        self._routes: List[int] = []     # ego route ids (add order)
        self._agent_ids: List[int] = []
        self._next_id = 1
        self._fresh = True               # no step since reset: added cars start from spawn
        self._pending: List[int] = []    # cars added since the last sync
        self._traffic_routes: Optional[List[int]] = None  # None = reference default (init_traffic_routes)
        # An env without egos still steps (IntersectionEnv.cpp:133-142: the count, truncation and the traffic
        # run with cars empty): its handle holds one ego slot with a dead car far off the map (_NO_EGO_XY).
        # Every ego loop of step skips a dead car, and the one reader of a dead ego, the NPC spawn test's
        # distance to every ego (TrafficFlow.cpp:240-259), never reaches it there.
        self._ghost = False        # self._h is such a handle
        self._ghost_reset = False  # reset() since: the next use resets it

    # ------------------------------------------------------------ config
    def configure(self, use_team: bool, respawn: bool, max_steps: int):
        self._use_team, self._respawn, self._max_steps = bool(use_team), bool(respawn), int(max_steps)
        if self._h is not None:
            self._h.configure(self._use_team, self._respawn, self._max_steps)

    def configure_traffic(self, enabled: bool, density: float):
        self._traffic, self._density = bool(enabled), max(0.0, float(density))
        if self._h is not None:
            self._h.configure_traffic(self._traffic, self._density)

    def configure_routes(self, routes: Sequence[Tuple[str, str]]):
        ids = []
        P = 8 * self.num_lanes
        for s, e in routes:
            si, ei = point_index(s, self.num_lanes), point_index(e, self.num_lanes)
            if si < 0 or ei < 0:
                raise IndexError(f"unknown lane id in route ({s!r}, {e!r})")
            ids.append(si * P + ei)
        self._traffic_routes = ids
        if self._h is not None:
            self._h.set_traffic_routes(ids)

    @property
    def reward_config(self) -> RewardConfig:
        return self._reward

    @reward_config.setter
    def reward_config(self, rc: RewardConfig):
        for k in RewardConfig._FIELDS:
            setattr(self._reward, k, getattr(rc, k))

    # ----------------------------------------------------------- episode
    def reset(self):
        """IntersectionEnv::reset (cpp/IntersectionEnv.cpp:66-76)."""
        self._routes, self._agent_ids, self._pending = [], [], []
        self._ghost_reset = self._ghost
        self._next_id = 1
        self._fresh = True
        self._lidar = DEFAULT_LIDAR  # add_car_with_route gives every new car a 96-ray Lidar

    def add_car_with_route(self, start_id: str, end_id: str):
        """cpp/IntersectionEnv.cpp:78-131: unknown start -> silently ignored; unknown end -> IndexError."""
        si = point_index(start_id, self.num_lanes)
        if si < 0:
            return
        ei = point_index(end_id, self.num_lanes)
        if ei < 0:
            raise IndexError(f"unknown lane id {end_id!r}")  # std::out_of_range from .at() (RouteGen.cpp:120)
        r = si * 8 * self.num_lanes + ei
        if self._lidar[0] == "per_car":  # the new car's own Lidar: 96 rays (IntersectionEnv.cpp:111-128)
            self._lidar = ("per_car", tuple(self._lidar[1]) + (_default_key(DEFAULT_LIDAR),))
        self._routes.append(r)
        self._pending.append(r)
        self._agent_ids.append(self._next_id)
        self._next_id += 1

    def _create(self, n: int, lidar):
        """A device handle for n cars of one LiDAR configuration `lidar` ((rays, fov, max, step)),
        or, per car (("per_car", keys), see _lidar_key), one handle per distinct key."""
        if lidar[0] == "per_car":
            keys = self._car_keys(lidar, n)
            uniq = list(dict.fromkeys(keys))
            return _LidarGroup([self._create(n, k[:4]) if k == _default_key(k[:4]) else self._create_rel(n, k)
                                for k in uniq], [uniq.index(k) for k in keys])
        h = _capi.Handle(num_envs=1, num_agents=n, num_lanes=self.num_lanes, lidar_rays=lidar[0],
                         lidar_fov_deg=lidar[1], lidar_max_dist=lidar[2], lidar_step=lidar[3], obs_dim=OBS_W,
                         traffic_flow=int(self._traffic), traffic_density=self._density,
                         use_team_reward=int(self._use_team), respawn_enabled=int(self._respawn),
                         max_steps=self._max_steps, reward=self._reward.as_list(),
                         max_npcs=self._max_npcs, device=self._device)
        for path, intent in self._custom:  # the caller's own routes keep their ids on a new handle
            h.add_route(path, intent)
        return h

    def _create_rel(self, n: int, key):
        h = self._create(n, key[:4])
        try:
            h.set_beam_angles(np.asarray(key[4][: key[0]], np.float32))  # Lidar::rel_angles[0 .. rays)
        except _capi.MevError as e:
            h.close()
            raise ValueError(f"Lidar.rel_angles: {e}") from None
        return h

    @staticmethod
    def _car_keys(lidar, n: int) -> List[tuple]:
        """Per-car keys for n cars: cars beyond the list got add_car_with_route's 96-ray Lidar."""
        keys = list(lidar[1][:n])
        return keys + [_default_key(DEFAULT_LIDAR)] * (n - len(keys))

    def _sync(self, ghost: bool = False) -> Optional[_capi.Handle]:
        """The device handle for the cars added so far; without cars None, or (ghost) the
        no-ego handle (see __init__)."""
        n = len(self._routes)
        if n == 0:
            return self._sync_ghost(ghost)
        h = self._h
        if h is None or h.N != n or self._h_lidar != self._lidar or self._ghost:
            keep = keep_dims = None
            if h is not None and not self._fresh:
                keep = h.get_state()  # cars added mid-episode keep the running episode
                keep_dims = h.car_dims() if h.car_dims_active() else None
                if self._ghost:  # (the placeholder is no car)
                    keep = {k: v for k, v in keep.items() if k.startswith("npc_") or v.ndim == 1}
                    keep_dims = (keep_dims[0][:, :0], keep_dims[1]) if keep_dims is not None else None
            self._ghost = False
            if h is not None:
                h.close()
            h = self._h = self._create(n, self._lidar)
            self._h_lidar = self._lidar
            self._reward_dirty = False
            if self._traffic_routes is not None:
                h.set_traffic_routes(self._traffic_routes)
            h.set_ego_routes(np.asarray(self._routes, np.int32)[None])
            h.reset()  # every car at the spawn of its route
            if keep is not None:
                self._restore_grown(keep, keep_dims)
            self._pending = []
            return h
        if self._reward_dirty:
            h.set_reward(self._reward.as_list())
            self._reward_dirty = False
        if self._pending:
            h.set_ego_routes(np.asarray(self._routes, np.int32)[None])
            if self._fresh:
                h.reset()
            self._pending = []
        return h

    def _sync_ghost(self, create: bool) -> Optional[_capi.Handle]:
        h = self._h
        if h is not None and self._ghost:
            if self._reward_dirty:
                h.set_reward(self._reward.as_list())
                self._reward_dirty = False
            if self._ghost_reset:
                h.reset()
                self._place_ghost(h)
                self._ghost_reset = False
            return h
        if not create:
            return None
        if h is not None:
            h.close()
        h = self._h = self._create(1, DEFAULT_LIDAR)
        self._h_lidar = DEFAULT_LIDAR
        self._ghost, self._ghost_reset, self._reward_dirty = True, False, False
        if self._traffic_routes is not None:
            h.set_traffic_routes(self._traffic_routes)
        h.set_ego_routes(np.zeros((1, 1), np.int32))
        h.reset()
        self._place_ghost(h)
        return h

    @staticmethod
    def _place_ghost(h, st=None):
        st = h.get_state() if st is None else st
        for k in ("x", "y", "spawn_x", "spawn_y"):
            st[k][0, 0] = _NO_EGO_XY
        st["alive"][0, 0] = 0
        h.set_state(st)

    def _restore_grown(self, old, old_dims=None):
        """Old cars keep their state (and size); newly added ones start at their spawn (add_car_with_route)."""
        h = self._h
        new = h.get_state()  # after creation == a reset: every car at its spawn
        m = old["x"].shape[1] if "x" in old else 0
        for k, v in old.items():
            if k.startswith("npc_") or v.ndim == 1:
                new[k] = v
            else:
                new[k][:, :m] = v
        h.set_state(new)
        if old_dims is not None:
            ego, npc = h.car_dims()
            ego[:, :m] = old_dims[0][:, :m]
            h.set_car_dims(ego, old_dims[1])

    @property
    def step_count(self) -> int:
        h = self._sync()
        return int(h.get_state()["step_count"][0]) if h is not None else 0

    @step_count.setter
    def step_count(self, value: int):
        h = self._sync(ghost=True)
        if h is not None:
            h.set_state({"step_count": np.array([int(value)], np.int32)})

    def step(self, throttles: Sequence[float], steerings: Sequence[float], dt: float = 1.0 / 60.0) -> StepResult:
        """IntersectionEnv::step (cpp/IntersectionEnv.cpp:133-392) on the GPU."""
        h = self._h
        if h is None or self._pending or self._reward_dirty or h.N != len(self._routes) or self._h_lidar != self._lidar \
                or self._ghost:
            h = self._sync(ghost=True)
        n = h.N
        # one action buffer and one output dict per handle (its args struct is reused by
        # Handle.step); the result's arrays are copies, like the reference's pybind conversions
        if self._out_h is not h:
            self._out_h, self._out, self._act = h, h.alloc_outputs(), np.zeros((1, n, 2), np.float32)
        act = self._act
        t = np.asarray(throttles, np.float32).reshape(-1)[:n]
        s = np.asarray(steerings, np.float32).reshape(-1)[:n]
        if t.size < n or s.size < n:  # missing inputs are zero
            act.fill(0.0)
        act[0, : t.size, 0] = t
        act[0, : s.size, 1] = s
        out = h.step(act, float(dt), out=self._out)
        self._fresh = False
        m = 0 if self._ghost else n
        res = StepResult.__new__(StepResult)
        res.obs = out["obs"][0][:m].copy()
        res.rewards = out["reward"][0][:m].copy()
        res.done = out["done"][0][:m].tolist()
        res.status = [STATUS[x] for x in out["status"][0][:m].tolist()]
        res.agent_ids = list(self._agent_ids)
        res.agents_alive = int(out["agents_alive"][0])
        res.terminated = bool(out["terminated"][0])
        res.truncated = bool(out["truncated"][0])
        res.step = int(out["step"][0])
        return res

    def get_observations(self) -> np.ndarray:
        """get_observations (cpp/IntersectionEnv.cpp:418-520): float32 [n, 127]."""
        h = self._sync()
        if h is None or self._ghost:
            return np.zeros((0, OBS_W), np.float32)
        return h.observations()[0]

    # ----------------------------------------------------------- cars
    def _cars_from(self, st, ego: bool, dims=None) -> List[Car]:
        out = []
        h = self._h
        if dims is None:
            dims = h.car_dims() if h.car_dims_active() else None
        if ego:
            n = 0 if self._ghost else h.N
            get = lambda k, i: st[k][0, i]  # noqa: E731
            count = n
        else:
            count = int(st["npc_count"][0])
            get = lambda k, i: st["npc_" + k][0, i]  # noqa: E731
        for i in range(count):
            c = Car()
            c.state = State(get("x", i), get("y", i), get("v", i), get("heading", i))
            c.acc, c.steering_angle = float(get("acc", i)), float(get("steering", i))
            c.alive = bool(get("alive", i))
            c.intention = int(get("intention", i))
            c.path_index = int(get("path_index", i))
            c._route = int(get("route", i))
            path = self._paths.get(c._route)
            if path is None:  # route tables are constant for the env's lane count: built once per route
                pts = h.route_info(c._route)[0][: h.route_len(c._route)]  # (a shorter path's own points)
                path = self._paths[c._route] = [tuple(map(float, p)) for p in pts]
            c.path = list(path)
            if dims is not None:  # Car::length / Car::width (cpp/Car.h:19-20)
                c.length, c.width = float(dims[0 if ego else 1][0, i, 0]), float(dims[0 if ego else 1][0, i, 1])
            if ego:
                c.spawn_state = State(st["spawn_x"][0, i], st["spawn_y"][0, i], st["spawn_v"][0, i],
                                      st["spawn_heading"][0, i])
                c.prev_dist_to_goal = float(st["prev_dist"][0, i])
                c.prev_action = (float(st["prev_a0"][0, i]), float(st["prev_a1"][0, i]))
            else:
                c.spawn_state = State(c.path[0][0], c.path[0][1], 0.0,
                                      math.atan2(-(c.path[1][1] - c.path[0][1]), c.path[1][0] - c.path[0][0]))
            out.append(c)
        return out

    @property
    def cars(self) -> List[Car]:
        h = self._sync()
        return [] if h is None else self._cars_from(h.get_state(), True)

    @property
    def traffic_cars(self) -> List[Car]:
        h = self._sync()
        return [] if h is None else self._cars_from(h.get_state(), False)

    @property
    def lidars(self) -> List[Lidar]:
        """One Lidar per car; distances recovered exactly from the observation
        (every distance is max_dist or a probe distance k*step)."""
        h = self._sync()
        if h is None or self._ghost:
            return []
        n = h.N
        keys = self._car_keys(self._lidar, n) if self._lidar[0] == "per_car" else [_default_key(self._lidar)] * n
        obs = h.observations()[0]
        out = []
        for row_all, (rays, fov, maxd, stp, rel) in zip(obs, keys):
            row = row_all[31:31 + min(rays, OBS_W - 31)]
            inv = np.float32(1.0) / np.float32(maxd)
            l_ = Lidar(rays, fov, maxd, stp)
            l_.rel_angles = list(rel)
            k = np.rint(row.astype(np.float64) * maxd / stp)
            cand = (k * stp).astype(np.float32)
            ok = (cand * inv) == row
            d = np.where(ok, cand, np.float32(maxd))
            l_.distances = d.tolist() + [maxd] * (rays - len(d))
            out.append(l_)
        return out

    @lidars.setter
    def lidars(self, lidars: Sequence[Lidar]):
        if not lidars:
            return
        keys = [_lidar_key(l_) for l_ in lidars]
        if len(set(keys)) == 1 and keys[0] == _default_key(keys[0][:4]):
            self._set_lidar(keys[0][:4])  # one configuration with its own offsets: one handle
            return
        n = len(self._routes)
        if len(set(keys)) > 1 and len(keys) != n:
            raise ValueError(f"{len(keys)} Lidars for {n} cars: one per car (or one configuration for all)")
        self._set_lidar(("per_car", tuple(keys * n if len(keys) == 1 else keys)))

    def _set_lidar(self, lidar):
        if lidar[0] != "per_car":
            lidar = (int(lidar[0]), float(lidar[1]), float(lidar[2]), float(lidar[3]))
        if lidar == self._lidar:
            return
        if self._h is not None and len(self._routes) == self._h.N and not self._ghost:
            st = self._h.get_state()
            dims = self._h.car_dims() if self._h.car_dims_active() else None
            self._h.close()
            self._h = self._create(len(self._routes), lidar)
            if self._traffic_routes is not None:
                self._h.set_traffic_routes(self._traffic_routes)
            self._h.set_ego_routes(np.asarray(self._routes, np.int32)[None])
            self._h.set_state(st)
            if dims is not None:
                self._h.set_car_dims(*dims)
            self._h_lidar = lidar
        self._lidar = lidar

    # ---------------------------------------------------------- snapshot
    def get_state(self) -> EnvState:
        """cpp/IntersectionEnv.cpp:394-404"""
        s = EnvState()
        h = self._sync()
        if h is not None:
            st = h.get_state()
            s.cars = self._cars_from(st, True)
            s.traffic_cars = self._cars_from(st, False)
            s.step_count = int(st["step_count"][0])
        s.agent_ids = list(self._agent_ids)
        s.next_agent_id = self._next_id
        return s

    def _route_of(self, c: Car) -> int:
        """The route id of Car.path (read-write in MARLEnv, cpp/bindings.cpp:29): a lane-layout route or one
        registered before, else a new route of the caller's own (mev_add_route_n; 2 .. 4096 points)."""
        if len(c.path) == 0:
            if c._route >= 0:
                return c._route
            raise ValueError("Car.path is empty")
        want = np.asarray(c.path, np.float32).reshape(-1, 2)
        if self._route_ids is None:
            P = 8 * self.num_lanes
            self._route_ids = {self._h.route_info(r)[0].tobytes(): r for r in range(P * P)}
            for k, (path, _) in enumerate(self._custom):
                self._route_ids[path.tobytes()] = P * P + k
        r = self._route_ids.get(want.tobytes())
        if r is not None:
            return r
        if not 2 <= len(want) <= _capi.MAX_PATH_LEN:
            raise ValueError(f"Car.path must have 2 .. {_capi.MAX_PATH_LEN} points (every path the reference "
                             f"generates has {_capi.PATH_LEN}, RouteGen.cpp:111-205); got {len(want)}")
        intent = min(max(int(c.intention), 0), 2)
        r = self._h.add_route(want, intent)
        self._custom.append((want.copy(), intent))
        self._route_ids[want.tobytes()] = r
        return r

    def set_state(self, s: EnvState):
        """cpp/IntersectionEnv.cpp:406-416; like the reference, the LiDAR objects
        are rebuilt with Lidar() defaults (72 rays) from here on."""
        self._agent_ids = list(s.agent_ids)
        self._next_id = int(s.next_agent_id)
        self._apply_state(s, CTOR_LIDAR)

    @cars.setter
    def cars(self, cars: Sequence[Car]):
        """IntersectionEnv.cars is read-write (cpp/bindings.cpp:66): the ego vector is replaced as given
        (state, path, hidden fields); the LiDAR configuration, agent ids, NPCs and step count stay."""
        s = self.get_state()
        s.cars = list(cars)
        n = len(s.cars)
        ids = list(self._agent_ids[:n])
        while len(ids) < n:  # (MARLEnv leaves agent_ids as they were; they index the egos here)
            ids.append(self._next_id)
            self._next_id += 1
        self._agent_ids = ids
        self._apply_state(s, self._lidar)

    @traffic_cars.setter
    def traffic_cars(self, cars: Sequence[Car]):
        """IntersectionEnv.traffic_cars is read-write (cpp/bindings.cpp:67): the NPC vector is replaced."""
        s = self.get_state()
        s.traffic_cars = list(cars)
        if self._routes or s.traffic_cars or self._ghost:
            self._apply_state(s, self._lidar)

    def _apply_state(self, s: EnvState, lidar):
        n = len(s.traffic_cars)
        if self._max_npcs < n <= 64:  # a written fleet beyond the handle's NPC slots: 64 slots (the ABI's limit)
            self._max_npcs = 64
            if self._h is not None:
                self._h.close()
            self._h, self._ghost = None, False
        n = len(s.cars)
        if n == 0:  # the cars vector emptied: the traffic and the step count stay (the no-ego handle)
            self._routes, self._pending = [], []
            if not s.traffic_cars and not s.step_count and not self._ghost:
                return
            self._sync_ghost(True)
            self._ghost_reset = False
        elif self._h is None or self._h.N != n or self._h_lidar != lidar or self._ghost:
            if self._h is not None:
                self._h.close()
            self._h = self._create(n, lidar)
            self._h_lidar = lidar
            self._ghost = False
        routes = [self._route_of(c) for c in s.cars]
        self._routes = routes
        if n:
            self._lidar = lidar
            if self._traffic_routes is not None:
                self._h.set_traffic_routes(self._traffic_routes)
            self._h.set_ego_routes(np.asarray(routes, np.int32)[None])
        st = self._h.get_state()
        for i, c in enumerate(s.cars):
            st["x"][0, i], st["y"][0, i], st["v"][0, i], st["heading"][0, i] = (c.state.x, c.state.y, c.state.v,
                                                                                 c.state.heading)
            st["acc"][0, i], st["steering"][0, i] = c.acc, c.steering_angle
            st["spawn_x"][0, i], st["spawn_y"][0, i] = c.spawn_state.x, c.spawn_state.y
            st["spawn_v"][0, i], st["spawn_heading"][0, i] = c.spawn_state.v, c.spawn_state.heading
            st["prev_dist"][0, i] = c.prev_dist_to_goal
            st["prev_a0"][0, i], st["prev_a1"][0, i] = c.prev_action
            st["path_index"][0, i], st["intention"][0, i] = c.path_index, c.intention
            st["alive"][0, i] = int(bool(c.alive))
            st["route"][0, i] = routes[i]
        k = len(s.traffic_cars)
        if k > self._h.K:
            raise ValueError(f"{k} traffic cars exceed max_npcs={self._h.K}")
        for j, c in enumerate(s.traffic_cars):
            st["npc_x"][0, j], st["npc_y"][0, j], st["npc_v"][0, j] = c.state.x, c.state.y, c.state.v
            st["npc_heading"][0, j], st["npc_acc"][0, j], st["npc_steering"][0, j] = (c.state.heading, c.acc,
                                                                                      c.steering_angle)
            st["npc_path_index"][0, j], st["npc_intention"][0, j] = c.path_index, c.intention
            st["npc_alive"][0, j] = int(bool(c.alive))
            st["npc_route"][0, j] = self._route_of(c)
        st["npc_count"][0] = k
        st["step_count"][0] = int(s.step_count)
        if n == 0:
            self._place_ghost(self._h, st)
        else:
            self._h.set_state(st)
        # Car::length / Car::width of every car (the reference copies them with the cars)
        ego_d = np.array([[[c.length, c.width] for c in s.cars]] if n else [[[54.0, 24.0]]], np.float32)
        npc_d = np.empty((1, self._h.K, 2), np.float32)
        npc_d[...] = (54.0, 24.0)
        if k:
            npc_d[0, :k] = [[c.length, c.width] for c in s.traffic_cars]
        if self._h.car_dims_active() or np.any(ego_d != (54.0, 24.0)) or np.any(npc_d != (54.0, 24.0)):
            self._h.set_car_dims(ego_d, npc_d)
        self._fresh = False
        self._pending = []

    # ---------------------------------------------- renderer (out of scope)
    def render(self, show_lane_ids: bool = False, show_lidar: bool = False):
        """The reference renderer is Windows/GLFW-only (Renderer.h:8-10); not provided."""
        return None

    def window_should_close(self) -> bool:
        return True

    def poll_events(self):
        return None

    def key_pressed(self, glfw_key: int) -> bool:
        return False

    def close(self):
        if self._h is not None:
            self._h.close()
            self._h = None
        self._ghost = False


# reference cpp_backend.py factories
_NO_EGO_XY = -1.0e5  # the no-ego handle's placeholder car (IntersectionEnv.__init__)


def _require():
    if not has_cpp_backend():
        raise RuntimeError("libmarlenv_hip.so is not built: run python -c 'import __graft_entry__ as g; g.build()'")
    return True
