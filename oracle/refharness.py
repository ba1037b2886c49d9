"""TEST INFRASTRUCTURE ONLY: ctypes driver for $MEV_REF_BUILD/libref_harness.so.

The library is the UNMODIFIED reference simulator (cpp/*.cpp of the reference,
built in place by oracle/build_ref.sh) plus oracle/ref_harness.cpp.  The build
lives outside the repository (default /tmp/marl_ref_build), so it never travels
to the GPU box.  Only
tests/golden/gen_golden.py and bench.py's ``cpu_baseline`` leg use it.
"""
from __future__ import annotations

import ctypes
import os
from typing import Sequence

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF_BUILD = os.environ.get("MEV_REF_BUILD", "/tmp/marl_ref_build")
LIB_PATH = os.path.join(REF_BUILD, "libref_harness.so")

NF = 15  # float fields per car record (see ref_harness.cpp car_to_rec)
NI = 4   # int fields: alive, intention, path_index, route
OBS_W = 127

_lib = None


def available() -> bool:
    return os.path.exists(LIB_PATH)


def lib():
    global _lib
    if _lib is None:
        if not available():
            raise FileNotFoundError(f"{LIB_PATH} missing: run oracle/build_ref.sh (needs /root/reference)")
        L = ctypes.CDLL(LIB_PATH)
        vp, i, f = ctypes.c_void_p, ctypes.c_int, ctypes.c_float
        fp = ctypes.POINTER(ctypes.c_float)
        ip = ctypes.POINTER(ctypes.c_int32)
        L.rh_create.restype = vp
        L.rh_create.argtypes = [i]
        L.rh_destroy.argtypes = [vp]
        L.rh_configure.argtypes = [vp, i, i, i]
        L.rh_configure_traffic.argtypes = [vp, i, f]
        L.rh_configure_routes.argtypes = [vp, ctypes.c_char_p]
        L.rh_num_traffic_routes.argtypes = [vp]
        L.rh_set_reward.argtypes = [vp, fp]
        L.rh_set_lidar.argtypes = [vp, i, f, f, f]
        L.rh_set_car_lidar.argtypes = [vp, i, i, f, f, f, fp, i]
        L.rh_reset.argtypes = [vp]
        L.rh_state_roundtrip.argtypes = [vp]
        L.rh_add_car.argtypes = [vp, ctypes.c_char_p, ctypes.c_char_p, i]
        L.rh_num_cars.argtypes = [vp]
        L.rh_num_npcs.argtypes = [vp]
        L.rh_step_count.argtypes = [vp]
        L.rh_get_cars.argtypes = [vp, i, fp, ip]
        L.rh_set_car.argtypes = [vp, i, fp, ip]
        L.rh_add_npc.argtypes = [vp, i, fp, ip]
        L.rh_get_lidar.argtypes = [vp, fp]
        L.rh_route_path.argtypes = [vp, i, fp]
        L.rh_add_custom_path.argtypes = [vp, fp, i]
        L.rh_set_car_path.argtypes = [vp, i, i, i]
        L.rh_geometry_grid.argtypes = [i, ctypes.POINTER(ctypes.c_uint8)]
        L.rh_is_on_road.argtypes = [i, f, f]
        L.rh_hits_yellow_line.argtypes = [i, f, f]
        L.rh_get_obs.argtypes = [vp, fp]
        L.rh_step.argtypes = [vp, i, fp, fp, f, fp, fp, ip, ip, ip, ip]
        L.rh_bench.restype = ctypes.c_double
        L.rh_bench.argtypes = [i, i, i, i, i, f, i, i, i, ctypes.c_uint]
        _lib = L
    return _lib


def _f(a: np.ndarray):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_float))


def _i(a: np.ndarray):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_int32))


class RefEnv:
    """One reference IntersectionEnv driven at the C++ level."""

    def __init__(self, num_lanes=3, use_team=False, respawn=True, max_steps=2000,
                 traffic=False, density=0.5, routes: Sequence[tuple[str, str]] = (),
                 reward: Sequence[float] | None = None, rays=96, fov=360.0, max_dist=250.0, step=4.0):
        L = lib()
        self.h = L.rh_create(num_lanes)
        L.rh_configure(self.h, int(use_team), int(respawn), int(max_steps))
        L.rh_configure_traffic(self.h, int(traffic), float(density))
        if routes:
            spec = ";".join(f"{s} {e}" for s, e in routes)
            L.rh_configure_routes(self.h, spec.encode())
        if reward is not None:
            L.rh_set_reward(self.h, _f(np.asarray(reward, np.float32)))
        L.rh_set_lidar(self.h, int(rays), float(fov), float(max_dist), float(step))
        self.rays = int(rays)

    def close(self):
        if self.h:
            lib().rh_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def reset(self):
        lib().rh_reset(self.h)

    def state_roundtrip(self):
        """IntersectionEnv::set_state(get_state()): the LiDAR objects become default Lidar() (72 rays)."""
        lib().rh_state_roundtrip(self.h)
        self.rays = 72

    @property
    def step_count(self) -> int:
        return lib().rh_step_count(self.h)

    def add_car(self, start: str, end: str, tag: int = -1) -> int:
        return lib().rh_add_car(self.h, start.encode(), end.encode(), int(tag))

    @property
    def n(self) -> int:
        return lib().rh_num_cars(self.h)

    @property
    def k(self) -> int:
        return lib().rh_num_npcs(self.h)

    def cars(self, which=0):
        cnt = self.n if which == 0 else self.k
        f = np.zeros((max(cnt, 1), NF), np.float32)
        i = np.zeros((max(cnt, 1), NI), np.int32)
        lib().rh_get_cars(self.h, which, _f(f), _i(i))
        return f[:cnt].copy(), i[:cnt].copy()

    def set_car(self, k: int, f: np.ndarray, i: np.ndarray):
        f = np.ascontiguousarray(f, np.float32)
        i = np.ascontiguousarray(i, np.int32)
        lib().rh_set_car(self.h, int(k), _f(f), _i(i))

    def add_npc(self, route: int, f: np.ndarray, i: np.ndarray) -> int:
        f = np.ascontiguousarray(f, np.float32)
        i = np.ascontiguousarray(i, np.int32)
        return lib().rh_add_npc(self.h, int(route), _f(f), _i(i))

    def add_custom_path(self, path: np.ndarray) -> int:
        """A path of the caller's own (n x 2); returns its index (NPCs on it report route 1000 + index)."""
        a = np.ascontiguousarray(path, np.float32).reshape(-1, 2)
        return lib().rh_add_custom_path(self.h, _f(a), len(a))

    def set_car_path(self, which: int, k: int, custom: int):
        """Car.path = custom path `custom` (ego k: which 0, NPC k: which 1), as pybind's setter does."""
        if lib().rh_set_car_path(self.h, int(which), int(k), int(custom)) != 0:
            raise IndexError("bad car or custom path index")

    def set_car_lidar(self, k: int, rays: int, fov: float, max_dist: float, step: float, rel=None):
        """IntersectionEnv.lidars[k] = a Lidar() with these members written (cpp/bindings.cpp:85-92);
        rel=None keeps Lidar()'s own 72 beam offsets.  (lidar() then no longer applies: the
        cars' ray counts differ.)"""
        r = None if rel is None else np.ascontiguousarray(rel, np.float32)
        lib().rh_set_car_lidar(self.h, int(k), int(rays), float(fov), float(max_dist), float(step),
                               None if r is None else _f(r), 0 if r is None else int(r.size))
        self.mixed_lidar = True

    def route_path(self, route: int) -> np.ndarray:
        out = np.zeros((512, 2), np.float32)
        n = lib().rh_route_path(self.h, int(route), _f(out))
        return out[:n].copy()

    def obs(self) -> np.ndarray:
        out = np.zeros((max(self.n, 1), OBS_W), np.float32)
        lib().rh_get_obs(self.h, _f(out))
        return out[: self.n].copy()

    def lidar(self) -> np.ndarray:
        if getattr(self, "mixed_lidar", False):
            raise ValueError("per-car LiDAR configurations: raw distances are not one [n][rays] array")
        out = np.zeros((max(self.n, 1), self.rays), np.float32)
        lib().rh_get_lidar(self.h, _f(out))
        return out[: self.n].copy()

    def step(self, actions: np.ndarray, dt: float = 1.0 / 60.0):
        a = np.ascontiguousarray(actions, np.float32).reshape(-1, 2)
        thr = np.ascontiguousarray(a[:, 0])
        st = np.ascontiguousarray(a[:, 1])
        n = self.n
        obs = np.zeros((max(n, 1), OBS_W), np.float32)
        rew = np.zeros(max(n, 1), np.float32)
        done = np.zeros(max(n, 1), np.int32)
        status = np.zeros(max(n, 1), np.int32)
        flags = np.zeros(4, np.int32)
        spawned = np.zeros(1, np.int32)
        r = lib().rh_step(self.h, len(thr), _f(thr), _f(st), float(dt), _f(obs), _f(rew), _i(done),
                          _i(status), _i(flags), _i(spawned))
        if r < 0:
            raise RuntimeError(f"rh_step failed ({r})")
        return dict(obs=obs[:n], rew=rew[:n], done=done[:n], status=status[:n],
                    terminated=int(flags[0]), truncated=int(flags[1]), agents_alive=int(flags[2]),
                    step=int(flags[3]), spawned=int(spawned[0]))


def geometry_grid(num_lanes: int) -> np.ndarray:
    out = np.zeros((750, 750), np.uint8)
    lib().rh_geometry_grid(int(num_lanes), out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)))
    return out


def bench(num_agents: int, rays: int, use_team: bool, traffic: bool, density: float,
          envs_per_thread: int, steps: int, threads: int, seed: int = 0) -> float:
    """Reference C++ throughput in agent-steps/s (see rh_bench)."""
    return float(lib().rh_bench(3, int(num_agents), int(rays), int(use_team), int(traffic), float(density),
                                int(envs_per_thread), int(steps), int(threads), int(seed)))
