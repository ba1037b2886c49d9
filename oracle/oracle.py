"""TEST INFRASTRUCTURE ONLY: ctypes driver for the plain-C restatement
(oracle/marl_oracle.c -> oracle/_build/libmarl_oracle.so).

Imported only by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
fallback — as the checker / baseline, never as the product path.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(HERE, "marl_oracle.c")
LIB = os.path.join(HERE, "_build", "libmarl_oracle.so")

CAR_DTYPE = np.dtype([(n, np.float32) for n in ("x", "y", "v", "h", "acc", "steer", "sx", "sy", "sv", "sh",
                                                 "prev_dist", "pa0", "pa1")] +
                     [(n, np.int32) for n in ("path_index", "route", "intention", "alive")] +
                     [(n, np.float32) for n in ("len", "wid")])  # Car::length / width (Car.h:19-20)


def new_cars(n: int) -> np.ndarray:
    """n zeroed car records of the reference's default size (54 x 24 px, Car.h:19-20)."""
    c = np.zeros(n, CAR_DTYPE)
    c["len"], c["wid"] = 54.0, 24.0
    return c

_lib = None


def build(force: bool = False) -> str:
    if not force and os.path.exists(LIB) and os.path.getmtime(LIB) >= os.path.getmtime(SRC):
        return LIB
    os.makedirs(os.path.dirname(LIB), exist_ok=True)
    # plain x86-64 SSE build, no FMA contraction: rounds exactly like the reference build
    cmd = ["gcc", "-O2", "-std=c11", "-ffp-contract=off", "-fPIC", "-shared", SRC, "-o", LIB + ".tmp", "-lm"]
    subprocess.run(cmd, check=True, capture_output=True)
    os.replace(LIB + ".tmp", LIB)
    return LIB


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        L = ctypes.CDLL(LIB)
        vp, i, f = ctypes.c_void_p, ctypes.c_int, ctypes.c_float
        L.orc_create.restype = vp
        L.orc_create.argtypes = [i, i, i, f, f, f, i, i, i, i, i, f, vp, i]
        L.orc_destroy.argtypes = [vp]
        L.orc_route_id.argtypes = [vp, i, i]
        L.orc_num_points.argtypes = [vp]
        L.orc_route_path.argtypes = [vp, i, vp, vp]
        L.orc_set_traffic_routes.argtypes = [vp, vp, i]
        L.orc_set_rel_angles.argtypes = [vp, vp]
        L.orc_add_route.argtypes = [vp, vp, i, i]
        L.orc_route_len.argtypes = [vp, i]
        L.orc_reset.argtypes = [vp, vp]
        L.orc_set_state.argtypes = [vp, vp, vp, i, i]
        L.orc_get_state.argtypes = [vp, vp, vp, vp, vp]
        L.orc_observe.argtypes = [vp, vp]
        L.orc_step.argtypes = [vp, vp, f, i, vp, vp, vp, vp, vp]
        L.orc_bench.restype = ctypes.c_double
        L.orc_bench.argtypes = [i, i, i, i, ctypes.c_uint]
        assert L.orc_sizeof_car() == CAR_DTYPE.itemsize
        _lib = L
    return _lib


class OracleEnv:
    """One environment of the C restatement."""

    def __init__(self, num_lanes=3, n_agents=1, rays=96, fov=360.0, max_dist=250.0, step=4.0, obs_dim=0,
                 use_team=False, respawn=True, max_steps=2000, traffic=False, density=0.5, reward=None, max_npcs=32):
        L = lib()
        rc = np.asarray(reward if reward is not None else [10.0, 1.0, -0.01, -10.0, -5.0, 10.0, -0.02, 0.2], np.float32)
        self.h = L.orc_create(num_lanes, n_agents, rays, fov, max_dist, step, obs_dim, int(use_team), int(respawn),
                              max_steps, int(traffic), density, rc.ctypes.data, max_npcs)
        if not self.h:
            raise ValueError("bad oracle configuration")
        self.n = n_agents
        self.rays = rays
        self.D = obs_dim if obs_dim > 0 else 31 + rays
        self.max_npcs = max_npcs
        self.P = L.orc_num_points(self.h)

    def close(self):
        if self.h:
            lib().orc_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def route_id(self, s, e):
        return lib().orc_route_id(self.h, int(s), int(e))

    def route_path(self, r):
        """(path [n, 2], intent) of route r (n = 160 for the lane-layout routes)."""
        out = np.zeros((lib().orc_route_len(self.h, int(r)), 2), np.float32)
        it = ctypes.c_int()
        lib().orc_route_path(self.h, int(r), out.ctypes.data, ctypes.addressof(it))
        return out, it.value

    def add_route(self, path, intent):
        """A written Car.path of n points, 2 <= n <= 4096 (cpp/bindings.cpp:29)."""
        a = np.ascontiguousarray(path, np.float32).reshape(-1, 2)
        r = lib().orc_add_route(self.h, a.ctypes.data, len(a), int(intent))
        if r < 0:
            raise ValueError("orc_add_route: 2 .. 4096 points")
        return r

    def set_rel_angles(self, rel):
        """Lidar::rel_angles[0 .. rays) (cpp/bindings.cpp:91)."""
        a = np.ascontiguousarray(np.asarray(rel, np.float32)[: self.rays])
        assert a.size == self.rays
        lib().orc_set_rel_angles(self.h, a.ctypes.data)

    def set_traffic_routes(self, ids):
        a = np.ascontiguousarray(ids, np.int32)
        lib().orc_set_traffic_routes(self.h, a.ctypes.data, len(a))

    def reset(self, routes):
        a = np.ascontiguousarray(routes, np.int32)
        lib().orc_reset(self.h, a.ctypes.data)

    def set_state(self, egos, npcs, step_count=0):
        e = np.ascontiguousarray(egos, CAR_DTYPE)
        n = np.ascontiguousarray(npcs, CAR_DTYPE) if len(npcs) else np.zeros(1, CAR_DTYPE)
        lib().orc_set_state(self.h, e.ctypes.data, n.ctypes.data, len(npcs), int(step_count))

    def get_state(self):
        e = np.zeros(self.n, CAR_DTYPE)
        n = np.zeros(max(1, 256), CAR_DTYPE)
        k = ctypes.c_int()
        sc = ctypes.c_int()
        lib().orc_get_state(self.h, e.ctypes.data, n.ctypes.data, ctypes.addressof(k), ctypes.addressof(sc))
        return e, n[: k.value].copy(), sc.value

    def observe(self):
        obs = np.zeros((self.n, self.D), np.float32)
        lib().orc_observe(self.h, obs.ctypes.data)
        return obs

    def step(self, actions, dt=1.0 / 60.0, spawn_route=-1):
        a = np.ascontiguousarray(actions, np.float32).reshape(-1)
        obs = np.zeros((self.n, self.D), np.float32)
        rew = np.zeros(self.n, np.float32)
        done = np.zeros(self.n, np.uint8)
        st = np.zeros(self.n, np.uint8)
        fl = np.zeros(4, np.int32)
        lib().orc_step(self.h, a.ctypes.data, float(dt), int(spawn_route), obs.ctypes.data, rew.ctypes.data,
                       done.ctypes.data, st.ctypes.data, fl.ctypes.data)
        return dict(obs=obs, rew=rew, done=done, status=st, terminated=int(fl[0]), truncated=int(fl[1]),
                    agents_alive=int(fl[2]), step=int(fl[3]))


def bench(n_agents: int, rays: int, use_team: bool, steps: int, seed: int = 0) -> float:
    """Single-thread agent-steps/s of the C restatement (cpu_baseline fallback)."""
    return float(lib().orc_bench(int(n_agents), int(rays), int(use_team), int(steps), int(seed)))
