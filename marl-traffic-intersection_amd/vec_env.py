"""Batched environment: E independent intersections advanced by one device
call per step (BASELINE north star; the reference steps one env per Python
call, reference env.py:152-195 / cpp/IntersectionEnv.cpp:133-392).

Two modes:
 * backend="torch": actions and outputs are CUDA (HIP) tensors on `device`;
   every step is one asynchronous launch pair ordered on torch's current
   stream, no host round trip.  The returned tensors are this env's output
   buffers and are overwritten by the next step (pass copy=True to clone).
 * backend="numpy": host arrays in and out (synchronous; for tests and
   small-scale use).

Per-agent semantics are exactly the reference's (bit-exact, see tests/);
auto_reset=True restarts an env in the step after it reported terminated or
truncated, which is what an RL rollout loop does with the reference env.

max_npcs (NPC slots per env, traffic mode) defaults to 32, the C ABI's default:
spawned traffic never holds more than 15 NPCs in one env (the reference's spawn
test, profiles/r6_fleet_probe.txt), and 32 slots run the compile-time one-ego
kernel (4096 envs at density 0.5: 159 M agent-steps/s against 75 M with 64
slots, profiles/r6_cfg4_k64.txt).  Pass max_npcs=64 to write up to 64 traffic
cars per env through set_state.
"""
from __future__ import annotations

from typing import Any, Dict, Optional, Sequence

import numpy as np

from . import _capi
from .utils import default_routes, point_index

_REWARD_ORDER = ("progress_scale", "stuck_speed_threshold", "stuck_penalty", "crash_vehicle_penalty",
                 "crash_object_penalty", "success_reward", "action_smoothness_scale", "team_alpha")
_REWARD_DEFAULT = (10.0, 1.0, -0.01, -10.0, -5.0, 10.0, -0.02, 0.2)


def reward_vector(reward_config) -> list:
    """env.py-style reward dict (or an 8-list in RewardConfig order) -> the C-ABI reward[8]."""
    if reward_config is None:
        return list(_REWARD_DEFAULT)
    if isinstance(reward_config, dict):
        return [float(reward_config.get(k, d)) for k, d in zip(_REWARD_ORDER, _REWARD_DEFAULT)]
    v = [float(x) for x in reward_config]
    if len(v) != 8:
        raise ValueError("reward_config must have 8 entries")
    return v


class VecIntersectionEnv:
    def __init__(self, num_envs: int, num_agents: int = 8, num_lanes: int = 3, lidar_rays: int = 96,
                 obs_dim: Optional[int] = None, use_team_reward: bool = False, respawn_enabled: bool = True,
                 max_steps: int = 2000, traffic_flow: bool = False, traffic_density: float = 0.5,
                 reward_config: Any = None, ego_routes: Optional[Sequence] = None, max_npcs: int = 32,
                 seed: int = 0, device: int = 0, backend: str = "torch", auto_reset: bool = True,
                 lidar_fov_deg: float = 360.0, lidar_max_dist: float = 250.0, lidar_step: float = 4.0):
        if backend not in ("torch", "numpy"):
            raise ValueError("backend must be 'torch' or 'numpy'")
        if traffic_flow and num_agents != 1:
            raise ValueError("traffic_flow mode has exactly one ego per env (reference env.py:84-87)")
        self.backend = backend
        self.auto_reset = bool(auto_reset)
        self.num_envs, self.num_agents, self.num_lanes = int(num_envs), int(num_agents), int(num_lanes)
        if obs_dim is None:
            obs_dim = 127 if lidar_rays <= 96 else 31 + lidar_rays
        self._h = _capi.Handle(num_envs=self.num_envs, num_agents=self.num_agents, num_lanes=self.num_lanes,
                               lidar_rays=int(lidar_rays), lidar_fov_deg=float(lidar_fov_deg),
                               lidar_max_dist=float(lidar_max_dist), lidar_step=float(lidar_step),
                               obs_dim=int(obs_dim), traffic_flow=int(bool(traffic_flow)),
                               traffic_density=float(traffic_density), use_team_reward=int(bool(use_team_reward)),
                               respawn_enabled=int(bool(respawn_enabled)), max_steps=int(max_steps),
                               reward=reward_vector(reward_config), max_npcs=int(max_npcs), seed=int(seed),
                               device=int(device))
        self.obs_dim = self._h.D
        self.device_index = int(device)
        if ego_routes is not None:
            self.set_ego_routes(ego_routes)
        self._stream = None
        self._out = None
        if backend == "torch":
            import torch
            self._torch = torch
            dev = torch.device("cuda", self.device_index)
            E, N, D = self.num_envs, self.num_agents, self.obs_dim
            self._out = dict(obs=torch.zeros((E, N, D), dtype=torch.float32, device=dev),
                             reward=torch.zeros((E, N), dtype=torch.float32, device=dev),
                             done=torch.zeros((E, N), dtype=torch.uint8, device=dev),
                             status=torch.zeros((E, N), dtype=torch.uint8, device=dev),
                             terminated=torch.zeros(E, dtype=torch.uint8, device=dev),
                             truncated=torch.zeros(E, dtype=torch.uint8, device=dev),
                             agents_alive=torch.zeros(E, dtype=torch.int32, device=dev),
                             step=torch.zeros(E, dtype=torch.int32, device=dev))
            self._bind_stream()
        else:
            self._out = self._h.alloc_outputs()

    # ----------------------------------------------------------------- utils
    @property
    def handle(self) -> _capi.Handle:
        return self._h

    def _bind_stream(self):
        s = self._torch.cuda.current_stream(self.device_index)
        if s.cuda_stream != self._stream:
            self._h.set_stream(s.cuda_stream)
            self._stream = s.cuda_stream

    def set_ego_routes(self, routes):
        """routes: [(start, end)] names per agent (same for every env), or an int array [E, N] of route ids."""
        if len(routes) and isinstance(routes[0], (tuple, list)) and isinstance(routes[0][0], str):
            P = 8 * self.num_lanes
            ids = []
            for s, e in routes:
                si, ei = point_index(s, self.num_lanes), point_index(e, self.num_lanes)
                if si < 0 or ei < 0:
                    raise IndexError(f"unknown lane id in route ({s!r}, {e!r})")
                ids.append(si * P + ei)
            routes = np.asarray(ids, np.int32)
        self._h.set_ego_routes(np.asarray(routes, np.int32))

    def set_reset_routes(self, routes):
        """Draw every agent's route from `routes` (names or ids) at each reset, as the
        reference test.py does with random.choice(all_routes); [] restores fixed routes."""
        ids = []
        P = 8 * self.num_lanes
        for r in routes:
            if isinstance(r, (tuple, list)):
                si, ei = point_index(r[0], self.num_lanes), point_index(r[1], self.num_lanes)
                if si < 0 or ei < 0:
                    raise IndexError(f"unknown lane id in route {tuple(r)!r}")
                ids.append(si * P + ei)
            else:
                ids.append(int(r))
        self._h.set_reset_routes(ids)

    def snapshot(self, out=None):
        """Whole-batch state + last outputs (torch: a device uint8 tensor; numpy: host bytes)."""
        if self.backend == "torch":
            self._bind_stream()
            if out is None:
                out = self._torch.empty(self._h.snapshot_size(), dtype=self._torch.uint8,
                                        device=self._out["obs"].device)
            self._h.snapshot(out, device=True)
            return out
        return self._h.snapshot(out)

    def restore(self, snap, env_mask=None):
        """Roll all envs (or those with env_mask != 0) back to `snap`; outputs follow."""
        if self.backend == "torch":
            self._bind_stream()
            mask = None
            if env_mask is not None:
                mask = self._torch.as_tensor(env_mask, device=self._out["obs"].device).to(self._torch.uint8)
                mask = mask.contiguous()
            self._h.restore(snap, env_mask=mask, device=True)
            self._h.get_outputs(self._out, device=True)
            return self._out["obs"]
        self._h.restore(snap, env_mask=env_mask)
        return self._h.get_outputs(self._out)["obs"]

    def set_traffic_routes(self, routes):
        """The NPC route list (reference configure_routes); names or route ids."""
        P = 8 * self.num_lanes
        ids = []
        for r in routes:
            if isinstance(r, (tuple, list)):
                si, ei = point_index(r[0], self.num_lanes), point_index(r[1], self.num_lanes)
                if si < 0 or ei < 0:
                    raise IndexError(f"unknown lane id in route {tuple(r)!r}")
                ids.append(si * P + ei)
            else:
                ids.append(int(r))
        self._h.set_traffic_routes(np.asarray(ids, np.int32))

    # ------------------------------------------------------------- episode
    def reset(self, env_mask=None):
        """Reset all envs (or those with env_mask != 0); returns the observation buffer."""
        if self.backend == "torch":
            self._bind_stream()
            mask = None
            if env_mask is not None:
                mask = self._torch.as_tensor(env_mask, device=self._out["obs"].device).to(self._torch.uint8)
                mask = mask.contiguous()
            self._h.reset(env_mask=mask, obs=self._out["obs"], device=True)
            return self._out["obs"]
        self._h.reset(env_mask=env_mask, obs=self._out["obs"])
        return self._out["obs"]

    def step(self, actions, dt: float = 1.0 / 60.0, copy: bool = False, spawn_route=None):
        """actions [E, N, 2] (throttle, steer) -> (obs, rewards, terminated, truncated, info)."""
        o = self._out
        if self.backend == "torch":
            t = self._torch
            self._bind_stream()
            a = actions
            if not (isinstance(a, t.Tensor) and a.is_cuda and a.dtype == t.float32 and a.is_contiguous()):
                a = t.as_tensor(a, dtype=t.float32, device=o["obs"].device).contiguous()
            if a.numel() != self.num_envs * self.num_agents * 2:
                raise ValueError(f"actions must be [{self.num_envs}, {self.num_agents}, 2], got {tuple(a.shape)}")
            if a.device.index != self.device_index:
                raise ValueError("actions are on another device")
            sp = None
            if spawn_route is not None:
                sp = t.as_tensor(spawn_route, dtype=t.int32, device=o["obs"].device).contiguous()
            self._h.step(a, float(dt), out=o, spawn_route=sp, auto_reset=self.auto_reset, device=True)
            if copy:
                o = {k: v.clone() for k, v in o.items()}
        else:
            self._h.step(actions, float(dt), out=o, spawn_route=spawn_route, auto_reset=self.auto_reset)
            if copy:
                o = {k: v.copy() for k, v in o.items()}
        info = {"done": o["done"], "status": o["status"], "agents_alive": o["agents_alive"], "step": o["step"]}
        return o["obs"], o["reward"], o["terminated"], o["truncated"], info

    def observations(self):
        return self._out["obs"]

    def get_state(self) -> Dict[str, np.ndarray]:
        if self.backend == "torch":
            self._torch.cuda.current_stream(self.device_index).synchronize()
        return self._h.get_state()

    def set_state(self, state: Dict[str, np.ndarray]):
        self._h.set_state(state)

    def close(self):
        if self._h is not None:
            self._h.close()
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def make_default_routes(num_agents: int, num_lanes: int):
    """Ego routes as env.py assigns them (mapping order, wrapping; reference env.py:138-145)."""
    table = default_routes(num_lanes)
    return [table[i % len(table)] for i in range(num_agents)]
