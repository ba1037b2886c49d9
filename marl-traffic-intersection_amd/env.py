"""Gym-style wrapper with the reference's env.py API (reference env.py:80-205).

Same config keys, same return shapes and the same info dict; the simulation
behind it is the GPU backend in cpp_backend.py (one env on the device).  For
thousands of envs per call use vec_env.VecIntersectionEnv instead — this
class exists so that code written against the reference runs unchanged.

Multi-agent mode: reset() -> (obs [N,127], {}); step() -> (obs [N,127],
rewards [N], terminated, truncated, info).  traffic_flow mode (one ego among
NPCs): obs [127] and a float reward.
"""
from __future__ import annotations

from typing import Any, Dict, List, Optional

import numpy as np

from . import cpp_backend
from .utils import DEFAULT_REWARD_CONFIG, build_lane_layout, default_routes

# config.reward_config key -> RewardConfig field (reference env.py:57-77)
_REWARD_KEYS = {
    "progress_scale": "k_prog",
    "stuck_speed_threshold": "v_min_ms",
    "stuck_penalty": "k_stuck",
    "crash_vehicle_penalty": "k_cv",
    "crash_object_penalty": "k_co",
    "success_reward": "k_succ",
    "action_smoothness_scale": "k_sm",
    "team_alpha": "alpha",
}


def _apply_reward_config(env: Any, reward_cfg: Dict[str, Any]) -> None:
    rc = getattr(env, "reward_config", None)
    if rc is None:
        return
    for key, field in _REWARD_KEYS.items():
        if key in reward_cfg:
            setattr(rc, field, float(reward_cfg[key]))


class IntersectionEnv:
    def __init__(self, config: Optional[Dict[str, Any]] = None):
        cfg = dict(config or {})
        self.traffic_flow = bool(cfg.get("traffic_flow", False))
        self.num_agents = 1 if self.traffic_flow else int(cfg.get("num_agents", 1))
        self.num_lanes = int(cfg.get("num_lanes", 3))
        self.render_mode = cfg.get("render_mode")
        self.show_lane_ids = bool(cfg.get("show_lane_ids", False))
        self.show_lidar = bool(cfg.get("show_lidar", False))
        team = bool(cfg.get("use_team_reward", DEFAULT_REWARD_CONFIG["use_team_reward"])) and not self.traffic_flow
        respawn = bool(cfg.get("respawn_enabled", True))
        max_steps = int(cfg.get("max_steps", 2000))

        routes = cfg.get("ego_routes")
        self.ego_routes = routes if routes is not None else self._default_routes(self.num_agents, self.num_lanes)
        self.lane_layout = build_lane_layout(self.num_lanes)
        self.points = self.lane_layout["points"]

        self.env = cpp_backend.IntersectionEnv(self.num_lanes, device=int(cfg.get("device", 0)))
        self.env.configure(team, respawn, max_steps)
        self.traffic_density = float(cfg.get("traffic_density", 0.5))
        try:  # the reference ignores failures here (env.py:115-124)
            self.env.configure_traffic(self.traffic_flow, self.traffic_density)
            self.env.configure_routes(default_routes(self.num_lanes))
        except Exception:
            pass

        reward_cfg = cfg.get("reward_config")
        if reward_cfg is None:
            reward_cfg = DEFAULT_REWARD_CONFIG["reward_config"]
        if isinstance(reward_cfg, dict):
            _apply_reward_config(self.env, reward_cfg)

        self.cars: List[cpp_backend.Car] = []
        self.traffic_cars: List[cpp_backend.Car] = []
        self.reset()

    @staticmethod
    def _default_routes(num_agents: int, num_lanes: int):
        table = default_routes(num_lanes)
        return [table[i % len(table)] for i in range(num_agents)]

    def reset(self):
        self.env.reset()
        for start, end in self.ego_routes[: self.num_agents]:
            self.env.add_car_with_route(start, end)
        self.cars = self.env.cars
        self._traffic_cars = None  # read from the device on first access (traffic_cars)
        obs = np.asarray(self.env.get_observations(), np.float32)
        return (obs[0], {}) if self.traffic_flow else (obs, {})

    def _coerce_actions(self, actions) -> np.ndarray:
        a = np.asarray(actions, np.float32)
        if self.traffic_flow:
            return a.reshape(1, 2)
        if a.ndim == 1:
            if a.size == 2 and self.num_agents == 1:
                return a.reshape(1, 2)
            raise ValueError(f"Expected actions shape (N,2) for multi-agent, got {a.shape}")
        return a

    def step(self, actions, dt: float = 1.0 / 60.0):
        a = self._coerce_actions(actions)
        res = self.env.step(a[:, 0], a[:, 1], float(dt))
        self._traffic_cars = None  # read from the device on first access (traffic_cars)
        obs = np.asarray(res.obs, np.float32)
        rewards = np.asarray(res.rewards, np.float32)
        first = float(rewards[0]) if len(rewards) else 0.0
        info = {
            "step": int(res.step),
            "rewards": first if self.traffic_flow else rewards.tolist(),
            "collisions": {int(aid): str(st) for aid, st in zip(res.agent_ids, res.status)},
            "agents_alive": int(res.agents_alive),
            "terminated": bool(res.terminated),
            "truncated": bool(res.truncated),
            "done": list(res.done),
            "status": list(res.status),
        }
        if self.traffic_flow:
            return obs[0], first, info["terminated"], info["truncated"], info
        return obs, rewards, info["terminated"], info["truncated"], info

    # The reference refreshes self.traffic_cars after every reset and step (env.py:155-157,
    # :184-186: a copy of the C++ Car list).  Here the list is built when it is first read
    # after a step -- the same cars, since nothing else moves them in between -- so a
    # training loop that never looks at the NPCs does not pay a device read-back per step.
    @property
    def traffic_cars(self) -> List[cpp_backend.Car]:
        if self._traffic_cars is None:
            try:
                self._traffic_cars = list(self.env.traffic_cars) if self.traffic_flow else []
            except Exception:  # (the reference's fallback)
                self._traffic_cars = []
        return self._traffic_cars

    @traffic_cars.setter
    def traffic_cars(self, cars):
        self._traffic_cars = cars

    def render(self, show_lane_ids: Optional[bool] = None, show_lidar: Optional[bool] = None):
        """The reference opens a GLFW window (Windows-only, Renderer.cpp).  Here
        render_mode "rgb_array" returns a frame from the headless debug renderer
        (render.py); any other mode is a no-op."""
        if self.render_mode != "rgb_array":
            return None
        from . import render as _render
        h = self.env._sync()
        if h is None:
            return None
        return _render.render(h, 0, show_lidar=self.show_lidar if show_lidar is None else bool(show_lidar))

    def close(self):
        self.env.close()
