"""Single-env step latency through the drop-in APIs (config 1: 1 env x 1 agent x
16 beams, random actions), the reference user's path: env.py's
IntersectionEnv.step (numpy in/out, one step per call, synchronous) and the
raw C-ABI host path (Handle.step with numpy buffers), on both kernel paths, each
with the persistent step server (mev_set_serve) on and off; plus the survey's
other single-env shapes through env.py.
    python tools/env_latency.py [--steps 3000]"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

import pkgload  # noqa: E402


def _time_env(envmod, cfg, acts, steps, serve, rays=None):
    from marl_traffic_intersection_amd import cpp_backend
    e = envmod.IntersectionEnv(cfg)
    if rays is not None:  # set through the bound Lidar objects, as the survey's reference measurement did
        e.env.lidars = [cpp_backend.Lidar(rays=rays) for _ in range(max(1, cfg.get("num_agents", 1)))]
    n = 1 if cfg.get("traffic_flow") else cfg.get("num_agents", 1)
    e.step(acts[0][:n])
    e.env._sync().set_serve(serve)
    for t in range(200):
        e.step(acts[t][:n])
    t0 = time.perf_counter()
    for t in range(steps):
        e.step(acts[t][:n])
    dt = (time.perf_counter() - t0) / steps
    stats = e.env._sync().serve_stats()
    e.close()
    return round(1.0 / dt, 1), stats


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=3000)
    a = ap.parse_args()
    mev = pkgload.load()
    from marl_traffic_intersection_amd import env as envmod
    rng = np.random.default_rng(0)
    res = {}
    acts = rng.uniform(-1, 1, (a.steps + 200, 8, 2)).astype(np.float32)
    # env.py, one env per call (the reference user's path); reference figures: BASELINE.md
    shapes = [
        ("1 agent, 16 beams (cfg1; reference 54,869)", {"num_agents": 1, "traffic_flow": False}, 16),
        ("1 agent, 96 beams (the reference's default LiDAR)", {"num_agents": 1, "traffic_flow": False}, None),
        ("1 agent, 64 beams (cfg2 shape; reference 24,370)", {"num_agents": 1, "traffic_flow": False}, 64),
        ("8 agents, team, 64 beams (cfg3 shape; reference 6,668)",
         {"num_agents": 8, "traffic_flow": False, "use_team_reward": True}, 64),
        ("8 agents, 96 beams (the reference's default LiDAR)", {"num_agents": 8, "traffic_flow": False}, None),
        ("traffic 0.5, 64 beams (cfg4 shape; reference 15,120)",
         {"num_agents": 1, "traffic_flow": True, "traffic_density": 0.5}, 64),
    ]
    for name, cfg, rays in shapes:
        for serve in (1, 0):
            v, st = _time_env(envmod, cfg, acts, a.steps, serve, rays)
            res[f"env.py {name}, server {'on' if serve else 'off'}"] = v
            if serve:
                res[f"env.py {name}, server stats"] = st
    for kernel in (0, 1, 2):
        for serve in ((1, 0) if kernel != 1 else (0,)):
            hh = mev.Handle(num_envs=1, num_agents=1, lidar_rays=16)
            if kernel:
                hh.set_step_kernel(kernel)
            hh.set_serve(serve)
            out = hh.alloc_outputs()
            for t in range(200):
                hh.step(acts[t][:1], out=out, auto_reset=True)
            t0 = time.perf_counter()
            for t in range(a.steps):
                hh.step(acts[t][:1], out=out, auto_reset=True)
            dt = (time.perf_counter() - t0) / a.steps
            res[f"Handle.step numpy 1x1x16 kernel={kernel or 'auto'} ({hh.step_kernel()}) server "
                f"{'on' if serve else 'off'}"] = round(1.0 / dt, 1)
            hh.close()
    print(json.dumps({"unit": "steps/s (= env-steps/s; agent-steps/s = x agents)", "steps": a.steps, **res},
                     indent=1))


if __name__ == "__main__":
    main()
