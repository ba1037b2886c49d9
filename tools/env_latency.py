"""Single-env step latency through the drop-in APIs (config 1: 1 env x 1 agent x
16 beams, random actions), the reference user's path: env.py's
IntersectionEnv.step (numpy in/out, one step per call, synchronous) and the
raw C-ABI host path (Handle.step with numpy buffers), on both kernel paths.
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=3000)
    a = ap.parse_args()
    mev = pkgload.load()
    from marl_traffic_intersection_amd import env as envmod
    rng = np.random.default_rng(0)
    res = {}
    acts = rng.uniform(-1, 1, (a.steps, 1, 2)).astype(np.float32)
    e = envmod.IntersectionEnv({"num_agents": 1, "traffic_flow": False})  # the reference's 96-ray LiDAR
    for t in range(200):
        e.step(acts[t])
    t0 = time.perf_counter()
    for t in range(a.steps):
        e.step(acts[t])
    dt = (time.perf_counter() - t0) / a.steps
    res["env.py (1 agent, 96 beams)"] = round(1.0 / dt, 1)
    e.close()
    # config 1's shape through env.py: 16 beams set through the bound Lidar objects,
    # as the survey's reference measurement did
    from marl_traffic_intersection_amd import cpp_backend
    e = envmod.IntersectionEnv({"num_agents": 1, "traffic_flow": False})
    e.env.lidars = [cpp_backend.Lidar(rays=16)]
    for t in range(200):
        e.step(acts[t])
    t0 = time.perf_counter()
    for t in range(a.steps):
        e.step(acts[t])
    dt = (time.perf_counter() - t0) / a.steps
    res["env.py (1 agent, 16 beams; reference 54,869 in the survey container)"] = round(1.0 / dt, 1)
    e.close()
    for kernel in (0, 1, 2):
        hh = mev.Handle(num_envs=1, num_agents=1, lidar_rays=16)
        if kernel:
            hh.set_step_kernel(kernel)
        out = hh.alloc_outputs()
        for t in range(200):
            hh.step(acts[t], out=out, auto_reset=True)
        t0 = time.perf_counter()
        for t in range(a.steps):
            hh.step(acts[t], out=out, auto_reset=True)
        dt = (time.perf_counter() - t0) / a.steps
        res[f"Handle.step numpy kernel={kernel or 'auto'} ({hh.step_kernel()})"] = round(1.0 / dt, 1)
        hh.close()
    print(json.dumps({"unit": "steps/s (= agent-steps/s, 1 agent)", "steps": a.steps, **res}, indent=1))


if __name__ == "__main__":
    main()
