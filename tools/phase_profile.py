"""Diagnostic: per-phase cycle shares of the step kernel (stamps build).

Builds/loads libmarlenv_hip_stamps.so (-DMEV_STAMPS: s_memtime at each phase
boundary of k_cars, lane 0 of every env) and prints median / mean cycles per
phase.  Shares only — the stamps' barriers perturb the schedule, so the
absolute length of this build is not the product kernel's.
    MEV_LIB_VARIANT=stamps python tools/phase_profile.py [--envs 4096 --agents 8 --rays 64 --traffic 0]
"""
import argparse
import os
import sys

os.environ.setdefault("MEV_LIB_VARIANT", "stamps")
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

import pkgload  # noqa: E402

PHASES = ["npc", "physics+status", "SAT", "resolve+respawn+writeback", "obstacles+candidates", "obs head"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=4096)
    ap.add_argument("--agents", type=int, default=8)
    ap.add_argument("--rays", type=int, default=64)
    ap.add_argument("--traffic", type=int, default=0)
    ap.add_argument("--density", type=float, default=0.5)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--step-kernel", type=int, default=0, help="0 auto, 1 k_cars + k_lidar, 2 fused k_step")
    args = ap.parse_args()
    mev = pkgload.load()
    h = mev.Handle(num_envs=args.envs, num_agents=args.agents, lidar_rays=args.rays, use_team_reward=1,
                   traffic_flow=args.traffic, traffic_density=args.density)
    h.set_step_kernel(args.step_kernel)
    rng = np.random.default_rng(0)
    acc = []
    for t in range(args.steps):
        a = rng.uniform(-1, 1, (args.envs, args.agents, 2)).astype(np.float32)
        h.step(a, auto_reset=True)
        if t >= args.steps // 2:
            s = h.debug_stamps().astype(np.int64)
            acc.append(np.diff(s[:, :7], axis=1))
    d = np.concatenate(acc)
    tot = d.sum(1)
    print(f"envs={args.envs} agents={args.agents} rays={args.rays} traffic={args.traffic}: "
          f"total per env median {np.median(tot):.0f} cycles")
    for k, name in enumerate(PHASES):
        print(f"  {name:24s} median {np.median(d[:, k]):9.0f}  mean {d[:, k].mean():9.0f}  share {d[:, k].sum() / tot.sum():6.1%}")


if __name__ == "__main__":
    main()
