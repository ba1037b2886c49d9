"""Diagnostic: where a fused step's wave spends its time (stampsq build: eight s_memtime stamps
held in LDS -- no global store, no wave barrier -- written out at the end of the kernel).
Per env: entry -> loads consumed -> NPC phase -> phase 1 (kinematics, status) -> rest of cars_pre
-> cars_post up to the observation head -> the head -> LiDAR; medians by the env's NPC count.
    MEV_LIB_VARIANT=stampsq python tools/qstamp_profile.py [--agents 1 --traffic 0.5 --warmup 600]"""
import argparse
import os
import sys

os.environ.setdefault("MEV_LIB_VARIANT", "stampsq")
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

import pkgload  # noqa: E402

PARTS = ["loads", "npc phase", "phase 1", "rest of cars_pre", "cars_post to head", "obs head", "lidar"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=4096)
    ap.add_argument("--agents", type=int, default=1)
    ap.add_argument("--rays", type=int, default=64)
    ap.add_argument("--traffic", type=float, default=0.5)
    ap.add_argument("--warmup", type=int, default=600)
    ap.add_argument("--steps", type=int, default=60)
    ap.add_argument("--split", type=int, default=0, help="mev_set_step_split mode (3: the traffic early split; "
                    "its car waves' last part is the deal append, not the LiDAR)")
    a = ap.parse_args()
    mev = pkgload.load()
    h = mev.Handle(num_envs=a.envs, num_agents=a.agents, lidar_rays=a.rays, use_team_reward=int(a.agents > 1),
                   traffic_flow=int(a.traffic > 0), traffic_density=a.traffic, max_npcs=32)
    h.set_step_kernel(2)
    if a.split:
        h.set_step_split(a.split)
    rng = np.random.default_rng(0)
    for t in range(a.warmup):
        h.step(rng.uniform(-1, 1, (a.envs, a.agents, 2)).astype(np.float32), auto_reset=True)
    D, K = [], []
    for t in range(a.steps):
        h.step(rng.uniform(-1, 1, (a.envs, a.agents, 2)).astype(np.float32), auto_reset=True)
        s = h.debug_stamps().astype(np.int64)
        D.append(np.diff(s, axis=1))
        K.append(h.get_state()["npc_count"].copy() if a.traffic > 0 else np.zeros(a.envs, np.int64))
    d = np.concatenate(D)
    k = np.concatenate(K)
    tot = d.sum(1)
    print(f"envs={a.envs} agents={a.agents} rays={a.rays} traffic={a.traffic}: wave median {np.median(tot):.0f} "
          f"cycles (s_memtime)")
    print("  part                    median     mean  share   | median by NPCs after the step: " +
          " ".join(f"{q:>6d}" for q in np.unique(k)))
    for j, name in enumerate(PARTS):
        row = " ".join(f"{np.median(d[k == q, j]):6.0f}" for q in np.unique(k))
        print(f"  {name:20s} {np.median(d[:, j]):8.0f} {d[:, j].mean():8.0f} {d[:, j].sum() / tot.sum():6.1%}   | {row}")
    print("  envs by NPCs: " + " ".join(f"{q}:{int((k == q).sum()) // a.steps}" for q in np.unique(k)))


if __name__ == "__main__":
    main()
