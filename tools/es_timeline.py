"""Diagnostic: wall-clock timeline of the early split (k_step ESPLIT, mev_set_step_split(3)) from
the stampses build (s_memrealtime, 100 MHz): car wave entry / kinematics end / barrier B / end and
LiDAR wave poses ready / road-march end / B passed / end, per env.
    MEV_LIB_VARIANT=stampses python tools/es_timeline.py [--envs 4096 --agents 8 --rays 64]
Prints percentiles in microseconds relative to the step's first car-wave entry."""
import argparse
import os
import sys

os.environ.setdefault("MEV_LIB_VARIANT", "stampses")
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

import pkgload  # noqa: E402

NAMES = ["car entry", "car kinematics end", "car barrier B", "car end", "lidar poses ready", "lidar road end",
         "lidar B passed", "lidar end"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=4096)
    ap.add_argument("--steps", type=int, default=60)
    ap.add_argument("--agents", type=int, default=8)
    ap.add_argument("--rays", type=int, default=64)
    a = ap.parse_args()
    mev = pkgload.load()
    h = mev.Handle(num_envs=a.envs, num_agents=a.agents, lidar_rays=a.rays, use_team_reward=int(a.agents > 1))
    h.set_step_kernel(2)
    h.set_step_pack(1)
    h.set_step_split(3)
    assert h.step_split() == 2, "the early split does not apply to this shape"
    rng = np.random.default_rng(0)
    rows = []
    for t in range(a.steps):
        h.step(rng.uniform(-1, 1, (a.envs, a.agents, 2)).astype(np.float32), auto_reset=True)
        if t >= a.steps // 2:
            rows.append(h.debug_stamps().astype(np.int64).reshape(a.envs, 8))
    q = (0, 10, 50, 90, 100)
    print(f"envs={a.envs} agents={a.agents} rays={a.rays}: us after the first car-wave entry "
          f"(p0 / p10 / p50 / p90 / p100)")
    for k, n in enumerate(NAMES):
        v = np.concatenate([(r[:, k] - r[:, 0].min()) / 100.0 for r in rows])
        print(f"  {n:18s} " + " ".join(f"{np.percentile(v, x):7.2f}" for x in q))
    print("per-env spans:")
    for lab, i, j in (("car kinematics", 0, 1), ("car rest of cars_pre + B", 1, 2), ("cars_post (B->end)", 2, 3),
                      ("lidar entry->poses", 0, 4), ("road march", 4, 5), ("wait for B", 5, 6),
                      ("redo+phase3+writes", 6, 7),
                      ("car wave life", 0, 3), ("env (entry->lidar end)", 0, 7)):
        d = np.concatenate([(r[:, j] - r[:, i]) / 100.0 for r in rows])
        print(f"  {lab:24s} " + " ".join(f"{np.percentile(d, x):7.2f}" for x in q))
    h.close()


if __name__ == "__main__":
    main()
