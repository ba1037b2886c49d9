"""Diagnostic: wall-clock timeline of one step (stampsr build, s_memrealtime at
100 MHz): k_cars wave entry / after its state loads / end per env, and the LiDAR
pools' entry / end of the car phase (two pools per env: k_lidar G = 4; one: k_step G = 8).
    MEV_LIB_VARIANT=stampsr python tools/timeline.py [--step-kernel 1|2]
Prints percentiles in microseconds relative to the first k_cars wave entry."""
import argparse
import os
import sys

os.environ.setdefault("MEV_LIB_VARIANT", "stampsr")
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

import pkgload  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=4096)
    ap.add_argument("--steps", type=int, default=60)
    ap.add_argument("--step-kernel", type=int, default=0)
    ap.add_argument("--agents", type=int, default=8)
    ap.add_argument("--rays", type=int, default=64)
    a = ap.parse_args()
    mev = pkgload.load()
    h = mev.Handle(num_envs=a.envs, num_agents=a.agents, lidar_rays=a.rays, use_team_reward=int(a.agents > 1))
    h.set_step_kernel(a.step_kernel)
    fused = h.step_kernel() == 2
    rng = np.random.default_rng(0)
    rows = []
    for t in range(a.steps):
        h.step(rng.uniform(-1, 1, (a.envs, a.agents, 2)).astype(np.float32), auto_reset=True)
        if t >= a.steps // 2:
            st = h.debug_stamps().astype(np.int64).reshape(a.envs, 8)
            st[:, 7] &= (1 << 40) - 1  # slot 7 carries HW_ID above bit 40
            pk = h.step_pack()
            rows.append(st[::pk] if pk > 1 else st)  # several envs per wave: the wave's first env holds its stamps
    names = ["cars entry", "cars loaded", "cars end", "lidar entry pool0", "lidar entry pool1", "lidar cars-phase end pool0",
             "lidar cars-phase end pool1"]
    if fused:  # one pool per env: slots 4 / 6 are its phase-1 / phase-2 ends
        names[4], names[6] = "lidar phase-1 end", "lidar phase-2 end"
    acc = {n: [] for n in names}
    for r in rows:
        t0 = r[:, 0].min()
        for k, n in enumerate(names):
            acc[n].append((r[:, k] - t0) / 100.0)  # 100 MHz ticks -> us
    print(f"envs={a.envs} step kernel={h.step_kernel()}: us after the first k_cars wave entry (p0 / p10 / p50 / p90 / p100)")
    for n in names:
        v = np.concatenate(acc[n])
        print(f"  {n:26s} " + " ".join(f"{np.percentile(v, q):7.2f}" for q in (0, 10, 50, 90, 100)))
    d = np.concatenate([(r[:, 2] - r[:, 0]) / 100.0 for r in rows])
    print(f"  k_cars wave lifetime       " + " ".join(f"{np.percentile(d, q):7.2f}" for q in (0, 10, 50, 90, 100)))
    if fused:
        for lab, i, j in (("lidar phase 1", 3, 4), ("lidar phase 2", 4, 6), ("lidar phase 3", 6, 5)):
            d = np.concatenate([(r[:, j] - r[:, i]) / 100.0 for r in rows])
            print(f"  {lab:26s} " + " ".join(f"{np.percentile(d, q):7.2f}" for q in (0, 10, 50, 90, 100)))
    d = np.concatenate([(r[:, 1] - r[:, 0]) / 100.0 for r in rows])
    print(f"  k_cars load phase          " + " ".join(f"{np.percentile(d, q):7.2f}" for q in (0, 10, 50, 90, 100)))


if __name__ == "__main__":
    main()
