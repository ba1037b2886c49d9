"""Diagnostic: road-march (LiDAR phase 2) statistics per beam pool, exp_iters build.
    python tools/iter_hist.py [--step-kernel 2]
Per pool (k_step: one per env): wave iterations, queued beams after phase 1, the
iteration at which the queue ran dry (after it only the tail of running beams
remains) and the lane utilisation (busy lane-iterations / 64 x iterations)."""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

import pkgload  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--step-kernel", type=int, default=2)
    ap.add_argument("--envs", type=int, default=4096)
    ap.add_argument("--agents", type=int, default=8)
    ap.add_argument("--rays", type=int, default=64)
    ap.add_argument("--pack", type=int, default=0)
    a = ap.parse_args()
    mev = pkgload.load()
    mev._capi.VARIANT = "exp_iters"
    h = mev.Handle(num_envs=a.envs, num_agents=a.agents, lidar_rays=a.rays, use_team_reward=1)
    h.set_step_kernel(a.step_kernel)
    h.set_step_pack(a.pack)
    rng = np.random.default_rng(0)
    for t in range(300):
        h.step(rng.uniform(-1, 1, (a.envs, a.agents, 2)).astype(np.float32), auto_reset=True)
    d = h.debug_stamps().reshape(a.envs, 8).astype(np.int64)
    it, qn, dry, busy = d[:, 0], d[:, 1], d[:, 2], d[:, 3]
    ok = it > 0

    def stat(name, v):
        print(f"  {name:28s} mean {v.mean():7.2f}  p10 {np.percentile(v, 10):6.1f}  p50 {np.percentile(v, 50):6.1f}"
              f"  p90 {np.percentile(v, 90):6.1f}  max {v.max():6.1f}")

    print(f"pools: {ok.sum()} of {a.envs}")
    stat("iterations", it[ok])
    stat("queued beams", qn[ok])
    stat("iteration queue ran dry", dry[ok])
    stat("tail iterations", (it - dry)[ok])
    stat("lane utilisation %", 100.0 * busy[ok] / (64.0 * it[ok]))
    print("phase 3 (car pairs):")
    stat("segments (agent, box)", d[ok, 4])
    stat("pairs (beam, box)", d[ok, 5])
    stat("64-pair chunks", d[ok, 6])
    stat("probe-loop trips", d[ok, 7])


if __name__ == "__main__":
    main()
