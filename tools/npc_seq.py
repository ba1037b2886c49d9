"""Diagnostic: how often the NPC controller's round B disagrees with round A at
config 4 (4096 envs x 1 agent x 64 beams, traffic density 0.5) and how many
sequential turns follow, per step, at steady-state traffic (mev_npc_stats).
    python tools/npc_seq.py [--envs 4096 --density 0.5 --warmup 600 --steps 200]"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

import pkgload  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=4096)
    ap.add_argument("--density", type=float, default=0.5)
    ap.add_argument("--warmup", type=int, default=600)
    ap.add_argument("--steps", type=int, default=200)
    a = ap.parse_args()
    mev = pkgload.load()
    h = mev.Handle(num_envs=a.envs, num_agents=1, lidar_rays=64, traffic_flow=1, traffic_density=a.density,
                   max_npcs=32)
    rng = np.random.default_rng(0)
    for _ in range(a.warmup):
        h.step(rng.uniform(-1, 1, (a.envs, 1, 2)).astype(np.float32), auto_reset=True)
    _, s0 = h.npc_stats()
    per = []
    ks = []
    for _ in range(a.steps):
        h.step(rng.uniform(-1, 1, (a.envs, 1, 2)).astype(np.float32), auto_reset=True)
        _, s1 = h.npc_stats()
        per.append(s1 - s0)
        s0 = s1
        ks.append(h.get_state()["npc_count"].copy())
    per = np.array(per)
    k = np.concatenate(ks)
    print(f"envs {a.envs} density {a.density}: sequential turns per step mean {per.mean():.2f} "
          f"p50 {np.percentile(per, 50):.0f} p90 {np.percentile(per, 90):.0f} max {per.max()}; "
          f"steps with none {np.mean(per == 0) * 100:.1f} %; NPCs per env mean {k.mean():.2f}, "
          f"histogram {np.bincount(k, minlength=8)[:10] / a.steps}")
    h.close()


if __name__ == "__main__":
    main()
