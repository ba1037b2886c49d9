"""Diagnostic: the largest NPC fleet one env reaches at high traffic densities (max_npcs = 64 slots;
mev_npc_overflow counts spawns dropped for want of a slot)."""
import sys, numpy as np
import os
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tests"))
import pkgload
mev = pkgload.load()
for dens in (20.0, 100.0, 1000.0):
    h = mev.Handle(num_envs=256, num_agents=1, lidar_rays=16, traffic_flow=1, traffic_density=dens, max_npcs=64, seed=1)
    h.reset()
    rng = np.random.default_rng(0)
    mx = 0
    for t in range(3000):
        h.step(rng.uniform(-1, 1, (256, 1, 2)).astype(np.float32), auto_reset=True)
        if t % 50 == 49:
            mx = max(mx, int(h.get_state()["npc_count"].max()))
    print(f"density {dens}: max NPCs over 256 envs x 3000 steps = {mx}, overflow = {h.npc_overflow()}", flush=True)
    h.close()
