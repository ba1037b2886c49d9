"""Diagnostic (stamps build): the NPC phase of k_cars in traffic mode -- cycles
per env by its NPC count, and the k_cars time of the step -- at steady-state
traffic (config 4 shape after a long warm-up).
    MEV_LIB_VARIANT=stamps python tools/npc_profile.py [--envs 4096 --density 0.5 --warmup 800]
    MEV_LIB_VARIANT=stampsn python tools/npc_profile.py --parts   (cycles per part, summed over the turns)"""
import argparse
import os
import sys

os.environ.setdefault("MEV_LIB_VARIANT", "stamps")
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

import pkgload  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=4096)
    ap.add_argument("--density", type=float, default=0.5)
    ap.add_argument("--warmup", type=int, default=800)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--parts", action="store_true", help="stampsn build: cycles per part of the NPC phase")
    a = ap.parse_args()
    mev = pkgload.load()
    h = mev.Handle(num_envs=a.envs, num_agents=1, lidar_rays=64, traffic_flow=1, traffic_density=a.density,
                   max_npcs=32)
    rng = np.random.default_rng(0)
    for t in range(a.warmup):
        h.step(rng.uniform(-1, 1, (a.envs, 1, 2)).astype(np.float32), auto_reset=True)
    h.kernel_timing(1)
    cyc, kk, tot, parts = [], [], [], []
    for t in range(a.steps):
        k_before = h.get_state()["npc_count"].copy()
        h.step(rng.uniform(-1, 1, (a.envs, 1, 2)).astype(np.float32), auto_reset=True)
        s = h.debug_stamps().astype(np.int64)
        parts.append(s.copy())
        cyc.append(s[:, 1] - s[:, 0])
        tot.append(s[:, 6] - s[:, 0])
        kk.append(k_before)
    c, l_, n = h.kernel_times()
    cyc, kk, tot = np.concatenate(cyc), np.concatenate(kk), np.concatenate(tot)
    print(f"k_cars {c / n * 1e3:.1f} us, k_lidar {l_ / n * 1e3:.1f} us per step; NPCs per env mean {kk.mean():.2f} "
          f"max {kk.max()}; per-step max NPCs over envs (mean) {np.mean(np.max(kk.reshape(a.steps, -1), 1)):.1f}")
    if a.parts:
        names = ["state+spawn", "part 1", "A: pairs", "moves (+seq)", "B: pairs", "scan passes #", "scans (A+B)",
                 "collide+erase"]
        dd = np.concatenate(parts)
        print("NPCs  envs  " + "  ".join(f"{n:>16s}" for n in names))
        for k in range(int(kk.max()) + 1):
            m = kk == k
            if m.sum():
                print(f"{k:4d} {int(m.sum()):6d}  " + "  ".join(f"{np.median(dd[m, q]):16.0f}" for q in range(8)))
        h.close()
        return
    print("NPCs  envs     npc-phase cycles (median / p90)   whole car part (median / p90)")
    for k in range(int(kk.max()) + 1):
        m = kk == k
        if m.sum():
            print(f"{k:4d} {int(m.sum()):7d}   {np.median(cyc[m]):9.0f} {np.percentile(cyc[m], 90):9.0f}"
                  f"        {np.median(tot[m]):9.0f} {np.percentile(tot[m], 90):9.0f}")
    h.close()


if __name__ == "__main__":
    main()
