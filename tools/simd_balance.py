"""Diagnostic: how k_step's waves (one per env) spread over the SIMDs and where
the step's time goes between them (stampsr build: wave entry in slot 0, wave end
and HW_ID/XCC_ID in slot 7).
    MEV_LIB_VARIANT=stampsr python tools/simd_balance.py
Per step: the span (first entry -> last end), each SIMD's finish time, its waves'
lifetimes; percentiles over the steps' SIMDs, in microseconds (100 MHz ticks)."""
import argparse
import os
import sys
from collections import Counter

os.environ.setdefault("MEV_LIB_VARIANT", "stampsr")
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

import pkgload  # noqa: E402

M40 = (1 << 40) - 1
# (from slot, to slot): car part, LiDAR phase 1, 2, 3, block writes
PHASES = [(0, 2), (3, 4), (4, 6), (6, 5), (5, 7)]
PH_NAMES = ["car part", "lidar phase 1", "lidar phase 2", "lidar phase 3", "block writes"]


def pct(v):
    return " ".join(f"{np.percentile(v, q):7.2f}" for q in (0, 10, 50, 90, 100))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=4096)
    ap.add_argument("--steps", type=int, default=60)
    ap.add_argument("--agents", type=int, default=8)
    ap.add_argument("--rays", type=int, default=64)
    ap.add_argument("--traffic", type=float, default=0.0, help="traffic density (config 4: --agents 1 --traffic 0.5)")
    ap.add_argument("--warmup", type=int, default=0, help="untimed steps first (traffic reaches steady state)")
    a = ap.parse_args()
    mev = pkgload.load()
    h = mev.Handle(num_envs=a.envs, num_agents=a.agents, lidar_rays=a.rays, use_team_reward=int(a.agents > 1),
                   traffic_flow=int(a.traffic > 0), traffic_density=a.traffic, max_npcs=32)
    h.set_step_kernel(2)
    rng = np.random.default_rng(0)
    slots, entries, ph, spans, fin, life, simd_sum, simd_max, simd_mean, nw, first_end = [], [], [], [], [], [], [], [], [], Counter(), []
    by_k = {}
    for t in range(a.warmup):
        h.step(rng.uniform(-1, 1, (a.envs, a.agents, 2)).astype(np.float32), auto_reset=True)
    for t in range(a.steps):
        k_after = None
        h.step(rng.uniform(-1, 1, (a.envs, a.agents, 2)).astype(np.float32), auto_reset=True)
        if t < a.steps // 2:
            continue
        if a.traffic > 0:
            k_after = h.get_state()["npc_count"].copy()
        r = h.debug_stamps().astype(np.uint64).reshape(a.envs, 8)
        if k_after is not None:
            lt_all = ((r[:, 7] & M40).astype(np.int64) - (r[:, 0] & M40).astype(np.int64)) / 100.0
            t0_all = (r[:, 0] & M40).astype(np.int64).min()
            end_all = ((r[:, 7] & M40).astype(np.int64) - t0_all) / 100.0
            for k in np.unique(k_after):
                m = k_after == k
                by_k.setdefault(int(k), []).append(np.stack([lt_all[m], end_all[m]], 1))
        r = r[r[:, 0] != 0]  # packed waves stamp only their first env's slots
        t_in = (r[:, 0] & M40).astype(np.int64)
        t_out = (r[:, 7] & M40).astype(np.int64)
        where = (r[:, 7] >> np.uint64(40)).astype(np.int64)
        simd = (where >> 16) << 16 | (where & 0xFF30)  # xcc, se, sh, cu, simd (no wave slot / pipe)
        t0 = t_in.min()
        spans.append((t_out.max() - t0) / 100.0)
        lt = (t_out - t_in) / 100.0
        life.append(lt)
        first_end.append((t_out.min() - t0) / 100.0)
        slots.append(where & 0xF)
        entries.append((t_in - t0) / 100.0)
        tt = (r.astype(np.int64) & M40)
        tt[:, 7] = t_out
        ph.append(np.stack([(tt[:, j] - tt[:, i]) / 100.0 for i, j in PHASES], 1))
        keys, inv = np.unique(simd, return_inverse=True)
        for k in range(len(keys)):
            m = inv == k
            nw[int(m.sum())] += 1
            fin.append((t_out[m].max() - t0) / 100.0)
            simd_sum.append(lt[m].sum())
            simd_max.append(lt[m].max())
            simd_mean.append(lt[m].mean())
    print(f"envs={a.envs} agents={a.agents} rays={a.rays}: SIMDs per step {len(fin) // len(spans)}, waves per SIMD {dict(sorted(nw.items()))}")
    print("  us (p0 / p10 / p50 / p90 / p100)")
    print(f"  step span (entry -> end)   {pct(spans)}")
    print(f"  first wave end             {pct(first_end)}")
    print(f"  SIMD finish                {pct(fin)}")
    print(f"  wave lifetime              {pct(np.concatenate(life))}")
    print(f"  SIMD: longest wave         {pct(simd_max)}")
    print(f"  SIMD: mean wave            {pct(simd_mean)}")
    print(f"  SIMD: sum of lifetimes     {pct(simd_sum)}")
    L = np.concatenate(life)
    P = np.concatenate(ph)
    lo, hi = L <= np.percentile(L, 10), L >= np.percentile(L, 90)
    print("  per-wave phase time: all p50 | mean of the 10 % shortest waves | of the 10 % longest")
    for k, n in enumerate(PH_NAMES):
        print(f"    {n:22s} {np.percentile(P[:, k], 50):7.2f} | {P[lo, k].mean():7.2f} | {P[hi, k].mean():7.2f}")
    S = np.concatenate(slots)
    E = np.concatenate(entries)
    print("  by wave slot on the SIMD (HW_ID wave_id): slot: waves, mean entry, mean lifetime, mean end")
    for k in np.unique(S):
        m = S == k
        print(f"    {k:2d}: {m.sum():7d} {E[m].mean():7.2f} {L[m].mean():7.2f} {(E[m] + L[m]).mean():7.2f}")
    if by_k:
        print("  by NPCs after the step: envs per step, wave lifetime p50 / p100, wave end p50 / p100 (us)")
        for k in sorted(by_k):
            X = np.concatenate(by_k[k])
            print(f"    {k:2d}: {len(X) / len(spans):8.1f} {np.percentile(X[:, 0], 50):7.2f} {X[:, 0].max():7.2f}"
                  f" {np.percentile(X[:, 1], 50):7.2f} {X[:, 1].max():7.2f}")
    c = np.corrcoef(simd_sum, fin)[0, 1]
    print(f"  corr(SIMD sum of lifetimes, SIMD finish) = {c:.3f}")


if __name__ == "__main__":
    main()
