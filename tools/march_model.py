"""CPU model of k_lidar's road march iteration counts (statistics only, not a
parity tool): per-beam iterations of the skip-ahead march on recorded ego
poses (tests/golden), and the wave cost of the lockstep schedule (max over the
64 beams of an agent) versus a pooled schedule (beams of several agents fed
to the 64 lanes from a queue)."""
from __future__ import annotations

import sys

import numpy as np

sys.path.insert(0, "tests")
import golden_replay as G  # noqa: E402

W = 750
STP, S = 4.0, 63


def march_iters(cx, cy, h, rel, rw=126.0, cr=84.0, directional=False):
    ccen = rw + cr
    out = np.zeros(len(rel), np.int32)
    stopk = np.zeros(len(rel), np.int32)
    for b, r in enumerate(rel):
        dx, dy = np.cos(h + r), -np.sin(h + r)
        adx, ady = abs(dx), abs(dy)
        iadx = 1 / adx if adx > 0 else 1e30
        iady = 1 / ady if ady > 0 else 1e30
        k, it = 0, 0
        while True:
            it += 1
            d = k * STP
            fx, fy = cx + dx * d, cy + dy * d
            px, py = int(fx), int(fy)
            off_screen = not (0 <= px < W and 0 <= py < W)
            iax, iay = abs(px - 375), abs(py - 375)
            qdx, qdy = iax - ccen, iay - ccen
            onv = max(min(min(iax, iay) - rw, max(iax, iay) - ccen), cr * cr + 1 - (qdx * qdx + qdy * qdy))
            off_road = k > 0 and onv > 0
            if off_screen or off_road:
                break
            ax, ay = abs(fx - 375), abs(fy - 375)
            if directional:
                sx = (375 + (rw - 1.5) - fx) * iadx if dx > 0 else (fx - (375 - rw + 1.5)) * iadx
                sy = (375 + (rw - 1.5) - fy) * iady if dy > 0 else (fy - (375 - rw + 1.5)) * iady
                mx, my = rw - 1.5 - ax, rw - 1.5 - ay
                strip = max(sx if mx > 0 else 0, sy if my > 0 else 0)
            else:
                mx, my = rw - 1.5 - ax, rw - 1.5 - ay
                strip = max(max(mx, 0) * iadx, max(my, 0) * iady)
            qx, qy = ax - ccen, ay - ccen
            corner = min(np.hypot(qx, qy) - cr, min(ccen - ax, ccen - ay)) - 1.55
            road = strip if max(mx, my) > 0 else (corner if max(ax, ay) < ccen else 0.0)
            tx = ((748.5 - fx) if dx > 0 else (fx - 0.5)) * iadx
            ty = ((748.5 - fy) if dy > 0 else (fy - 0.5)) * iady
            safe = min(road, tx, ty)
            jump = int(safe / STP) if safe >= 2 * STP else 1
            k += jump
            if k >= S:
                break
        out[b] = it
        stopk[b] = k
    return out, stopk


def main():
    g = G.load("cfg3_team_policy")
    R = 64
    rel = np.array([(-180.0 + i * (360.0 / (R - 1))) * np.pi / 180.0 for i in range(R)], np.float32)
    for directional in (False, True):
        per_agent = []
        for t in range(0, len(g["ego_f"]), 10):
            for i in range(g["ego_f"].shape[1]):
                x, y, _, h = g["ego_f"][t, i, :4]
                it, _ = march_iters(float(x), float(y), float(h), rel, directional=directional)
                per_agent.append(it)
        A = np.array(per_agent)
        lock = A.max(axis=1).mean()
        mean = A.mean()
        # pooled: 64 lanes fed from a queue of the beams of `pool` agents
        res = {}
        for pool in (1, 2, 4, 8):
            costs = []
            for s in range(0, len(A) - pool + 1, pool):
                beams = np.sort(A[s:s + pool].reshape(-1))[::-1]
                lanes = np.zeros(64)
                for b in beams:  # LPT-ish: the real queue is FIFO; greedy to the least-loaded lane
                    lanes[lanes.argmin()] += b
                costs.append(lanes.max() / pool)
            res[pool] = np.mean(costs)
        print(f"directional={directional}: mean beam iters {mean:.2f}, lockstep wave cost/agent {lock:.2f}, "
              f"pooled cost/agent {res}")


if __name__ == "__main__":
    main()
