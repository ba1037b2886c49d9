"""CPU model of k_lidar's road march (statistics only, not a parity tool):
iterations per beam for variants of the road/screen safe-distance bound, on
poses from the C oracle stepping uniform random actions with auto-reset (the
bench workload).  Each iteration = one exact probe + one bound evaluation.
    python tools/road_bound_model.py [--envs 64] [--steps 200]"""
from __future__ import annotations

import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

f32 = np.float32
W = 750


def poses(envs, steps, n=8, rays=64, seed=0):
    from oracle.oracle import OracleEnv
    rng = np.random.default_rng(seed)
    out = []
    for e in range(envs):
        env = OracleEnv(n_agents=n, rays=rays, use_team=True)
        P = env.P
        env.reset(rng.integers(0, 12, n))  # route ids of the default 3-lane layout
        for t in range(steps):
            r = env.step(rng.uniform(-1, 1, (n, 2)).astype(np.float32))
            if r["terminated"] or r["truncated"]:
                env.reset(rng.integers(0, 12, n))
            if t % 10 == 9:
                eg, _, _ = env.get_state()
                for i in range(n):
                    if eg["alive"][i]:
                        out.append((eg["x"][i], eg["y"][i], eg["h"][i]))
        env.close()
    return np.array(out, np.float32)


def safe_v0(fx, fy, dx, dy, rw):
    """The current device bound (road_safe in mev_kernels.hip)."""
    ccen, crf = f32(rw + 84), f32(84)
    rwm = f32(rw - 1.5)
    idx, idy = f32(1) / dx, f32(1) / dy
    iadx, iady = np.abs(idx), np.abs(idy)
    rx, ry = fx - f32(375), fy - f32(375)
    ax, ay = np.abs(rx), np.abs(ry)
    sx = np.where(ax < rwm, rwm * iadx - rx * idx, 0)
    sy = np.where(ay < rwm, rwm * iady - ry * idy, 0)
    sqm, rg = ccen - f32(1.55), crf + f32(2)
    ocx = rx - np.where(np.where(rx != 0, rx, dx) >= 0, ccen, -ccen)
    ocy = ry - np.where(np.where(ry != 0, ry, dy) >= 0, ccen, -ccen)
    return _rest(fx, fy, dx, dy, idx, idy, iadx, iady, rx, ry, ax, ay, sx, sy, sqm, rg, ocx, ocy, f32(0.5), f32(748.5))


def safe_v1(fx, fy, dx, dy, rw, strip_half=None):
    """Per-axis exact intervals about 375.5 (truncation = floor on screen): strips
    hold pixels |p - 375| <= rw - 1 (the tangent pixels of the grass discs sit at
    |p - 375| = rw), the square |p - 375| <= rw + cr, the disc grown by sqrt(2)/2
    about the pixel-offset centre, the screen [0, 750)."""
    eps = f32(0.01)
    ccen, crf = f32(rw + 84), f32(84)
    rwm = f32(rw - 0.5) - eps if strip_half is None else f32(strip_half)
    idx, idy = f32(1) / dx, f32(1) / dy
    iadx, iady = np.abs(idx), np.abs(idy)
    rx, ry = fx - f32(375.5), fy - f32(375.5)
    ax, ay = np.abs(rx), np.abs(ry)
    sx = np.where(ax < rwm, rwm * iadx - rx * idx, 0)
    sy = np.where(ay < rwm, rwm * iady - ry * idy, 0)
    sqm, rg = ccen + f32(0.5) - eps, crf + f32(0.7072) + eps
    ocx = rx - np.where(np.where(rx != 0, rx, dx) >= 0, ccen, -ccen)
    ocy = ry - np.where(np.where(ry != 0, ry, dy) >= 0, ccen, -ccen)
    return _rest(fx, fy, dx, dy, idx, idy, iadx, iady, rx, ry, ax, ay, sx, sy, sqm, rg, ocx, ocy, eps, f32(750) - eps)


def _rest(fx, fy, dx, dy, idx, idy, iadx, iady, rx, ry, ax, ay, sx, sy, sqm, rg, ocx, ocy, slo, shi):
    big = f32(1e6)
    bq = ocx * dx + ocy * dy
    cq = ocx * ocx + ocy * ocy - rg * rg
    disc = bq * bq - cq
    with np.errstate(invalid="ignore"):
        root = -bq - np.sqrt(np.maximum(disc, 0))
    tdisc = np.where(cq <= 0, 0, np.where((disc < 0) | (bq >= 0), big, root))
    tsq = np.minimum(sqm * iadx - rx * idx, sqm * iady - ry * idy)
    tq = np.minimum(np.where(rx * dx < 0, -rx * idx, big), np.where(ry * dy < 0, -ry * idy, big))
    sc = np.where(np.maximum(ax, ay) < sqm, np.minimum(tdisc, np.minimum(tsq, tq)), 0)
    road = np.maximum(np.maximum(sx, sy), sc)
    tx = np.where(dx > 0, shi - fx, fx - slo) * iadx
    ty = np.where(dy > 0, shi - fy, fy - slo) * iady
    return np.minimum(road, np.minimum(tx, ty))


def on_road_px(px, py, rw):
    ccen, cr = rw + 84, 84
    iax, iay = np.abs(px - 375), np.abs(py - 375)
    qdx, qdy = iax - ccen, iay - ccen
    onv = np.maximum(np.minimum(np.minimum(iax, iay) - rw, np.maximum(iax, iay) - ccen), cr * cr + 1 - (qdx * qdx + qdy * qdy))
    return onv <= 0


def march(P, rel, safe_fn, rw=126, stp=4.0, S=63):
    """Returns (iterations per beam, stop index per beam) with the exact probe rule."""
    A, R = len(P), len(rel)
    cx = np.repeat(P[:, 0], R); cy = np.repeat(P[:, 1], R)
    ang = (np.repeat(P[:, 2], R) + np.tile(rel, A)).astype(f32)
    dx, dy = np.cos(ang).astype(f32), (-np.sin(ang)).astype(f32)
    stp = f32(stp)
    # phase 1: first probe from the centre
    px, py = cx.astype(np.int32), cy.astype(np.int32)
    onscr = (px >= 0) & (px < W) & (py >= 0) & (py < W)
    s0 = safe_fn(cx, cy, dx, dy, rw)
    k = np.where(onscr, np.where(s0 >= 2 * stp, (s0 / stp).astype(np.int32), 1), 0)
    it = np.zeros(len(cx), np.int32)
    stop = np.full(len(cx), -1, np.int32)
    act = np.ones(len(cx), bool)
    while act.any():
        i = np.nonzero(act)[0]
        kk = k[i]
        past = kk >= S
        d = np.minimum(kk, S - 1).astype(f32) * stp
        fx, fy = cx[i] + dx[i] * d, cy[i] + dy[i] * d
        qx, qy = np.trunc(fx).astype(np.int64), np.trunc(fy).astype(np.int64)
        off = (qx < 0) | (qx >= W) | (qy < 0) | (qy >= W)
        stp_ = ~past & (off | ((kk > 0) & ~on_road_px(qx, qy, rw)))
        s = safe_fn(fx, fy, dx[i], dy[i], rw)
        kn = kk + np.where(s >= 2 * stp, (s / stp).astype(np.int32), 1)
        fin = past | stp_ | (kn >= S)
        it[i] += 1
        stop[i[fin]] = np.where(stp_[fin], kk[fin], S)
        act[i[fin]] = False
        k[i] = kn
    return it, stop


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=32)
    ap.add_argument("--steps", type=int, default=300)
    a = ap.parse_args()
    P = poses(a.envs, a.steps)
    R = 64
    rel = np.array([np.float32(np.float32(-180.0) + np.float32(i) * np.float32(360.0 / (R - 1))) for i in range(R)],
                   np.float32) * np.float32(np.pi / 180.0)
    base_it, base_stop = march(P, rel, safe_v0)
    print(f"{len(P)} agent poses x {R} beams")
    for name, fn in [("v0 (current)", safe_v0), ("v1 exact axes", safe_v1)]:
        it, stop = march(P, rel, fn)
        assert (stop == base_stop).all(), f"{name}: stop index differs from the current bound"
        print(f"{name:16s} mean iterations/beam {it.mean():.3f}  hist {np.bincount(it, minlength=8)[:10]}")


if __name__ == "__main__":
    main()
