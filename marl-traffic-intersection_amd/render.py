"""Headless debug renderer (stands in for the reference's
Windows-only GLFW renderer, cpp/Renderer.cpp:520-646): rasterises one env of a
device handle on the host — road and grass from the same integer-pixel road
predicate the kernels use, the line mask, route paths, ego and NPC cars and
the LiDAR hit points decoded from the observation — into an RGB array or a
PNG.  Debug tooling only: it reads state through mev_get_state /
mev_get_outputs and never touches the step path."""
from __future__ import annotations

import math
from typing import Optional

import numpy as np

W = H = 750
LANE_W, CORNER_R = 42, 84

ROAD = (60, 60, 60)
GRASS = (34, 139, 34)
YELLOW = (255, 204, 0)
WHITE = (240, 240, 240)
ROUTE = (0, 255, 255)
EGO = (30, 110, 230)
EGO_DEAD = (90, 90, 120)
NPC = (150, 150, 150)
HIT = (255, 0, 0)
RAY = (0, 255, 0)


def road_mask(num_lanes: int) -> np.ndarray:
    """RoadGeometry::is_on_road at integer pixels (RoadGeometry.h:19-58), vectorised."""
    rw = num_lanes * LANE_W
    ccen = rw + CORNER_R
    y, x = np.mgrid[0:H, 0:W]
    ax, ay = np.abs(x - 375), np.abs(y - 375)
    in_disc = (ax - ccen) ** 2 + (ay - ccen) ** 2 <= CORNER_R * CORNER_R
    in_strip = np.minimum(ax, ay) <= rw
    in_square = np.maximum(ax, ay) <= ccen
    return (in_strip | in_square) & ~in_disc


def line_mask(num_lanes: int) -> np.ndarray:
    """LineMask rectangles (LineMask.cpp:14-72): double lines up to the stop offset."""
    stop = num_lanes * LANE_W + CORNER_R
    m = np.zeros((H, W), bool)
    for off in (-3, -2, -1, 1, 2, 3):
        c = 375 + off
        m[: 375 - stop + 1, c] = True
        m[375 + stop:, c] = True
        m[c, : 375 - stop + 1] = True
        m[c, 375 + stop:] = True
    return m


def _corners(x, y, h, length=54.0, width=24.0):
    """Car::corners (Car.cpp:86-103)."""
    c, s = math.cos(h), math.sin(h)
    hx, hy = width * 0.5, length * 0.5
    pts = [(hy, hx), (hy, -hx), (-hy, -hx), (-hy, hx)]
    return [(x + lx * c - ly * s, y - (lx * s + ly * c)) for lx, ly in pts]


def render(handle, env: int = 0, show_lidar: bool = True, show_routes: bool = True) -> np.ndarray:
    """RGB uint8 [750, 750, 3] image of env `env` of a _capi.Handle."""
    from PIL import Image, ImageDraw

    L = handle.config["num_lanes"]
    img = np.empty((H, W, 3), np.uint8)
    img[:] = GRASS
    img[road_mask(L)] = ROAD
    img[line_mask(L)] = WHITE
    img[375, :] = img[:, 375] = YELLOW
    im = Image.fromarray(img)
    dr = ImageDraw.Draw(im)
    st = handle.get_state()
    obs = handle.observations()[env]
    N, R = handle.N, handle.R
    maxd, fov = handle.config["lidar_max_dist"], handle.config["lidar_fov_deg"]
    poses = [(float(st["x"][env, i]), float(st["y"][env, i]), float(st["heading"][env, i]),
              bool(st["alive"][env, i])) for i in range(N)]
    if show_routes:
        for i in range(N):
            path = handle.route_info(int(st["route"][env, i]))[0]
            dr.line([tuple(p) for p in path], fill=ROUTE, width=1)
    hits = []
    if show_lidar:
        slots = min(R, obs.shape[-1] - 31)
        for i, (x, y, h, alive) in enumerate(poses):
            if not alive:
                continue
            for b in range(slots):
                d = float(obs[i, 31 + b]) * maxd
                a = h + math.radians(-fov / 2 + b * (fov / (R - 1) if R > 1 else 0.0))
                ex, ey = x + math.cos(a) * d, y - math.sin(a) * d
                dr.line([(x, y), (ex, ey)], fill=RAY, width=1)
                if d < maxd:
                    hits.append((ex, ey))
    for x, y, h, alive in poses:
        dr.polygon(_corners(x, y, h), fill=EGO if alive else EGO_DEAD, outline=(0, 0, 0))
    for k in range(int(np.asarray(st["npc_count"])[env])):
        if st["npc_alive"][env, k]:
            dr.polygon(_corners(float(st["npc_x"][env, k]), float(st["npc_y"][env, k]),
                                float(st["npc_heading"][env, k])), fill=NPC, outline=(0, 0, 0))
    for ex, ey in hits:
        dr.ellipse([ex - 2, ey - 2, ex + 2, ey + 2], fill=HIT)
    return np.asarray(im)


def save_png(handle, path: str, env: int = 0, **kw) -> str:
    from PIL import Image
    Image.fromarray(render(handle, env, **kw)).save(path)
    return path


def frames_to_png(frames, path_prefix: str, every: int = 1) -> list:
    """Write a list of RGB frames as numbered PNGs; returns the paths."""
    from PIL import Image
    out = []
    for t, f in enumerate(frames[::every]):
        p = f"{path_prefix}{t:05d}.png"
        Image.fromarray(f).save(p)
        out.append(p)
    return out


def render_cpp_backend(env, env_index: Optional[int] = None) -> Optional[np.ndarray]:
    """Frame of a cpp_backend.IntersectionEnv (None before any car exists)."""
    h = env._sync()
    return None if h is None else render(h, 0 if env_index is None else env_index)
