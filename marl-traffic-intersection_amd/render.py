"""Headless renderer: the reference's Windows-only GLFW/OpenGL
renderer (cpp/Renderer.cpp, colours cpp/RenderColors.h) restated as a display
list in pixel coordinates plus a small rasteriser, for one env of a device
handle -- an RGB array or a PNG instead of a window.

scene() follows Renderer::render's drawing rules and order (Renderer.cpp:202-234):
the road (draw_road :518-556: surface strips, corner squares, grass discs as
32-segment fans, yellow centre lines, white stop lines, dashed lane lines, black
boundaries with 48-segment corner arcs), car 0's route and look-ahead target
(draw_route :377-403), every alive car as a body quad plus a head-marker quad
(draw_cars :559-609: agents coloured by index, NPCs grey with a black marker),
and the LiDAR hit rays only, each with a 6-segment dot at its end (draw_lidar
:612-646).  Vertices are computed in float32 with the reference's formulas
(rotation by -heading, ray end = centre + dist * (cos, -sin) of heading +
rel_angle).  tests/test_render.py checks scene() against a line-by-line
restatement of Renderer.cpp (tests/render_oracle.py) on golden states recorded
from the reference.  The rasteriser (PIL polygons and lines, alpha blended) is
not the GPU's OpenGL rasterisation; the geometry and colours are the
reference's.  Debug tooling only: it reads state through mev_get_state /
mev_get_outputs and never touches the step path."""
from __future__ import annotations

import math
from typing import List, Optional, Sequence, Tuple

import numpy as np

W = H = 750
LANE_W, CORNER_R = 42.0, 84.0
CAR_LENGTH, CAR_WIDTH = 54.0, 24.0

# cpp/RenderColors.h (r, g, b, a in [0, 1])
BACKGROUND = (34 / 255, 139 / 255, 34 / 255, 1.0)
ROAD_SURFACE = (60 / 255, 60 / 255, 60 / 255, 1.0)
GRASS_C = (34 / 255, 139 / 255, 34 / 255, 1.0)
CENTER_YELLOW = (1.0, 0.8, 0.0, 1.0)
MARKING_WHITE = (0.94, 0.94, 0.94, 1.0)
ROUTE_CYAN = (0.0, 1.0, 1.0, 0.8)
TARGET_RED = (1.0, 0.0, 0.0, 1.0)
TRAFFIC_GRAY = (150 / 255, 150 / 255, 150 / 255, 1.0)
TRAFFIC_HEAD = (0.0, 0.0, 0.0, 1.0)
AGENT_HEAD = (200 / 255, 200 / 255, 200 / 255, 1.0)
LIDAR_GREEN = (0.0, 1.0, 0.0, 0.35)
LIDAR_HIT = (1.0, 0.0, 0.0, 1.0)
BOUNDARY = (0.0, 0.0, 0.0, 1.0)
# agent body colours by index (Renderer.cpp:597-599)
AGENT_COLORS = ((231 / 255, 76 / 255, 60 / 255, 1.0), (52 / 255, 152 / 255, 219 / 255, 1.0),
                (46 / 255, 204 / 255, 113 / 255, 1.0), (155 / 255, 89 / 255, 182 / 255, 1.0),
                (241 / 255, 196 / 255, 15 / 255, 1.0), (230 / 255, 126 / 255, 34 / 255, 1.0))

# kept for callers of the earlier renderer: 8-bit RGB of the main colours
ROAD = tuple(int(round(c * 255)) for c in ROAD_SURFACE[:3])
GRASS = tuple(int(round(c * 255)) for c in GRASS_C[:3])
EGO = tuple(int(round(c * 255)) for c in AGENT_COLORS[0][:3])
NPC = tuple(int(round(c * 255)) for c in TRAFFIC_GRAY[:3])
HIT = tuple(int(round(c * 255)) for c in LIDAR_HIT[:3])

f32 = np.float32
PI_F = f32(3.14159265358979323846)

# display-list primitives (pixel coordinates, y down):
#   ("quad", ((x, y) * 4), rgba)   ("fan", ((x, y) ...), rgba)   ("line", (x0, y0, x1, y1), width, rgba)
Prim = tuple


def road_mask(num_lanes: int) -> np.ndarray:
    """RoadGeometry::is_on_road at integer pixels (RoadGeometry.h:19-58), vectorised: the predicate
    the kernels use (pinned against the reference raster by tests/test_dropin_cpu.py)."""
    rw = num_lanes * int(LANE_W)
    ccen = rw + int(CORNER_R)
    y, x = np.mgrid[0:H, 0:W]
    ax, ay = np.abs(x - 375), np.abs(y - 375)
    in_disc = (ax - ccen) ** 2 + (ay - ccen) ** 2 <= int(CORNER_R) ** 2
    in_strip = np.minimum(ax, ay) <= rw
    in_square = np.maximum(ax, ay) <= ccen
    return (in_strip | in_square) & ~in_disc


def line_mask(num_lanes: int) -> np.ndarray:
    """LineMask rectangles (LineMask.cpp:14-72): double lines up to the stop offset."""
    stop = num_lanes * int(LANE_W) + int(CORNER_R)
    m = np.zeros((H, W), bool)
    for off in (-3, -2, -1, 1, 2, 3):
        c = 375 + off
        m[: 375 - stop + 1, c] = True
        m[375 + stop:, c] = True
        m[c, : 375 - stop + 1] = True
        m[c, 375 + stop:] = True
    return m


def _rect(x, y, w, h, col) -> Prim:  # draw_rect_ndc (:36-48)
    x, y, w, h = f32(x), f32(y), f32(w), f32(h)
    return ("quad", ((x, y), (x + w, y), (x + w, y + h), (x, y + h)), col)


def _circle(cx, cy, radius, segments, col) -> Prim:  # draw_circle_px (:59-70): a triangle fan
    cx, cy, radius = f32(cx), f32(cy), f32(radius)
    pts = []
    for i in range(segments + 1):
        a = f32(2.0) * PI_F * f32(i) / f32(segments)
        pts.append((cx + f32(math.cos(a)) * radius, cy + f32(math.sin(a)) * radius))
    return ("fan", tuple(pts), col)


def _line(x0, y0, x1, y1, width, col) -> Prim:  # draw_line_px (:50-57)
    return ("line", (f32(x0), f32(y0), f32(x1), f32(y1)), float(width), col)


def road_scene(num_lanes: int) -> List[Prim]:
    """draw_road (:518-556) with its helpers: centre lines (:405-422), stop lines (:424-434),
    boundaries (:436-472) and lane dashes (:474-516)."""
    rw = f32(num_lanes) * f32(LANE_W)
    cr, cx, cy = f32(CORNER_R), f32(W * 0.5), f32(H * 0.5)
    out = [_rect(f32(W * 0.5) - rw, 0, f32(2) * rw, H, ROAD_SURFACE),
           _rect(0, f32(H * 0.5) - rw, W, f32(2) * rw, ROAD_SURFACE)]
    for px, py in ((cx - rw - cr, cy - rw - cr), (cx + rw, cy - rw - cr), (cx - rw - cr, cy + rw), (cx + rw, cy + rw)):
        out.append(_rect(px, py, cr, cr, ROAD_SURFACE))
    for gx, gy in ((cx - rw - cr, cy - rw - cr), (cx + rw + cr, cy - rw - cr), (cx - rw - cr, cy + rw + cr),
                   (cx + rw + cr, cy + rw + cr)):
        out.append(_circle(gx, gy, cr, 32, GRASS_C))
    stop = rw + f32(CORNER_R)
    g = f32(2.0)
    for x0, y0, x1, y1 in ((cx - g, 0, cx - g, cy - stop), (cx + g, 0, cx + g, cy - stop),
                           (cx - g, H, cx - g, cy + stop), (cx + g, H, cx + g, cy + stop),
                           (0, cy - g, cx - stop, cy - g), (0, cy + g, cx - stop, cy + g),
                           (W, cy - g, cx + stop, cy - g), (W, cy + g, cx + stop, cy + g)):
        out.append(_line(x0, y0, x1, y1, 2, CENTER_YELLOW))
    for x0, y0, x1, y1 in ((cx - rw, cy - stop, cx, cy - stop), (cx, cy + stop, cx + rw, cy + stop),
                           (cx - stop, cy, cx - stop, cy + rw), (cx + stop, cy, cx + stop, cy - rw)):
        out.append(_line(x0, y0, x1, y1, 4, MARKING_WHITE))
    out += _lane_dashes(num_lanes, rw, cx, cy, stop)
    out += _boundaries(rw, cx, cy, cr)
    return out


def _lane_dashes(num_lanes, rw, cx, cy, stop) -> List[Prim]:
    out = []

    def dash(x0, y0, x1, y1):
        x0, y0, x1, y1 = f32(x0), f32(y0), f32(x1), f32(y1)
        dist = f32(math.hypot(float(x1 - x0), float(y1 - y0)))
        dash_len = f32(20.0)
        steps = int(dist / (dash_len * f32(2)))
        dx, dy = (x1 - x0) / dist, (y1 - y0) / dist
        for i in range(steps + 1):
            sx = x0 + dx * f32(i) * dash_len * f32(2)
            sy = y0 + dy * f32(i) * dash_len * f32(2)
            ex, ey = sx + dx * dash_len, sy + dy * dash_len
            t_end = f32(1.0) if i == steps else f32(f32(i) * dash_len * f32(2) + dash_len) / dist
            if t_end >= f32(1.0):
                ex, ey = x1, y1
            out.append(_line(sx, sy, ex, ey, 2, MARKING_WHITE))

    for i in range(1, num_lanes):
        off = f32(i) * f32(LANE_W)
        dash(cx - off, 0, cx - off, cy - stop)
        dash(cx + off, 0, cx + off, cy - stop)
        dash(cx - off, H, cx - off, cy + stop)
        dash(cx + off, H, cx + off, cy + stop)
        dash(0, cy - off, cx - stop, cy - off)
        dash(0, cy + off, cx - stop, cy + off)
        dash(W, cy - off, cx + stop, cy - off)
        dash(W, cy + off, cx + stop, cy + off)
    return out


def _boundaries(rw, cx, cy, cr) -> List[Prim]:
    w = 3
    out = [_line(cx - rw, 0, cx - rw, cy - rw - cr, w, BOUNDARY), _line(cx + rw, 0, cx + rw, cy - rw - cr, w, BOUNDARY),
           _line(cx - rw, H, cx - rw, cy + rw + cr, w, BOUNDARY), _line(cx + rw, H, cx + rw, cy + rw + cr, w, BOUNDARY),
           _line(0, cy - rw, cx - rw - cr, cy - rw, w, BOUNDARY), _line(0, cy + rw, cx - rw - cr, cy + rw, w, BOUNDARY),
           _line(W, cy - rw, cx + rw + cr, cy - rw, w, BOUNDARY), _line(W, cy + rw, cx + rw + cr, cy + rw, w, BOUNDARY)]

    def arc(ox, oy, a0, a1):
        a0, a1 = f32(a0), f32(a1)
        px, py = ox + cr * f32(math.cos(a0)), oy + cr * f32(math.sin(a0))
        for i in range(1, 49):
            t = f32(i) / f32(48)
            a = a0 + (a1 - a0) * t
            x, y = ox + cr * f32(math.cos(a)), oy + cr * f32(math.sin(a))
            out.append(_line(px, py, x, y, w, BOUNDARY))
            px, py = x, y

    arc(cx - rw - cr, cy - rw - cr, 0.0, 1.57079632679)
    arc(cx + rw + cr, cy - rw - cr, 1.57079632679, 3.14159265359)
    arc(cx - rw - cr, cy + rw + cr, -1.57079632679, 0.0)
    arc(cx + rw + cr, cy + rw + cr, 3.14159265359, 4.71238898038)
    return out


def car_quads(x, y, heading, body, head) -> List[Prim]:
    """draw_cars' draw_one (:561-594): body rot(+-hl, +-hw) and the head marker, rotation by -heading."""
    x, y, heading = f32(x), f32(y), f32(heading)
    hl, hw = f32(CAR_LENGTH) * f32(0.5), f32(CAR_WIDTH) * f32(0.5)
    c, s = f32(math.cos(-heading)), f32(math.sin(-heading))

    def rot(lx, ly):
        lx, ly = f32(lx), f32(ly)
        return (x + (lx * c - ly * s), y + (lx * s + ly * c))

    length = f32(CAR_LENGTH)
    x0, x1 = -hl + f32(0.70) * length, -hl + f32(0.95) * length
    y0, y1 = -hw + f32(2.0), hw - f32(2.0)
    return [("quad", (rot(hl, hw), rot(hl, -hw), rot(-hl, -hw), rot(-hl, hw)), body),
            ("quad", (rot(x0, y0), rot(x1, y0), rot(x1, y1), rot(x0, y1)), head)]


def lidar_rel_angles(rays: int, fov_deg: float = 360.0) -> np.ndarray:
    """The reference's beam offsets (IntersectionEnv.cpp:119-127, Lidar.cpp:4-14), float32."""
    start = -f32(fov_deg) * f32(0.5)
    step = f32(fov_deg) / f32(rays - 1) if rays > 1 else f32(0.0)
    return np.array([(start + f32(i) * step) * PI_F / f32(180.0) for i in range(rays)], np.float32)


def lidar_prims(x, y, heading, dists: Sequence[float], rel: Sequence[float], max_dist: float) -> List[Prim]:
    """draw_lidar (:612-646): hit rays only (dist < max_dist - 0.1), a line and a 6-segment dot each."""
    out = []
    x, y, heading, mx = f32(x), f32(y), f32(heading), f32(max_dist)
    for d, r in zip(dists, rel):
        d = f32(d)
        if not d < mx - f32(0.1):
            continue
        ang = heading + f32(r)
        ex = x + d * f32(math.cos(ang))
        ey = y - d * f32(math.sin(ang))
        out.append(_line(x, y, ex, ey, 2.0, LIDAR_GREEN))
        out.append(_circle(ex, ey, 2.0, 6, LIDAR_HIT))
    return out


def route_prims(path: np.ndarray, path_index: int) -> List[Prim]:
    """draw_route (:377-403): car 0's path as a 2-px cyan strip and its look-ahead target dot."""
    out = [("strip", tuple((f32(px), f32(py)) for px, py in path), 2.0, ROUTE_CYAN)]
    t = min(max(int(path_index) + 10, 0), len(path) - 1)
    out.append(_circle(path[t][0], path[t][1], 4.0, 10, TARGET_RED))
    return out


def scene(num_lanes: int, cars: Sequence[Tuple[float, float, float, bool]],
          npcs: Sequence[Tuple[float, float, float, bool]] = (), lidar: Optional[Sequence] = None,
          route0: Optional[Tuple[np.ndarray, int]] = None) -> List[Prim]:
    """Renderer::render's display list (:202-234).  cars / npcs: (x, y, heading, alive) in index
    order; lidar: per car (distances, rel_angles, max_dist) or None; route0: (path, path_index)
    of car 0."""
    out = road_scene(num_lanes)
    if route0 is not None and len(cars):
        out += route_prims(*route0)
    for i, (x, y, h, alive) in enumerate(cars):
        if alive:
            out += car_quads(x, y, h, AGENT_COLORS[i % len(AGENT_COLORS)], AGENT_HEAD)
    for x, y, h, alive in npcs:
        if alive:
            out += car_quads(x, y, h, TRAFFIC_GRAY, TRAFFIC_HEAD)
    if lidar is not None:
        for (x, y, h, alive), lid in zip(cars, lidar):
            if alive and lid is not None:
                out += lidar_prims(x, y, h, *lid)
    return out


def _rgba8(col):
    return tuple(int(round(c * 255)) for c in col)


def rasterize(prims: Sequence[Prim]) -> np.ndarray:
    """RGB uint8 [750, 750, 3] of a display list: polygons filled, lines of their width, colours
    with alpha < 1 blended over what is below (PIL, on the 750 x 750 logical canvas)."""
    from PIL import Image, ImageDraw

    im = Image.new("RGB", (W, H), _rgba8(BACKGROUND)[:3])
    dr = ImageDraw.Draw(im, "RGBA")
    for p in prims:
        kind = p[0]
        if kind in ("quad", "fan"):
            pts = [(float(a), float(b)) for a, b in p[1]]
            dr.polygon(pts, fill=_rgba8(p[2]))
        elif kind == "line":
            x0, y0, x1, y1 = (float(v) for v in p[1])
            dr.line([(x0, y0), (x1, y1)], fill=_rgba8(p[3]), width=max(1, int(round(p[2]))))
        elif kind == "strip":
            dr.line([(float(a), float(b)) for a, b in p[1]], fill=_rgba8(p[3]), width=max(1, int(round(p[2]))),
                    joint="curve")
    return np.asarray(im)


def lidar_distances(obs_row: np.ndarray, rays: int, max_dist: float, step: float) -> np.ndarray:
    """The LiDAR distances behind an observation row (obs[31:31+R] = dist * (1 / max_dist)): each
    value is matched to the probe distance it came from (dist += step accumulated in float32, as
    Lidar.cpp:33 does), so the distances are the reference's exact floats."""
    inv = f32(1.0) / f32(max_dist)
    dists, d = [], f32(0.0)
    while d < f32(max_dist):
        dists.append(d)
        d = f32(d + f32(step))
    table = {float(f32(v) * inv): float(v) for v in dists}
    table[float(f32(max_dist) * inv)] = float(max_dist)
    vals = np.asarray(obs_row[31:31 + rays], np.float32)
    return np.array([table.get(float(v), float(v) * float(max_dist)) for v in vals], np.float32)


def handle_scene(handle, env: int = 0, show_lidar: bool = True, show_route: bool = True) -> List[Prim]:
    """scene() of env `env` of a _capi.Handle (state from mev_get_state, LiDAR from the observation)."""
    L = int(handle.config["num_lanes"])
    st = handle.get_state()
    N, R = handle.N, handle.R
    cars = [(float(st["x"][env, i]), float(st["y"][env, i]), float(st["heading"][env, i]), bool(st["alive"][env, i]))
            for i in range(N)]
    k = int(np.asarray(st["npc_count"])[env])
    npcs = [(float(st["npc_x"][env, j]), float(st["npc_y"][env, j]), float(st["npc_heading"][env, j]),
             bool(st["npc_alive"][env, j])) for j in range(k)]
    lidar = None
    if show_lidar:
        obs = handle.observations()[env]
        maxd, step, fov = (float(handle.config[n]) for n in ("lidar_max_dist", "lidar_step", "lidar_fov_deg"))
        slots = min(R, obs.shape[-1] - 31)
        rel = lidar_rel_angles(R, fov)[:slots]
        lidar = [(lidar_distances(obs[i], slots, maxd, step), rel, maxd) for i in range(N)]
    route0 = None
    if show_route and N:
        r0 = int(st["route"][env, 0])
        route0 = (handle.route_info(r0)[0][: handle.route_len(r0)], int(st["path_index"][env, 0]))
    return scene(L, cars, npcs, lidar, route0)


def render(handle, env: int = 0, show_lidar: bool = True, show_routes: bool = True) -> np.ndarray:
    """RGB uint8 [750, 750, 3] frame of env `env` of a _capi.Handle."""
    return rasterize(handle_scene(handle, env, show_lidar, show_routes))


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
