"""Test infrastructure: the reference renderer's drawing rules restated statement by
statement (cpp/Renderer.cpp:36-70 primitives, :377-403 draw_route, :405-556
draw_road and helpers, :559-609 draw_cars, :612-646 draw_lidar; colours
cpp/RenderColors.h), emitting the vertices it hands to OpenGL in pixel
coordinates (before ndc_x/ndc_y, :32-33) instead of issuing GL calls.  Floats are
float32 as in the C++ (std::cos/std::sin of floats evaluated in double and
rounded: within an ulp of glibc's cosf/sinf, far below a pixel).  Only
tests/test_render.py uses it, as the checker of marl_traffic_intersection_amd.render."""
import math

import numpy as np

F = np.float32
WIDTH = HEIGHT = 750
LANE_WIDTH_PX, CORNER_RADIUS = F(42.0), F(84.0)
CAR_LENGTH, CAR_WIDTH = F(54.0), F(24.0)


def rgba(r, g, b, a=1.0):
    return (float(r), float(g), float(b), float(a))


# RenderColors.h
Background = rgba(34 / 255, 139 / 255, 34 / 255)
RoadSurface = rgba(60 / 255, 60 / 255, 60 / 255)
Grass = rgba(34 / 255, 139 / 255, 34 / 255)
CenterLineYellow = rgba(1.0, 0.8, 0.0)
MarkingWhite = rgba(0.94, 0.94, 0.94)
RouteCyan = rgba(0.0, 1.0, 1.0, 0.8)
TargetRed = rgba(1.0, 0.0, 0.0)
TrafficBodyGray = rgba(150 / 255, 150 / 255, 150 / 255)
TrafficHeadBlack = rgba(0.0, 0.0, 0.0)
AgentHeadMarker = rgba(200 / 255, 200 / 255, 200 / 255)
LidarRayGreen = rgba(0.0, 1.0, 0.0, 0.35)
LidarHitRed = rgba(1.0, 0.0, 0.0)
RoadBoundary = rgba(0.0, 0.0, 0.0)


class Recorder:
    """Collects what Renderer.cpp would draw, in its order."""

    def __init__(self):
        self.prims = []

    # draw_rect_ndc (:36-48): GL_QUADS (x, y), (x + w, y), (x + w, y + h), (x, y + h)
    def draw_rect(self, x_px, y_px, w_px, h_px, col):
        x_px, y_px, w_px, h_px = F(x_px), F(y_px), F(w_px), F(h_px)
        self.prims.append(("quad", ((x_px, y_px), (x_px + w_px, y_px), (x_px + w_px, y_px + h_px),
                                    (x_px, y_px + h_px)), col))

    # draw_line_px (:50-57)
    def draw_line(self, x0, y0, x1, y1, width, col):
        self.prims.append(("line", (F(x0), F(y0), F(x1), F(y1)), float(width), col))

    # draw_circle_px (:59-70): GL_TRIANGLE_FAN of segments + 1 rim points
    def draw_circle(self, cx, cy, radius, segments, col):
        pts = []
        for i in range(segments + 1):
            PI_F = F(3.14159265358979323846)
            a = F(2.0) * PI_F * F(float(i)) / F(float(segments))
            x = F(cx) + F(math.cos(a)) * F(radius)
            y = F(cy) + F(math.sin(a)) * F(radius)
            pts.append((x, y))
        self.prims.append(("fan", tuple(pts), col))


def draw_road(rec, num_lanes):
    rw = F(num_lanes) * LANE_WIDTH_PX
    rec.draw_rect(F(WIDTH * 0.5) - rw, 0, 2 * rw, HEIGHT, RoadSurface)
    rec.draw_rect(0, F(HEIGHT * 0.5) - rw, WIDTH, 2 * rw, RoadSurface)
    cr = CORNER_RADIUS
    cx, cy = F(WIDTH * 0.5), F(HEIGHT * 0.5)
    for px, py in [(cx - rw - cr, cy - rw - cr), (cx + rw, cy - rw - cr), (cx - rw - cr, cy + rw), (cx + rw, cy + rw)]:
        rec.draw_rect(px, py, cr, cr, RoadSurface)
    for gx, gy in [(cx - rw - cr, cy - rw - cr), (cx + rw + cr, cy - rw - cr), (cx - rw - cr, cy + rw + cr),
                   (cx + rw + cr, cy + rw + cr)]:
        rec.draw_circle(gx, gy, cr, 32, Grass)
    draw_center_lines(rec, num_lanes, rw)
    draw_stop_lines(rec, rw)
    draw_lane_dashes(rec, num_lanes, rw)
    draw_road_boundaries(rec, rw)


def draw_center_lines(rec, num_lanes, rw):
    center_gap = F(2.0)
    cx, cy = F(WIDTH * 0.5), F(HEIGHT * 0.5)
    stop_off = rw + CORNER_RADIUS
    Y = CenterLineYellow
    rec.draw_line(cx - center_gap, 0, cx - center_gap, cy - stop_off, 2, Y)
    rec.draw_line(cx + center_gap, 0, cx + center_gap, cy - stop_off, 2, Y)
    rec.draw_line(cx - center_gap, HEIGHT, cx - center_gap, cy + stop_off, 2, Y)
    rec.draw_line(cx + center_gap, HEIGHT, cx + center_gap, cy + stop_off, 2, Y)
    rec.draw_line(0, cy - center_gap, cx - stop_off, cy - center_gap, 2, Y)
    rec.draw_line(0, cy + center_gap, cx - stop_off, cy + center_gap, 2, Y)
    rec.draw_line(WIDTH, cy - center_gap, cx + stop_off, cy - center_gap, 2, Y)
    rec.draw_line(WIDTH, cy + center_gap, cx + stop_off, cy + center_gap, 2, Y)


def draw_stop_lines(rec, rw):
    cx, cy = F(WIDTH * 0.5), F(HEIGHT * 0.5)
    stop_off = rw + CORNER_RADIUS
    w = 4.0
    rec.draw_line(cx - rw, cy - stop_off, cx, cy - stop_off, w, MarkingWhite)
    rec.draw_line(cx, cy + stop_off, cx + rw, cy + stop_off, w, MarkingWhite)
    rec.draw_line(cx - stop_off, cy, cx - stop_off, cy + rw, w, MarkingWhite)
    rec.draw_line(cx + stop_off, cy, cx + stop_off, cy - rw, w, MarkingWhite)


def draw_road_boundaries(rec, rw):
    cx, cy = F(WIDTH * 0.5), F(HEIGHT * 0.5)
    cr = CORNER_RADIUS
    w = 3.0
    B = RoadBoundary
    rec.draw_line(cx - rw, 0, cx - rw, cy - rw - cr, w, B)
    rec.draw_line(cx + rw, 0, cx + rw, cy - rw - cr, w, B)
    rec.draw_line(cx - rw, HEIGHT, cx - rw, cy + rw + cr, w, B)
    rec.draw_line(cx + rw, HEIGHT, cx + rw, cy + rw + cr, w, B)
    rec.draw_line(0, cy - rw, cx - rw - cr, cy - rw, w, B)
    rec.draw_line(0, cy + rw, cx - rw - cr, cy + rw, w, B)
    rec.draw_line(WIDTH, cy - rw, cx + rw + cr, cy - rw, w, B)
    rec.draw_line(WIDTH, cy + rw, cx + rw + cr, cy + rw, w, B)

    def draw_arc(ox, oy, a0, a1):
        segments = 48
        a0, a1 = F(a0), F(a1)
        prev_x = ox + cr * F(math.cos(a0))
        prev_y = oy + cr * F(math.sin(a0))
        for i in range(1, segments + 1):
            t = F(float(i)) / F(float(segments))
            a = a0 + (a1 - a0) * t
            x = ox + cr * F(math.cos(a))
            y = oy + cr * F(math.sin(a))
            rec.draw_line(prev_x, prev_y, x, y, w, B)
            prev_x, prev_y = x, y

    draw_arc(cx - rw - cr, cy - rw - cr, 0.0, 1.57079632679)
    draw_arc(cx + rw + cr, cy - rw - cr, 1.57079632679, 3.14159265359)
    draw_arc(cx - rw - cr, cy + rw + cr, -1.57079632679, 0.0)
    draw_arc(cx + rw + cr, cy + rw + cr, 3.14159265359, 4.71238898038)


def draw_lane_dashes(rec, num_lanes, rw):
    cx, cy = F(WIDTH * 0.5), F(HEIGHT * 0.5)
    stop_off = rw + CORNER_RADIUS

    def dash(x0, y0, x1, y1):
        x0, y0, x1, y1 = F(x0), F(y0), F(x1), F(y1)
        dist = F(math.hypot(float(x1 - x0), float(y1 - y0)))
        dash_len = F(20.0)
        steps = int(dist / (dash_len * 2))
        dx = (x1 - x0) / dist
        dy = (y1 - y0) / dist
        for i in range(steps + 1):
            sx = x0 + dx * F(i) * dash_len * 2
            sy = y0 + dy * F(i) * dash_len * 2
            ex = sx + dx * dash_len
            ey = sy + dy * dash_len
            t_end = F(1.0) if i == steps else F(F(i) * dash_len * 2 + dash_len) / dist
            if t_end >= 1.0:
                ex, ey = x1, y1
            rec.draw_line(sx, sy, ex, ey, 2, MarkingWhite)

    for i in range(1, num_lanes):
        off = F(i) * LANE_WIDTH_PX
        dash(cx - off, 0, cx - off, cy - stop_off)
        dash(cx + off, 0, cx + off, cy - stop_off)
        dash(cx - off, HEIGHT, cx - off, cy + stop_off)
        dash(cx + off, HEIGHT, cx + off, cy + stop_off)
        dash(0, cy - off, cx - stop_off, cy - off)
        dash(0, cy + off, cx - stop_off, cy + off)
        dash(WIDTH, cy - off, cx + stop_off, cy - off)
        dash(WIDTH, cy + off, cx + stop_off, cy + off)


def draw_route(rec, path, path_index):
    rec.prims.append(("strip", tuple((F(p[0]), F(p[1])) for p in path), 2.0, RouteCyan))
    target_idx = int(path_index) + 10
    if target_idx < 0:
        target_idx = 0
    if target_idx >= len(path):
        target_idx = len(path) - 1
    rec.draw_circle(path[target_idx][0], path[target_idx][1], 4.0, 10, TargetRed)


def draw_one(rec, car, col, npc):
    x, y, heading, alive = car
    if not alive:
        return
    x, y, heading = F(x), F(y), F(heading)
    length, wid = CAR_LENGTH, CAR_WIDTH
    hl, hw = length * F(0.5), wid * F(0.5)

    def rot(lx, ly):
        lx, ly = F(lx), F(ly)
        vx = lx * F(math.cos(-heading)) - ly * F(math.sin(-heading))
        vy = lx * F(math.sin(-heading)) + ly * F(math.cos(-heading))
        return (x + vx, y + vy)

    rec.prims.append(("quad", (rot(+hl, +hw), rot(+hl, -hw), rot(-hl, -hw), rot(-hl, +hw)), col))
    m = TrafficHeadBlack if npc else AgentHeadMarker
    x0 = -hl + F(0.70) * length
    x1 = -hl + F(0.95) * length
    y0 = -hw + F(2.0)
    y1 = +hw - F(2.0)
    rec.prims.append(("quad", (rot(x0, y0), rot(x1, y0), rot(x1, y1), rot(x0, y1)), m))


COLORS = [rgba(231 / 255, 76 / 255, 60 / 255), rgba(52 / 255, 152 / 255, 219 / 255),
          rgba(46 / 255, 204 / 255, 113 / 255), rgba(155 / 255, 89 / 255, 182 / 255),
          rgba(241 / 255, 196 / 255, 15 / 255), rgba(230 / 255, 126 / 255, 34 / 255)]


def draw_cars(rec, cars, npcs):
    for idx, car in enumerate(cars):
        draw_one(rec, car, COLORS[idx % len(COLORS)], False)
    for npc in npcs:
        draw_one(rec, npc, TrafficBodyGray, True)


def draw_lidar(rec, cars, lidars):
    for car, lid in zip(cars, lidars):
        x, y, heading, alive = car
        if not alive:
            continue
        distances, rel_angles, max_dist = lid
        for k in range(len(distances)):
            dist = F(distances[k])
            hit = dist < F(max_dist) - F(0.1)
            if not hit:
                continue
            ang = F(heading) + F(rel_angles[k])
            ex = F(x) + dist * F(math.cos(ang))
            ey = F(y) - dist * F(math.sin(ang))
            rec.draw_line(x, y, ex, ey, 2.0, LidarRayGreen)
            rec.draw_circle(ex, ey, 2.0, 6, LidarHitRed)


def rel_angles(rays, fov_deg=360.0):
    """IntersectionEnv.cpp:119-127."""
    start_angle_deg = -F(fov_deg) * F(0.5)
    step_deg = F(fov_deg) / F(rays - 1) if rays > 1 else F(0.0)
    PI_F2 = F(3.14159265358979323846)
    return [(start_angle_deg + F(ii) * step_deg) * PI_F2 / F(180.0) for ii in range(rays)]


def render_scene(num_lanes, cars, npcs, lidars, route0):
    """Renderer::render (:202-234): road, route, cars, LiDAR (show_lidar)."""
    rec = Recorder()
    draw_road(rec, num_lanes)
    if route0 is not None and cars:
        draw_route(rec, *route0)
    draw_cars(rec, cars, npcs)
    if lidars is not None:
        draw_lidar(rec, cars, lidars)
    return rec.prims
