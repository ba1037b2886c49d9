// mev_world.h — static world + per-car arithmetic of the intersection, shared
// by the gfx950 kernels and the host route builder.  Every expression keeps
// the reference's evaluation order (compile with -ffp-contract=off); the
// reference file:line each piece restates is cited inline.
#pragma once

#include "mev_math.h"

namespace mev {

// reference cpp/constants.h:4-20, cpp/IntersectionEnv.h:19
constexpr int WIDTH = 750;
constexpr int HEIGHT = 750;
constexpr float SCALE = 12.0f;
constexpr float FPS = 60.0f;
constexpr float CAR_LENGTH = 54.0f;
constexpr float CAR_WIDTH = 24.0f;
constexpr float WHEELBASE = CAR_LENGTH;
constexpr float LANE_WIDTH_PX = 42.0f;
constexpr float CORNER_RADIUS = 84.0f;
constexpr float MAX_ACC = 15.0f;
constexpr float MAX_STEERING_ANGLE = 0.6108652381980153f;
constexpr float PHYSICS_MAX_SPEED = 8.0f;
constexpr float PI_F = 3.14159265358979323846f;
constexpr int NEIGHBOR_COUNT = 5;
constexpr int PATH_LEN = 160;  // 50 + 60 + 50 points (cpp/RouteGen.cpp:160-237)
// A route-table row: the path's PATH_LEN points, then at ROUTE_END, ROUTE_END + 1 its
// last segment (path[n-2], path[n-1]) for the SUCCESS axis (IntersectionEnv.cpp:177-182),
// then zeros up to ROUTE_PTS points (1408 B: rows stay aligned to 128-B lines).  A
// written Car.path of n < PATH_LEN points is stored padded with its last point:
// every other read of a path -- the index search's first minimum (Car.cpp:56-73),
// the look-ahead targets clamped to n-1 (IntersectionEnv.cpp:446, TrafficFlow.cpp:55),
// the ghost scan (TrafficFlow.cpp:89-185: a repeated point repeats its verdict),
// path.back() -- then reads exactly what the n-point path gives.
// (A table with a written path longer than PATH_LEN has rows of plen = that length rounded
// up to 16 points and plen + 16 points per row, the last segment at plen: RouteTab.)
constexpr int ROUTE_END = PATH_LEN;
constexpr int ROUTE_PTS = 176;
constexpr int MAX_PATH_LEN = 4096;  // mev_add_route_n's bound on a written path
constexpr int OBS_HEAD = 6 + 5 * NEIGHBOR_COUNT;  // 31

enum Status : uint8_t { ST_ALIVE = 0, ST_DEAD = 1, ST_SUCCESS = 2, ST_CRASH_WALL = 3, ST_CRASH_LINE = 4, ST_CRASH_CAR = 5 };
enum Intent { INTENT_STRAIGHT = 0, INTENT_LEFT = 1, INTENT_RIGHT = 2 };

// wrap to [-pi, pi): cpp/IntersectionEnv.cpp:9-13 (and Car.cpp:33-36, TrafficFlow.cpp:8-12)
MEV_HD float wrap_angle(float a) {
    a = fmodf(a + PI_F, 2.0f * PI_F);
    if (a < 0) a += 2.0f * PI_F;
    return a - PI_F;
}

// RoadGeometry::is_on_road, cpp/RoadGeometry.h:19-58 (real-valued query, used for car corners).
MEV_HD bool is_on_road(float x, float y, float rw) {
    const float CX = WIDTH * 0.5f;
    const float CY = HEIGHT * 0.5f;
    const float cr = CORNER_RADIUS;
    const float r2 = cr * cr;
    const float gx[4] = {CX - rw - cr, CX + rw + cr, CX - rw - cr, CX + rw + cr};
    const float gy[4] = {CY - rw - cr, CY - rw - cr, CY + rw + cr, CY + rw + cr};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const float dx = x - gx[k];
        const float dy = y - gy[k];
        if (dx * dx + dy * dy <= r2) return false;
    }
    if ((x >= CX - rw && x <= CX + rw) || (y >= CY - rw && y <= CY + rw)) return true;
    if (x >= CX - rw - cr && x <= CX - rw && y >= CY - rw - cr && y <= CY - rw) return true;
    if (x >= CX + rw && x <= CX + rw + cr && y >= CY - rw - cr && y <= CY - rw) return true;
    if (x >= CX - rw - cr && x <= CX - rw && y >= CY + rw && y <= CY + rw + cr) return true;
    if (x >= CX + rw && x <= CX + rw + cr && y >= CY + rw && y <= CY + rw + cr) return true;
    return false;
}

// The same predicate at an integer pixel (the LiDAR march only ever asks at
// float(int) points, cpp/Lidar.cpp:44).  The road is symmetric about the
// centre lines, so with ax = |x-375|, ay = |y-375| (exact integers) it reduces
// to: not inside the one grass circle centred at (rw+cr, rw+cr), and either in
// a strip (ax <= rw or ay <= rw) or in the corner square.  Exhaustively checked
// against the reference on the 750x750 grid (tests/test_geometry.py).
// irw = rw (integer when num_lanes*42 is), icr = 84.
MEV_HD bool is_on_road_px(int x, int y, int irw) {
    const int icr = 84;
    int ax = x - 375;
    ax = ax < 0 ? -ax : ax;
    int ay = y - 375;
    ay = ay < 0 ? -ay : ay;
    const int dx = ax - (irw + icr);
    const int dy = ay - (irw + icr);
    if (dx * dx + dy * dy <= icr * icr) return false;
    if (ax <= irw || ay <= irw) return true;
    return ax <= irw + icr && ay <= irw + icr;
}

// RoadGeometry::hits_yellow_line, cpp/RoadGeometry.h:60-67
MEV_HD bool hits_yellow_line(float x, float y, float rw) {
    const float cx = WIDTH * 0.5f;
    const float cy = HEIGHT * 0.5f;
    const float gap = 2.0f;
    if (fabs_f(x - cx) <= gap && fabs_f(y - cy) > rw) return true;
    if (fabs_f(y - cy) <= gap && fabs_f(x - cx) > rw) return true;
    return false;
}

// LineMask::is_line, cpp/LineMask.h:15-18 over the grid drawn by
// cpp/LineMask.cpp:47-72 (8 three-pixel strips), as a closed-form test.
// stop = int(L*int(42)) + 84.
MEV_HD bool is_line_px(int x, int y, int stop) {
    if (x < 0 || x >= WIDTH || y < 0 || y >= HEIGHT) return false;
    const int c = WIDTH / 2;  // 375 (== HEIGHT / 2)
    const bool xband = (x >= c - 3 && x <= c - 1) || (x >= c + 1 && x <= c + 3);
    const bool yband = (y >= c - 3 && y <= c - 1) || (y >= c + 1 && y <= c + 3);
    const bool yout = (y <= c - stop) || (y >= c + stop);
    const bool xout = (x <= c - stop) || (x >= c + stop);
    return (xband && yout) || (yband && xout);
}

// Car::corners, cpp/Car.cpp:86-103 (y-up rotation kept: SURVEY §7.3 quirk 6), for a
// car of length len and width wid (Car::length / Car::width, cpp/Car.h:19-20).
MEV_HD void car_corners_d(float x, float y, float cosA, float sinA, float len, float wid, float* cx, float* cy) {
    const float hx = wid * 0.5f;
    const float hy = len * 0.5f;
    const float lx[4] = {hy, hy, -hy, -hy};
    const float ly[4] = {hx, -hx, -hx, hx};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        cx[k] = x + lx[k] * cosA - ly[k] * sinA;
        cy[k] = y + lx[k] * sinA + ly[k] * cosA;
    }
}
// the reference's default 54 x 24 px car (constant-folded)
MEV_HD void car_corners(float x, float y, float cosA, float sinA, float* cx, float* cy) {
    car_corners_d(x, y, cosA, sinA, CAR_LENGTH, CAR_WIDTH, cx, cy);
}

// project + Car::check_collision, cpp/Car.cpp:105-141 (SAT on 4 axes).
MEV_HD void sat_project(const float* px, const float* py, float ax, float ay, float* mn, float* mx) {
    float minP = __builtin_inff(), maxP = -__builtin_inff();
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const float proj = px[k] * ax + py[k] * ay;
        minP = (proj < minP) ? proj : minP;
        maxP = (maxP < proj) ? proj : maxP;
    }
    *mn = minP;
    *mx = maxP;
}

MEV_HD bool sat_collide(const float* c1x, const float* c1y, float cos1, float sin1,
                        const float* c2x, const float* c2y, float cos2, float sin2) {
    const float axx[4] = {cos1, -sin1, cos2, -sin2};
    const float axy[4] = {sin1, cos1, sin2, cos2};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        float mn1, mx1, mn2, mx2;
        sat_project(c1x, c1y, axx[k], axy[k], &mn1, &mx1);
        sat_project(c2x, c2y, axx[k], axy[k], &mn2, &mx2);
        if (mx1 < mn2 || mx2 < mn1) return false;
    }
    return true;
}

// Car::update, cpp/Car.cpp:9-40: kinematic bicycle, position without dt.
// Returns cos/sin of the new heading (reused by corners, SAT and LiDAR).
struct Kin {
    float x, y, v, h, acc, steer;
};
MEV_HD void car_update(Kin& k, float throttle, float steer_input, float dt, float* cosH, float* sinH) {
    k.acc = throttle * MAX_ACC;
    const float target_steering = steer_input * MAX_STEERING_ANGLE;
    k.steer += (target_steering - k.steer) * 0.2f;
    if (throttle == 0.0f) k.v *= 0.95f;
    k.v += k.acc * dt;
    if (k.v < 0.0f) k.v = 0.0f;
    if (k.v > PHYSICS_MAX_SPEED) k.v = PHYSICS_MAX_SPEED;
    if (fabs_f(k.v) > 0.1f) {
        const float ang_vel = (k.v / WHEELBASE) * tanf(k.steer);
        k.h += ang_vel;
    }
    k.h = fmodf(k.h + PI_F, 2.0f * PI_F);
    if (k.h < 0) k.h += 2.0f * PI_F;
    k.h -= PI_F;
    float s, c;
    sincosf(k.h, &s, &c);
    k.x += k.v * c;
    k.y -= k.v * s;
    *cosH = c;
    *sinH = s;
}

// Car::update up to its new heading (steering, speed, heading, wrapped): the
// caller takes sincosf of the heading and moves the position with
// car_update_move -- car_update's operations in its order, split so that a
// wave whose agents are partly dead (heading unchanged) runs one sincosf.
MEV_HD void car_update_heading(Kin& k, float throttle, float steer_input, float dt) {
    k.acc = throttle * MAX_ACC;
    const float target_steering = steer_input * MAX_STEERING_ANGLE;
    k.steer += (target_steering - k.steer) * 0.2f;
    if (throttle == 0.0f) k.v *= 0.95f;
    k.v += k.acc * dt;
    if (k.v < 0.0f) k.v = 0.0f;
    if (k.v > PHYSICS_MAX_SPEED) k.v = PHYSICS_MAX_SPEED;
    if (fabs_f(k.v) > 0.1f) {
        const float ang_vel = (k.v / WHEELBASE) * tanf(k.steer);
        k.h += ang_vel;
    }
    k.h = fmodf(k.h + PI_F, 2.0f * PI_F);
    if (k.h < 0) k.h += 2.0f * PI_F;
    k.h -= PI_F;
}
MEV_HD void car_update_move(Kin& k, float c, float s) {
    k.x += k.v * c;
    k.y -= k.v * s;
}

// Car::update split for the NPC controller, whose steering input is known
// before its throttle: car_steer is the steering part (its new angle), and
// car_update_steered the rest given that angle and its tangent -- the same
// operations in the same order as car_update.
MEV_HD float car_steer(float steer, float steer_input) {
    const float target_steering = steer_input * MAX_STEERING_ANGLE;
    return steer + (target_steering - steer) * 0.2f;
}
MEV_HD void car_update_steered(Kin& k, float throttle, float new_steer, float tan_steer, float dt, float* cosH,
                               float* sinH) {
    k.acc = throttle * MAX_ACC;
    k.steer = new_steer;
    if (throttle == 0.0f) k.v *= 0.95f;
    k.v += k.acc * dt;
    if (k.v < 0.0f) k.v = 0.0f;
    if (k.v > PHYSICS_MAX_SPEED) k.v = PHYSICS_MAX_SPEED;
    if (fabs_f(k.v) > 0.1f) {
        const float ang_vel = (k.v / WHEELBASE) * tan_steer;
        k.h += ang_vel;
    }
    k.h = fmodf(k.h + PI_F, 2.0f * PI_F);
    if (k.h < 0) k.h += 2.0f * PI_F;
    k.h -= PI_F;
    float s, c;
    sincosf(k.h, &s, &c);
    k.x += k.v * c;
    k.y -= k.v * s;
    *cosH = c;
    *sinH = s;
}

// LiDAR obstacle box: rotated rectangle's AABB (cpp/Lidar.cpp:65-75) turned
// into an inclusive integer pixel range — `float(px) >= x - ex` <=> px >= ceil(x - ex).
struct PxBox {
    int x0, x1, y0, y1;
};
// (len, wid: the car's Car::length / Car::width, Lidar.cpp:67-68)
MEV_HD PxBox aabb_px_d(float x, float y, float cosA, float sinA, float len, float wid) {
    const float hl = len * 0.5f;
    const float hw = wid * 0.5f;
    const float ex = fabs_f(cosA) * hl + fabs_f(sinA) * hw;
    const float ey = fabs_f(sinA) * hl + fabs_f(cosA) * hw;
    PxBox b;
    const float lx = x - ex, hx_ = x + ex, ly = y - ey, hy_ = y + ey;
    // clamp to a safe int range before converting (cars never leave [-1e6, 1e6])
    auto cl = [](float f) { return f < -1.0e6f ? -1.0e6f : (f > 1.0e6f ? 1.0e6f : f); };
    b.x0 = (int)__builtin_ceilf(cl(lx));
    b.x1 = (int)__builtin_floorf(cl(hx_));
    b.y0 = (int)__builtin_ceilf(cl(ly));
    b.y1 = (int)__builtin_floorf(cl(hy_));
    return b;
}
MEV_HD PxBox aabb_px(float x, float y, float cosA, float sinA) {
    return aabb_px_d(x, y, cosA, sinA, CAR_LENGTH, CAR_WIDTH);
}

}  // namespace mev
