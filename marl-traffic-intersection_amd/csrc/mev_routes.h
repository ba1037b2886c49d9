// mev_routes.h — host-side lane layout and route-table builder.
//
// Restates reference cpp/RouteGen.cpp (build_lane_layout_cpp :7-53,
// determine_intent :55-87, project_to_box :89-101, bezier_point :103-109,
// generate_path_cpp :111-205) and the spawn heading of
// IntersectionEnv::add_car_with_route (cpp/IntersectionEnv.cpp:88-93).
// Instead of string-keyed maps, lane points are integers:
//   point p < 4L  is "IN_{p+1}",  point p >= 4L is "OUT_{p-4L+1}".
// Every (start, end) pair is precomputed once per handle and uploaded as a
// constant table; cars then carry a route id = start * 8L + end.
// Trig goes through mev_math.h (bit-identical to glibc; no compile-time folding).
#pragma once

#include <stdint.h>

#include <vector>

#include "mev_world.h"

namespace mev {

struct LanePoint {
    float x, y;
    char dir;  // 'N','E','S','W'
    int idx;   // lane index j within its direction
};

inline std::vector<LanePoint> build_lane_points(int num_lanes) {
    const float CX = WIDTH * 0.5f;
    const float CY = HEIGHT * 0.5f;
    const float MARGIN = 30.0f;
    const char dirs[4] = {'N', 'E', 'S', 'W'};
    std::vector<LanePoint> pts(size_t(8 * num_lanes));
    for (int d_idx = 0; d_idx < 4; ++d_idx) {
        const char d = dirs[d_idx];
        for (int j = 0; j < num_lanes; ++j) {
            const float offset = LANE_WIDTH_PX * (0.5f + float(j));
            float in_x = 0, in_y = 0, out_x = 0, out_y = 0;
            if (d == 'N') { in_x = CX - offset; in_y = MARGIN; out_x = CX + offset; out_y = MARGIN; }
            else if (d == 'S') { in_x = CX + offset; in_y = HEIGHT - MARGIN; out_x = CX - offset; out_y = HEIGHT - MARGIN; }
            else if (d == 'E') { in_x = WIDTH - MARGIN; in_y = CY - offset; out_x = WIDTH - MARGIN; out_y = CY + offset; }
            else { in_x = MARGIN; in_y = CY + offset; out_x = MARGIN; out_y = CY - offset; }
            const int k = d_idx * num_lanes + j;
            pts[size_t(k)] = {in_x, in_y, d, j};
            pts[size_t(4 * num_lanes + k)] = {out_x, out_y, d, j};
        }
    }
    return pts;
}

inline char opposite_dir(char d) { return d == 'N' ? 'S' : d == 'S' ? 'N' : d == 'E' ? 'W' : 'E'; }
inline char left_dir(char d) { return d == 'N' ? 'E' : d == 'E' ? 'S' : d == 'S' ? 'W' : 'N'; }
inline char right_dir(char d) { return d == 'N' ? 'W' : d == 'W' ? 'S' : d == 'S' ? 'E' : 'N'; }

inline int route_intent(const LanePoint& s, const LanePoint& e) {
    if (e.dir == opposite_dir(s.dir)) return INTENT_STRAIGHT;
    if (e.dir == left_dir(s.dir)) return INTENT_LEFT;
    if (e.dir == right_dir(s.dir)) return INTENT_RIGHT;
    return INTENT_LEFT;
}

inline void project_to_box(float x, float y, int num_lanes, float* ox, float* oy) {
    const float CX = WIDTH * 0.5f;
    const float CY = HEIGHT * 0.5f;
    const float turn_bound = num_lanes * LANE_WIDTH_PX;
    const float bx_l = CX - turn_bound, bx_r = CX + turn_bound;
    const float by_t = CY - turn_bound, by_b = CY + turn_bound;
    if (y < by_t) { *ox = x; *oy = by_t; return; }
    if (y > by_b) { *ox = x; *oy = by_b; return; }
    if (x < bx_l) { *ox = bx_l; *oy = y; return; }
    *ox = bx_r;
    *oy = y;
}

// Fills path[PATH_LEN][2]; returns the intent.
inline int generate_route(const std::vector<LanePoint>& pts, int num_lanes, int start, int end, float* path) {
    const float CX = WIDTH * 0.5f;
    const float CY = HEIGHT * 0.5f;
    const LanePoint& ps = pts[size_t(start)];
    const LanePoint& pe = pts[size_t(end)];
    const int intent = route_intent(ps, pe);
    float ex, ey, xx, xy;
    project_to_box(ps.x, ps.y, num_lanes, &ex, &ey);
    project_to_box(pe.x, pe.y, num_lanes, &xx, &xy);
    int o = 0;
    auto push = [&](float a, float b) { path[2 * o] = a; path[2 * o + 1] = b; ++o; };
    if (intent == INTENT_STRAIGHT || intent == INTENT_LEFT) {
        for (int i = 0; i < 50; ++i) {
            const float t = float(i) / 50.0f;
            push(ps.x + (ex - ps.x) * t, ps.y + (ey - ps.y) * t);
        }
        for (int i = 0; i < 60; ++i) {
            const float t = float(i) / 60.0f;
            if (intent == INTENT_STRAIGHT) {
                push(ex + (xx - ex) * t, ey + (xy - ey) * t);
            } else {
                // quadratic Bezier with control point at the box centre
                const float u = 1 - t;
                push(u * u * ex + 2 * u * t * CX + t * t * xx, u * u * ey + 2 * u * t * CY + t * t * xy);
            }
        }
        for (int i = 0; i < 50; ++i) {
            const float t = float(i) / 50.0f;
            push(xx + (pe.x - xx) * t, xy + (pe.y - xy) * t);
        }
        return intent;
    }
    // right turn: circular arc around the corner's grass circle
    const float road_half_width = num_lanes * LANE_WIDTH_PX;
    float cx_c, cy_c, th0, th1;
    if (ps.dir == 'N') { cx_c = CX - road_half_width - CORNER_RADIUS; cy_c = CY - road_half_width - CORNER_RADIUS; th0 = 0.0f; th1 = PI_F / 2.0f; }
    else if (ps.dir == 'E') { cx_c = CX + road_half_width + CORNER_RADIUS; cy_c = CY - road_half_width - CORNER_RADIUS; th0 = PI_F / 2.0f; th1 = PI_F; }
    else if (ps.dir == 'S') { cx_c = CX + road_half_width + CORNER_RADIUS; cy_c = CY + road_half_width + CORNER_RADIUS; th0 = PI_F; th1 = 3.0f * PI_F / 2.0f; }
    else { cx_c = CX - road_half_width - CORNER_RADIUS; cy_c = CY + road_half_width + CORNER_RADIUS; th0 = -PI_F / 2.0f; th1 = 0.0f; }
    const float r = CORNER_RADIUS + 0.5f * LANE_WIDTH_PX;
    float s0, c0, s1, c1;
    sincosf(th0, &s0, &c0);
    sincosf(th1, &s1, &c1);
    const float as_x = cx_c + r * c0, as_y = cy_c + r * s0;
    const float ae_x = cx_c + r * c1, ae_y = cy_c + r * s1;
    for (int i = 0; i < 50; ++i) {
        const float t = float(i) / 50.0f;
        push(ps.x + (as_x - ps.x) * t, ps.y + (as_y - ps.y) * t);
    }
    for (int i = 0; i < 60; ++i) {
        const float t = float(i) / 60.0f;
        const float theta = th0 + (th1 - th0) * t;
        float st, ct;
        sincosf(theta, &st, &ct);
        push(cx_c + r * ct, cy_c + r * st);
    }
    for (int i = 0; i < 50; ++i) {
        const float t = float(i) / 50.0f;
        push(ae_x + (pe.x - ae_x) * t, ae_y + (pe.y - ae_y) * t);
    }
    return intent;
}

// Heading of a car spawned on a path: atan2(-dy, dx) of its first segment
// (cpp/IntersectionEnv.cpp:88-93, cpp/TrafficFlow.cpp:293-298).
inline float spawn_heading(const float* path) {
    const float dx = path[2] - path[0];
    const float dy = path[3] - path[1];
    return atan2f(-dy, dx);
}

// Reference default NPC route list (init_traffic_routes, cpp/TrafficFlow.cpp:198-238):
// for each direction N,E,S,W and each IN lane j: (IN, straight OUT[j]), (IN, left OUT[j]).
inline std::vector<int> default_traffic_routes(int num_lanes) {
    std::vector<int> routes;
    const char dirs[4] = {'N', 'E', 'S', 'W'};
    auto dir_index = [&](char d) { for (int k = 0; k < 4; ++k) if (dirs[k] == d) return k; return 0; };
    const int P = 8 * num_lanes;
    for (int d_idx = 0; d_idx < 4; ++d_idx) {
        const int so = dir_index(opposite_dir(dirs[d_idx]));
        const int lo = dir_index(left_dir(dirs[d_idx]));
        for (int j = 0; j < num_lanes; ++j) {
            const int start = d_idx * num_lanes + j;
            routes.push_back(start * P + 4 * num_lanes + so * num_lanes + j);
            routes.push_back(start * P + 4 * num_lanes + lo * num_lanes + j);
        }
    }
    return routes;
}

}  // namespace mev
