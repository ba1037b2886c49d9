// TEST INFRASTRUCTURE ONLY — never shipped, never measured as the product.
//
// C-callable harness around the UNMODIFIED reference simulator
// (/root/reference/cpp, compiled in place by oracle/build_ref.sh into
// $MEV_REF_BUILD/libref_harness.so, outside the repository).  It is used for exactly two things:
//   1. generating the golden vectors under tests/golden/ (tests/golden/gen_golden.py);
//   2. the `cpu_baseline` leg of bench.py (kind "reference").
//
// Nothing here re-implements simulator behaviour: every step, observation and
// reward comes from the reference's own IntersectionEnv::step /
// get_observations (cpp/IntersectionEnv.cpp:133-520, cpp/TrafficFlow.cpp:317-367).
// The harness only (a) reads/writes the public Car members the pybind layer
// does not expose (cpp/Car.h:16-46), (b) replaces the ego LiDAR objects with an
// R-beam one built by the same formula as cpp/IntersectionEnv.cpp:111-128, and
// (c) records which NPC the reference's unseeded RNG spawned each step
// (cpp/TrafficFlow.cpp:275-329) so that the device path can replay it.
#include "IntersectionEnv.h"

#include <chrono>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <random>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

namespace {

enum StatusCode { ST_ALIVE = 0, ST_DEAD = 1, ST_SUCCESS = 2, ST_CRASH_WALL = 3, ST_CRASH_LINE = 4, ST_CRASH_CAR = 5 };

int status_code(const std::string& s) {
    if (s == "ALIVE") return ST_ALIVE;
    if (s == "DEAD") return ST_DEAD;
    if (s == "SUCCESS") return ST_SUCCESS;
    if (s == "CRASH_WALL") return ST_CRASH_WALL;
    if (s == "CRASH_LINE") return ST_CRASH_LINE;
    if (s == "CRASH_CAR") return ST_CRASH_CAR;
    return -1;
}

struct Harness {
    IntersectionEnv env;
    // Route bookkeeping so the harness can name the route of every car.
    std::vector<std::vector<std::pair<float, float>>> npc_route_paths;  // index = traffic_routes idx
    std::vector<int> ego_route_of;  // per ego car, caller-provided tag
    // paths of the caller's own, written into Car.path (cpp/bindings.cpp:29: a plain
    // read-write member, assigned without Car::set_path, so path_index stays)
    std::vector<std::vector<std::pair<float, float>>> custom_paths;
    int lidar_rays{96};
    float lidar_fov{360.0f}, lidar_max{250.0f}, lidar_step{4.0f};
    explicit Harness(int lanes) : env(lanes) {}

    void rebuild_npc_route_paths() {
        npc_route_paths.clear();
        for (const auto& r : env.traffic_routes) {
            try {
                int intent = determine_intent(env.lane_layout, r.first, r.second);
                npc_route_paths.push_back(generate_path_cpp(env.lane_layout, env.num_lanes, intent, r.first, r.second));
            } catch (...) {
                npc_route_paths.emplace_back();
            }
        }
    }
    // the traffic-route index of an NPC's path, 1000 + k for custom path k, or -1
    int npc_route_index(const Car& c) const {
        for (size_t i = 0; i < npc_route_paths.size(); ++i)
            if (npc_route_paths[i] == c.path) return int(i);
        for (size_t i = 0; i < custom_paths.size(); ++i)
            if (custom_paths[i] == c.path) return 1000 + int(i);
        return -1;
    }
    // Same LiDAR construction as cpp/IntersectionEnv.cpp:111-128, with R rays.
    Lidar make_lidar() const {
        Lidar lid;
        lid.rays = lidar_rays;
        lid.fov_deg = lidar_fov;
        lid.max_dist = lidar_max;
        lid.step_size = lidar_step;
        lid.distances.assign(lid.rays, lid.max_dist);
        lid.rel_angles.clear();
        const float start_angle_deg = -lid.fov_deg * 0.5f;
        const float step_deg = (lid.rays > 1) ? (lid.fov_deg / float(lid.rays - 1)) : 0.0f;
        constexpr float PI_F2 = 3.14159265358979323846f;
        for (int ii = 0; ii < lid.rays; ++ii) {
            float deg = start_angle_deg + ii * step_deg;
            lid.rel_angles.push_back(deg * PI_F2 / 180.0f);
        }
        return lid;
    }
};

// Car record exchanged with Python: 15 floats + 4 ints.
constexpr int NF = 15;
constexpr int NI = 4;

void car_to_rec(const Car& c, int route, float* f, int32_t* i) {
    f[0] = c.state.x; f[1] = c.state.y; f[2] = c.state.v; f[3] = c.state.heading;
    f[4] = c.acc; f[5] = c.steering_angle;
    f[6] = c.spawn_state.x; f[7] = c.spawn_state.y; f[8] = c.spawn_state.v; f[9] = c.spawn_state.heading;
    f[10] = c.prev_dist_to_goal; f[11] = c.prev_action.first; f[12] = c.prev_action.second;
    f[13] = c.length; f[14] = c.width;
    i[0] = c.alive ? 1 : 0; i[1] = c.intention; i[2] = c.path_index; i[3] = route;
}

void rec_to_car(const float* f, const int32_t* i, Car& c) {
    c.state.x = f[0]; c.state.y = f[1]; c.state.v = f[2]; c.state.heading = f[3];
    c.acc = f[4]; c.steering_angle = f[5];
    c.spawn_state.x = f[6]; c.spawn_state.y = f[7]; c.spawn_state.v = f[8]; c.spawn_state.heading = f[9];
    c.prev_dist_to_goal = f[10]; c.prev_action = {f[11], f[12]};
    c.length = f[13]; c.width = f[14];
    c.alive = i[0] != 0; c.intention = i[1]; c.path_index = i[2];
}

}  // namespace

extern "C" {

int rh_record_floats() { return NF; }
int rh_record_ints() { return NI; }

void* rh_create(int num_lanes) {
    auto* h = new Harness(num_lanes);
    h->rebuild_npc_route_paths();
    return h;
}
void rh_destroy(void* p) { delete static_cast<Harness*>(p); }

void rh_configure(void* p, int use_team, int respawn, int max_steps) {
    static_cast<Harness*>(p)->env.configure(use_team != 0, respawn != 0, max_steps);
}
void rh_configure_traffic(void* p, int enabled, float density) {
    static_cast<Harness*>(p)->env.configure_traffic(enabled != 0, density);
}
// routes given as "START END" pairs separated by ';'
void rh_configure_routes(void* p, const char* spec) {
    auto* h = static_cast<Harness*>(p);
    std::vector<std::pair<std::string, std::string>> routes;
    std::string s(spec);
    size_t pos = 0;
    while (pos < s.size()) {
        size_t semi = s.find(';', pos);
        if (semi == std::string::npos) semi = s.size();
        std::string item = s.substr(pos, semi - pos);
        size_t sp = item.find(' ');
        if (sp != std::string::npos) routes.emplace_back(item.substr(0, sp), item.substr(sp + 1));
        pos = semi + 1;
    }
    h->env.configure_routes(routes);
    h->rebuild_npc_route_paths();
}
int rh_num_traffic_routes(void* p) { return int(static_cast<Harness*>(p)->env.traffic_routes.size()); }

void rh_set_reward(void* p, const float* rc) {
    auto& r = static_cast<Harness*>(p)->env.reward_config;
    r.k_prog = rc[0]; r.v_min_ms = rc[1]; r.k_stuck = rc[2]; r.k_cv = rc[3];
    r.k_co = rc[4]; r.k_succ = rc[5]; r.k_sm = rc[6]; r.alpha = rc[7];
}

void rh_set_lidar(void* p, int rays, float fov, float maxd, float step) {
    auto* h = static_cast<Harness*>(p);
    h->lidar_rays = rays; h->lidar_fov = fov; h->lidar_max = maxd; h->lidar_step = step;
    for (auto& l : h->env.lidars) l = h->make_lidar();
}

// IntersectionEnv.lidars[i] = a Lidar whose fields the caller wrote (cpp/bindings.cpp:68,
// 85-92: Lidar() then rays / fov_deg / max_dist / step_size / rel_angles assigned as
// plain members; distances stay as Lidar() made them -- update() resizes them).
void rh_set_car_lidar(void* p, int i, int rays, float fov, float maxd, float step, const float* rel, int nrel) {
    auto* h = static_cast<Harness*>(p);
    Lidar l;
    l.rays = rays;
    l.fov_deg = fov;
    l.max_dist = maxd;
    l.step_size = step;
    if (rel) l.rel_angles.assign(rel, rel + nrel);
    h->env.lidars.at(size_t(i)) = l;
}

void rh_reset(void* p) {
    auto* h = static_cast<Harness*>(p);
    h->env.reset();
    h->ego_route_of.clear();
}

// 0 = added, 1 = unknown start (reference silently skips), 2 = unknown end (reference throws)
int rh_add_car(void* p, const char* start, const char* end, int route_tag) {
    auto* h = static_cast<Harness*>(p);
    size_t before = h->env.cars.size();
    try {
        h->env.add_car_with_route(start, end);
    } catch (const std::out_of_range&) {
        return 2;
    }
    if (h->env.cars.size() == before) return 1;
    h->ego_route_of.push_back(route_tag);
    // Non-default beam count: replace the LiDAR object just created.
    if (h->lidar_rays != 96 || h->lidar_fov != 360.0f || h->lidar_max != 250.0f || h->lidar_step != 4.0f)
        h->env.lidars.back() = h->make_lidar();
    return 0;
}

// IntersectionEnv::set_state(get_state()) (cpp/IntersectionEnv.cpp:394-416): the
// same cars, NPCs, ids and step count, and -- the point of the round trip --
// every LiDAR object rebuilt as a default Lidar() (72 rays, cpp/Lidar.h:11).
void rh_state_roundtrip(void* p) {
    auto* h = static_cast<Harness*>(p);
    const EnvState s = h->env.get_state();
    h->env.set_state(s);
}

int rh_num_cars(void* p) { return int(static_cast<Harness*>(p)->env.cars.size()); }
int rh_num_npcs(void* p) { return int(static_cast<Harness*>(p)->env.traffic_cars.size()); }
int rh_step_count(void* p) { return static_cast<Harness*>(p)->env.step_count; }

void rh_get_cars(void* p, int which, float* f, int32_t* i) {
    auto* h = static_cast<Harness*>(p);
    if (which == 0) {
        for (size_t k = 0; k < h->env.cars.size(); ++k)
            car_to_rec(h->env.cars[k], k < h->ego_route_of.size() ? h->ego_route_of[k] : -1, f + k * NF, i + k * NI);
    } else {
        for (size_t k = 0; k < h->env.traffic_cars.size(); ++k)
            car_to_rec(h->env.traffic_cars[k], h->npc_route_index(h->env.traffic_cars[k]), f + k * NF, i + k * NI);
    }
}

// Overwrite ego k with a record (path stays the one of its route).
void rh_set_car(void* p, int k, const float* f, const int32_t* i) {
    rec_to_car(f, i, static_cast<Harness*>(p)->env.cars[size_t(k)]);
}

// Append an NPC on traffic route `route` with the given record (state injection).
int rh_add_npc(void* p, int route, const float* f, const int32_t* i) {
    auto* h = static_cast<Harness*>(p);
    if (route < 0 || size_t(route) >= h->env.traffic_routes.size()) return 1;
    const auto& r = h->env.traffic_routes[size_t(route)];
    Car c;
    c.intention = determine_intent(h->env.lane_layout, r.first, r.second);
    c.path = generate_path_cpp(h->env.lane_layout, h->env.num_lanes, c.intention, r.first, r.second);
    rec_to_car(f, i, c);
    h->env.traffic_cars.push_back(std::move(c));
    h->env.traffic_lidars.emplace_back();
    return 0;
}

// A path of the caller's own (n points, xy interleaved); returns its index.
int rh_add_custom_path(void* p, const float* xy, int n) {
    auto* h = static_cast<Harness*>(p);
    std::vector<std::pair<float, float>> path;
    for (int k = 0; k < n; ++k) path.emplace_back(xy[2 * k], xy[2 * k + 1]);
    h->custom_paths.push_back(std::move(path));
    return int(h->custom_paths.size()) - 1;
}

// Car.path = custom path `custom` of ego k (which 0) or NPC k (which 1): the member
// assignment pybind's def_readwrite performs (cpp/bindings.cpp:29), nothing else changes.
int rh_set_car_path(void* p, int which, int k, int custom) {
    auto* h = static_cast<Harness*>(p);
    if (custom < 0 || size_t(custom) >= h->custom_paths.size()) return 1;
    auto& v = which == 0 ? h->env.cars : h->env.traffic_cars;
    if (k < 0 || size_t(k) >= v.size()) return 1;
    v[size_t(k)].path = h->custom_paths[size_t(custom)];
    return 0;
}

// The 160-point path of traffic route `route` as generated by the reference
// (cpp/RouteGen.cpp:111-205); returns the point count.
int rh_route_path(void* p, int route, float* out) {
    auto* h = static_cast<Harness*>(p);
    if (route < 0 || size_t(route) >= h->npc_route_paths.size()) return 0;
    const auto& path = h->npc_route_paths[size_t(route)];
    for (size_t k = 0; k < path.size(); ++k) { out[2 * k] = path[k].first; out[2 * k + 1] = path[k].second; }
    return int(path.size());
}

// Reference geometry probes (cpp/RoadGeometry.h:19-67, cpp/LineMask.h:15-18)
// evaluated on the 750x750 integer pixel grid: out[y*750+x] bit0 = is_on_road,
// bit1 = hits_yellow_line, bit2 = LineMask::is_line.
void rh_geometry_grid(int num_lanes, uint8_t* out) {
    RoadGeometry geom(num_lanes);
    LineMask lm(num_lanes);
    for (int y = 0; y < HEIGHT; ++y)
        for (int x = 0; x < WIDTH; ++x) {
            uint8_t v = 0;
            if (geom.is_on_road(float(x), float(y))) v |= 1;
            if (geom.hits_yellow_line(float(x), float(y))) v |= 2;
            if (lm.is_line(x, y)) v |= 4;
            out[y * WIDTH + x] = v;
        }
}
int rh_is_on_road(int num_lanes, float x, float y) { return RoadGeometry(num_lanes).is_on_road(x, y) ? 1 : 0; }
int rh_hits_yellow_line(int num_lanes, float x, float y) { return RoadGeometry(num_lanes).hits_yellow_line(x, y) ? 1 : 0; }

// Raw LiDAR distances of every ego (n x rays).
void rh_get_lidar(void* p, float* out) {
    auto* h = static_cast<Harness*>(p);
    size_t o = 0;
    for (const auto& l : h->env.lidars)
        for (float d : l.distances) out[o++] = d;
}

void rh_get_obs(void* p, float* out) {
    auto obs = static_cast<Harness*>(p)->env.get_observations();
    size_t o = 0;
    for (const auto& row : obs)
        for (float v : row) out[o++] = v;
}

// One reference step.  Outputs sized by the current ego count n (obs n x 127).
// `spawned` receives the traffic-route index of the NPC the reference spawned
// during this step, or -1.
int rh_step(void* p, int n_act, const float* thr, const float* st, float dt,
            float* obs, float* rew, int32_t* done, int32_t* status, int32_t* flags /*term,trunc,alive,step*/,
            int32_t* spawned) {
    auto* h = static_cast<Harness*>(p);
    // Identity of NPCs before the step (route index + position) for spawn detection.
    struct Id { int route; float x, y; };
    std::vector<Id> before;
    for (const auto& c : h->env.traffic_cars) before.push_back({h->npc_route_index(c), c.state.x, c.state.y});

    std::vector<float> t(thr, thr + n_act), s(st, st + n_act);
    StepResult res = h->env.step(t, s, dt);

    *spawned = -1;
    {
        size_t bp = 0;
        const auto& after = h->env.traffic_cars;
        for (size_t q = 0; q < after.size(); ++q) {
            int rq = h->npc_route_index(after[q]);
            bool matched = false;
            while (bp < before.size()) {
                const Id& b = before[bp++];
                if (b.route == rq && std::fabs(b.x - after[q].state.x) <= 10.0f &&
                    std::fabs(b.y - after[q].state.y) <= 10.0f) { matched = true; break; }
            }
            if (!matched) {
                if (q + 1 != after.size()) return -10;  // a new NPC can only be appended
                *spawned = rq;
            }
        }
    }

    const size_t n = res.rewards.size();
    size_t o = 0;
    for (const auto& row : res.obs)
        for (float v : row) obs[o++] = v;
    for (size_t k = 0; k < n; ++k) {
        rew[k] = res.rewards[k];
        done[k] = res.done[k];
        status[k] = status_code(res.status[k]);
    }
    flags[0] = res.terminated ? 1 : 0;
    flags[1] = res.truncated ? 1 : 0;
    flags[2] = res.agents_alive;
    flags[3] = res.step;
    return int(n);
}

// Reference CPU throughput: `threads` workers, each owning `envs_per_thread`
// independent IntersectionEnv instances, stepping `steps` times with uniform
// [-1,1) actions and auto-reset on terminated/truncated (the survey's
// mp_bench protocol without the Python layer).  Returns agent-steps/s.
double rh_bench(int num_lanes, int num_agents, int rays, int use_team, int traffic, float density,
                int envs_per_thread, int steps, int threads, unsigned seed) {
    static const char* k3[12][2] = {{"IN_1", "OUT_4"}, {"IN_2", "OUT_8"}, {"IN_3", "OUT_12"}, {"IN_4", "OUT_7"},
                                    {"IN_5", "OUT_11"}, {"IN_6", "OUT_3"}, {"IN_7", "OUT_10"}, {"IN_8", "OUT_2"},
                                    {"IN_9", "OUT_6"}, {"IN_10", "OUT_1"}, {"IN_11", "OUT_5"}, {"IN_12", "OUT_9"}};
    if (num_lanes != 3) return -1.0;
    auto worker = [&](int tid, long long* agent_steps) {
        std::mt19937 rng(seed + 7919u * unsigned(tid));
        std::uniform_real_distribution<float> U(-1.0f, 1.0f);
        std::vector<Harness*> hs;
        std::string routes;
        for (int r = 0; r < 12; ++r) { routes += k3[r][0]; routes += ' '; routes += k3[r][1]; routes += ';'; }
        const int n = traffic ? 1 : num_agents;
        for (int e = 0; e < envs_per_thread; ++e) {
            Harness* h = static_cast<Harness*>(rh_create(num_lanes));
            rh_configure(h, traffic ? 0 : use_team, 1, 2000);
            rh_configure_traffic(h, traffic, density);
            rh_configure_routes(h, routes.c_str());
            rh_set_lidar(h, rays, 360.0f, 250.0f, 4.0f);
            hs.push_back(h);
        }
        auto do_reset = [&](Harness* h) {
            rh_reset(h);
            for (int i = 0; i < n; ++i) rh_add_car(h, k3[i % 12][0], k3[i % 12][1], i % 12);
        };
        for (auto* h : hs) do_reset(h);
        std::vector<float> thr(static_cast<size_t>(n)), st(static_cast<size_t>(n));
        long long cnt = 0;
        for (int s = 0; s < steps; ++s) {
            for (auto* h : hs) {
                for (int i = 0; i < n; ++i) { thr[size_t(i)] = U(rng); st[size_t(i)] = U(rng); }
                StepResult res = h->env.step(thr, st, 1.0f / 60.0f);
                cnt += n;
                if (res.terminated || res.truncated) do_reset(h);
            }
        }
        for (auto* h : hs) rh_destroy(h);
        *agent_steps = cnt;
    };
    std::vector<long long> counts(size_t(threads), 0);
    auto t0 = std::chrono::steady_clock::now();
    std::vector<std::thread> pool;
    for (int t = 0; t < threads; ++t) pool.emplace_back(worker, t, &counts[size_t(t)]);
    for (auto& th : pool) th.join();
    double sec = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    long long total = 0;
    for (auto c : counts) total += c;
    return double(total) / sec;
}

}  // extern "C"
