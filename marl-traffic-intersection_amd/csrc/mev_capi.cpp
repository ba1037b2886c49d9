// mev_capi.cpp — the extern "C" boundary (include/marlenv.h): handle
// lifetime, route tables, device buffers and the host side of reset / step /
// state transfer.  Replaces the reference's pybind11 module MARLEnv
// (cpp/bindings.cpp:11-95); see INTEGRATION.md for the caller-side bindings.
#include "marlenv.h"

#include <hip/hip_runtime.h>
#include <math.h>
#include <rccl/rccl.h>
#include <string.h>

#include <atomic>
#include <chrono>
#include <mutex>
#include <cstdio>
#include <string>
#include <thread>
#include <vector>

#include "mev_kernels.h"
#include "mev_routes.h"
#include "mev_world.h"

namespace {

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
    g_err = msg;
    return code;
}

#define HIP_TRY(expr)                                                                          \
    do {                                                                                       \
        hipError_t _e = (expr);                                                                \
        if (_e != hipSuccess) return fail(MEV_E_HIP, std::string(#expr) + ": " + hipGetErrorString(_e)); \
    } while (0)

// reference utils.py:29-52 default ego route mappings (IN_k -> OUT_m), as point indices
const int kMap3[12][2] = {{1, 4}, {2, 8}, {3, 12}, {4, 7}, {5, 11}, {6, 3},
                          {7, 10}, {8, 2}, {9, 6}, {10, 1}, {11, 5}, {12, 9}};
const int kMap2[7][2] = {{1, 3}, {2, 6}, {3, 5}, {4, 8}, {6, 2}, {7, 1}, {8, 4}};

template <class T>
hipError_t dalloc(T** p, size_t n) {
    return hipMalloc(reinterpret_cast<void**>(p), (n ? n : 1) * sizeof(T));
}

}  // namespace

struct mev_handle {
    mev_config cfg{};
    int D = 0, lidar_slots = 0, P = 0, nroutes = 0;
    int route_cap = 0;  // routes the device route tables have room for (mev_add_route)
    std::vector<mev::LanePoint> pts;
    std::vector<float> h_paths, h_spawn;  // h_paths: [nroutes][row_pts][2] (mev_world.h)
    std::vector<int32_t> h_len;           // points of each route's path (2 .. MAX_PATH_LEN)
    // the table's row geometry (RouteTab::plen / row): PATH_LEN / ROUTE_PTS until a written
    // path longer than PATH_LEN is added, then that path's length rounded up to 16
    int plen = mev::PATH_LEN, row_pts = mev::ROUTE_PTS;
    std::vector<float> h_pbox;  // [nroutes][3][4] piece bounding boxes (RouteTab::pbox)
    std::vector<int32_t> h_intent;
    // route_hash[r]: FNV-1a of routes [0, r) (paths and intents), so a snapshot or a gather
    // peer can tell whether its route ids name the same routes here (routes are only appended)
    std::vector<uint64_t> route_hash{1469598103934665603ull};
    void extend_route_hash() {
        while (route_hash.size() <= size_t(nroutes)) {
            const size_t r = route_hash.size() - 1;
            uint64_t x = route_hash.back();
            auto mix = [&x](const void* p, size_t n) {
                const uint8_t* b = static_cast<const uint8_t*>(p);
                for (size_t i = 0; i < n; ++i) x = (x ^ b[i]) * 1099511628211ull;
            };
            // a path as its first max(n, PATH_LEN) row points, its last segment and, up to
            // PATH_LEN, the ROUTE_PTS row's zero tail: the same bytes whatever the row stride
            const float* row = &h_paths[r * 2 * size_t(row_pts)];
            const int n = std::max(h_len[r], mev::PATH_LEN);
            mix(row, 2 * size_t(n) * sizeof(float));
            mix(row + 2 * plen, 4 * sizeof(float));
            if (n == mev::PATH_LEN) {
                const float z[2 * (mev::ROUTE_PTS - mev::ROUTE_END - 2)] = {};
                mix(z, sizeof(z));
            }
            mix(&h_intent[r], sizeof(int32_t));
            route_hash.push_back(x);
        }
    }
    std::vector<int32_t> h_traffic;
    hipStream_t own_stream = nullptr;
    hipStream_t stream = nullptr;
    std::vector<void*> allocs;
    mev::SimParams sp{};
    mev::SimParams* d_sp = nullptr;  // device copy of sp read by k_step (refreshed when sp changes)
    mev::SimParams sp_dev{};         // what d_sp holds
    bool sp_valid = false;
    mev::Outputs internal{};
    mev::Outputs last{};  // where the most recent outputs were written
    float* d_actions = nullptr;
    int32_t* d_spawn = nullptr;
    uint8_t* d_mask = nullptr;
    float* d_paths = nullptr;
    int32_t* d_rlen = nullptr;  // [route_cap] each path's own length (RouteTab::len)
    float* d_pbox = nullptr;
    float* d_spawn_tab = nullptr;
    int32_t* d_intent = nullptr;
    float* d_rel = nullptr;
    int32_t* d_traffic = nullptr;
    int32_t* d_reset_routes = nullptr;  // [nroutes]: pool for per-reset route draws
    uint8_t* d_snap_stage = nullptr;    // device copy of a host snapshot (masked restore)
    size_t snap_stage_bytes = 0;
    uint64_t rng_counter = 0;
    // per-kernel timing (mev_kernel_timing): 3 events per step, folded into sums when the ring fills
    std::vector<hipEvent_t> tev;
    int tn = 0;
    int t_every = 1;       // record events on every t_every-th step
    int64_t t_phase = 0;   // steps since timing was enabled
    double t_cars_ms = 0.0, t_lidar_ms = 0.0;
    int64_t t_steps = 0;
    // multi-GPU gather (mev_comm_init): packed outputs, double buffered by step parity
    ncclComm_t comm = nullptr;
    int world = 1, rank = 0, root = 0, slots = 0;
    uint64_t pk_off[MEV_PK_FIELDS] = {};
    int gather_fmt = MEV_GATHER_F32;  // mev_set_gather_format
    std::vector<float> h_lidar_table;  // [256] decode table of the compact format (mev_lidar_decode_table)
    float* d_lidar_table = nullptr;
    uint64_t pk_bytes = 0;
    uint8_t* pk_buf[2] = {nullptr, nullptr};  // root: [world][pk_bytes]; other ranks: [pk_bytes]
    hipStream_t comm_stream = nullptr;
    hipEvent_t ev_step[2] = {nullptr, nullptr}, ev_gather[2] = {nullptr, nullptr};
    bool gather_pending[2] = {false, false};
    int64_t gathers = 0;  // gathered steps so far; the last one used buffer (gathers - 1) & 1
    // NPC-aware deal of the fused traffic kernel: valid while every step since the
    // last state change went through it (the rings then hold one entry per env)
    bool deal_valid = false;
    // the rings were built by a step with MEV_AUTO_RESET: an env that ended there is in class
    // 0 (no NPC slot loaded), which only the next step's auto-reset makes true
    bool deal_ar = false;
    bool deal_on = true;  // mev_set_env_deal (default: on unless MEV_NO_DEAL=1)
    int deal_ring = 0;

    template <class T>
    hipError_t alloc(T** p, size_t n) {
        hipError_t e = dalloc(p, n);
        if (e == hipSuccess) {
            allocs.push_back(*p);
            e = hipMemsetAsync(*p, 0, (n ? n : 1) * sizeof(T), stream);
        }
        return e;
    }
    hipError_t fold_timing() {
        if (tn == 0) return hipSuccess;
        hipError_t e = hipEventSynchronize(tev[size_t(3 * tn - 1)]);
        if (e != hipSuccess) return e;
        for (int i = 0; i < tn; ++i) {
            float a = 0.f, b = 0.f;
            if ((e = hipEventElapsedTime(&a, tev[size_t(3 * i)], tev[size_t(3 * i + 1)])) != hipSuccess) return e;
            if ((e = hipEventElapsedTime(&b, tev[size_t(3 * i + 1)], tev[size_t(3 * i + 2)])) != hipSuccess) return e;
            t_cars_ms += a;
            t_lidar_ms += b;
        }
        t_steps += tn;
        tn = 0;
        return hipSuccess;
    }
    void free_timing() {
        for (hipEvent_t ev : tev) (void)hipEventDestroy(ev);
        tev.clear();
        tn = 0;
    }
    void free_comm() {
        if (comm) (void)ncclCommDestroy(comm);
        comm = nullptr;
        for (int b = 0; b < 2; ++b) {
            if (pk_buf[b]) (void)hipFree(pk_buf[b]);
            if (ev_step[b]) (void)hipEventDestroy(ev_step[b]);
            if (ev_gather[b]) (void)hipEventDestroy(ev_gather[b]);
            pk_buf[b] = nullptr;
            ev_step[b] = ev_gather[b] = nullptr;
            gather_pending[b] = false;
        }
        if (comm_stream) (void)hipStreamDestroy(comm_stream);
        comm_stream = nullptr;
        world = 1; rank = root = 0; gathers = 0;
    }
    // Host-mode steps of a small handle (outputs <= kPinMax bytes): actions and
    // outputs in one block of host-mapped pinned memory that the kernels read
    // and write directly (zero-copy), so a step is one launch and one stream
    // synchronization instead of nine pageable copies (~150 us at 1 env).
    static constexpr size_t kPinMax = 256 * 1024;
    uint8_t* pin = nullptr;     // host address of the block (hipHostMalloc, mapped, coherent)
    uint8_t* pin_dev = nullptr; // its device address
    size_t pin_off[10] = {};    // actions, spawn, obs, reward, done, status, term, trunc, alive, step
    mev::Outputs pin_out{};     // device addresses of the pinned outputs
    // Persistent step server (k_serve, mev_set_serve): host-mode steps of a small
    // handle posted to a resident kernel through a mailbox in pinned memory
    int serve_mode = 1;                 // 0 off, 1 automatic
    mev::ServeBox* sbox = nullptr;      // host address of the mailbox (mapped, coherent)
    mev::ServeBox* sbox_dev = nullptr;  // its device address
    // (atomic: serve_slot reads other handles' flags, which their own threads write)
    std::atomic<bool> serve_running{false};  // an instance may be resident on `stream`
    int serve_wg = 0;                        // its workgroups
    uint32_t serve_seq = 0, serve_sid = 0;
    std::atomic<uint32_t> serve_epoch{0};
    uint64_t serve_steps = 0, serve_launches = 0;
    // Adaptive idle limit: a resident server makes every device-wide
    // wait of the process (hipDeviceSynchronize, torch.cuda.synchronize, some frees)
    // wait for its idle exit, so it stays only a few host gaps long: 8 x the moving
    // average of the host's time between an answer and the next post (each gap
    // counted up to 2 ms), within [0.2, 2] ms; it starts at the cap and follows the
    // host's pace.  Posts that keep finding the server gone (a device-wide wait, or
    // a host slower than 2 ms between steps) pause serving: the next kPausedSteps
    // host steps are launched.
    double serve_gap_us = 250.0;
    int serve_misses = 0;
    uint64_t serve_pause = 0;
    uint64_t serve_misses_total = 0;
    std::chrono::steady_clock::time_point serve_t_answer{};
    // steady-clock ns of the handle's last host-mode step (serve_slot: a slot's owner
    // that has made no host step for kServeStaleMs may lose it to another handle)
    std::atomic<int64_t> serve_last_ns{0};
    // the server's own stream: non-blocking, at the highest priority, whose hardware
    // queues are not the ones normal-priority streams share (GPU_MAX_HW_QUEUES of them):
    // a resident kernel holds back whatever another stream queues behind it on its queue
    hipStream_t serve_stream = nullptr;
    hipEvent_t serve_ev = nullptr;  // orders the server after the handle's stream
    uint8_t* gs_pin = nullptr;  // pinned staging of mev_get_state
    size_t gs_cap = 0;
    ~mev_handle() {
        if (comm_stream) (void)hipStreamSynchronize(comm_stream);
        free_comm();
        free_timing();
        if (pin) (void)hipHostFree(pin);
        if (sbox) (void)hipHostFree(sbox);
        if (serve_ev) (void)hipEventDestroy(serve_ev);
        if (serve_stream) (void)hipStreamDestroy(serve_stream);
        if (gs_pin) (void)hipHostFree(gs_pin);
        if (d_snap_stage) (void)hipFree(d_snap_stage);
        for (void* p : allocs) (void)hipFree(p);
        if (own_stream) (void)hipStreamDestroy(own_stream);
    }
};

extern "C" {

static int serve_stop(mev_handle* h);  // with mev_step: the resident step server leaves the stream
namespace {
void serve_unlist(mev_handle* h);  // (with mev_step) the handle leaves the resident-server list

// SimParams::beam_cull: the LiDAR's per-box beam culling models the offsets as
// rel[b] = rel[0] + b*d (to 1e-5 rad, the slack its 2e-4 rad margin covers) with d > 0 and
// the fan within one revolution, (R-1)*d <= 2*pi.  Any other list (a written
// Lidar.rel_angles, cpp/bindings.cpp:91: descending, constant, uneven, several turns) is
// simulated without the culling.
int beam_cull_ok(const float* rel, int R) {
    if (R <= 1) return 1;
    const double d = (double(rel[R - 1]) - double(rel[0])) / double(R - 1);
    if (!(d > 0.0) || double(R - 1) * d > 6.283185307179586 + 1.0e-4) return 0;
    for (int b = 1; b < R - 1; ++b)
        if (fabs(double(rel[b]) - (double(rel[0]) + b * d)) > 1.0e-5) return 0;
    return 1;
}
}  // namespace

const char* mev_last_error(void) { return g_err.c_str(); }
int mev_abi_version(void) { return MEV_ABI_VERSION; }
int mev_path_len(void) { return mev::PATH_LEN; }

int mev_device_count(int32_t* count) {
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess) n = 0;
    if (count) *count = n;
    return MEV_OK;
}

int mev_config_default(mev_config* c) {
    if (!c) return fail(MEV_E_INVALID, "null config");
    memset(c, 0, sizeof(*c));
    c->num_envs = 1;
    c->num_agents = 1;
    c->num_lanes = 3;
    c->lidar_rays = 96;  // cpp/IntersectionEnv.cpp:113-116
    c->lidar_fov_deg = 360.0f;
    c->lidar_max_dist = 250.0f;
    c->lidar_step = 4.0f;
    c->obs_dim = 0;
    c->traffic_flow = 0;
    c->traffic_density = 0.5f;  // cpp/IntersectionEnv.h:35
    c->use_team_reward = 0;
    c->respawn_enabled = 1;
    c->max_steps = 2000;
    const float rc[8] = {10.0f, 1.0f, -0.01f, -10.0f, -5.0f, 10.0f, -0.02f, 0.2f};  // cpp/Reward.h:5-14
    memcpy(c->reward, rc, sizeof(rc));
    c->max_npcs = 32;
    c->seed = 0;
    c->device = 0;
    return MEV_OK;
}

int mev_create(const mev_config* cfg, mev_handle** out) {
    if (!cfg || !out) return fail(MEV_E_INVALID, "null argument");
    const mev_config& c = *cfg;
    if (c.num_envs < 1) return fail(MEV_E_INVALID, "num_envs must be >= 1");
    if (c.num_agents < 1 || c.num_agents > 64) return fail(MEV_E_INVALID, "num_agents must be in [1, 64]");
    if (c.num_lanes < 1 || c.num_lanes > 8) return fail(MEV_E_INVALID, "num_lanes must be in [1, 8]");
    if (c.lidar_rays < 1 || c.lidar_rays > 1024) return fail(MEV_E_INVALID, "lidar_rays must be in [1, 1024]");
    if (!(c.lidar_step > 0.0f) || !(c.lidar_max_dist > 0.0f)) return fail(MEV_E_INVALID, "lidar step/max_dist must be > 0");
    if (c.max_npcs < 0 || c.max_npcs > 64) return fail(MEV_E_INVALID, "max_npcs must be in [0, 64]");
    const int D = c.obs_dim > 0 ? c.obs_dim : mev::OBS_HEAD + c.lidar_rays;
    if (D < mev::OBS_HEAD) return fail(MEV_E_INVALID, "obs_dim must be >= 31");
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return fail(MEV_E_HIP, "no HIP device available");
    if (c.device < 0 || c.device >= ndev) return fail(MEV_E_INVALID, "device ordinal out of range");
    HIP_TRY(hipSetDevice(c.device));
    // LiDAR probe distances exactly as Lidar.cpp:33 accumulates them (validated
    // before any allocation: this error path owns nothing)
    std::vector<float> dists;
    bool dist_mul_exact = true;
    for (float dist = 0.0f; dist < c.lidar_max_dist; dist += c.lidar_step) {
        if (dist != float(dists.size()) * c.lidar_step) dist_mul_exact = false;
        dists.push_back(dist);
        if (dists.size() > (1u << 20)) return fail(MEV_E_INVALID, "lidar_max_dist / lidar_step too large");
    }

    auto* h = new mev_handle();
    h->cfg = c;
    {
        const char* nd = getenv("MEV_NO_DEAL");
        h->deal_on = !(nd && nd[0] == '1');
    }
    if (h->cfg.traffic_density < 0.0f) h->cfg.traffic_density = 0.0f;  // configure_traffic (:56-60)
    h->D = D;
    h->lidar_slots = std::min(c.lidar_rays, D - mev::OBS_HEAD);
    {  // the compact gather format's LiDAR codes -> floats (Lidar::normalized, Lidar.cpp:92-98)
        const float inv = (c.lidar_max_dist > 0.0f) ? (1.0f / c.lidar_max_dist) : 0.0f;
        h->h_lidar_table.assign(256, 0.0f);
        h->h_lidar_table[0] = c.lidar_max_dist * inv;  // no hit: max_dist
        for (size_t k = 0; k < dists.size() && k + 1 < size_t(mev::kLidarCodeDead); ++k)
            h->h_lidar_table[k + 1] = dists[k] * inv;  // hit at probe k
        h->h_lidar_table[mev::kLidarCodeDead] = 0.0f;  // dead agent
    }
    h->P = 8 * c.num_lanes;
    h->nroutes = h->P * h->P;
    h->route_cap = h->nroutes;
    h->pts = mev::build_lane_points(c.num_lanes);
    h->h_paths.resize(size_t(h->nroutes) * 2 * mev::ROUTE_PTS);
    h->h_len.assign(size_t(h->nroutes), mev::PATH_LEN);
    h->h_intent.resize(size_t(h->nroutes));
    h->h_spawn.resize(size_t(h->nroutes) * 3);
    for (int s = 0; s < h->P; ++s)
        for (int e = 0; e < h->P; ++e) {
            const int r = s * h->P + e;
            float* path = &h->h_paths[size_t(r) * 2 * mev::ROUTE_PTS];
            h->h_intent[size_t(r)] = mev::generate_route(h->pts, c.num_lanes, s, e, path);
            std::copy(path + 2 * (mev::PATH_LEN - 2), path + 2 * mev::PATH_LEN, path + 2 * mev::ROUTE_END);
            h->h_spawn[size_t(3 * r)] = h->pts[size_t(s)].x;
            h->h_spawn[size_t(3 * r + 1)] = h->pts[size_t(s)].y;
            h->h_spawn[size_t(3 * r + 2)] = mev::spawn_heading(path);
        }
    // each route's pieces [0, 50), [50, 110), [110, 160): bounding boxes of the float points
    h->h_pbox.resize(size_t(h->nroutes) * 12);
    for (int r = 0; r < h->nroutes; ++r) {
        const float* path = &h->h_paths[size_t(r) * 2 * mev::ROUTE_PTS];
        const int cut[4] = {0, 50, 110, mev::PATH_LEN};
        for (int q = 0; q < 3; ++q) {
            float x0 = path[2 * cut[q]], x1 = x0, y0 = path[2 * cut[q] + 1], y1 = y0;
            for (int i = cut[q]; i < cut[q + 1]; ++i) {
                x0 = std::min(x0, path[2 * i]); x1 = std::max(x1, path[2 * i]);
                y0 = std::min(y0, path[2 * i + 1]); y1 = std::max(y1, path[2 * i + 1]);
            }
            float* b = &h->h_pbox[size_t(r) * 12 + size_t(q) * 4];
            b[0] = x0; b[1] = x1; b[2] = y0; b[3] = y1;
        }
    }
    // LiDAR beam offsets, cpp/IntersectionEnv.cpp:119-127 (== Lidar.cpp:4-14)
    std::vector<float> rel(size_t(c.lidar_rays));
    {
        const float start_angle_deg = -c.lidar_fov_deg * 0.5f;
        const float step_deg = (c.lidar_rays > 1) ? (c.lidar_fov_deg / float(c.lidar_rays - 1)) : 0.0f;
        const float PI_F2 = 3.14159265358979323846f;
        for (int ii = 0; ii < c.lidar_rays; ++ii) {
            const float deg = start_angle_deg + float(ii) * step_deg;
            rel[size_t(ii)] = deg * PI_F2 / 180.0f;
        }
    }
    h->sp.beam_cull = beam_cull_ok(rel.data(), c.lidar_rays);
    h->h_traffic = mev::default_traffic_routes(c.num_lanes);
    h->extend_route_hash();

    if (hipStreamCreateWithFlags(&h->own_stream, hipStreamNonBlocking) != hipSuccess) {
        delete h;
        return fail(MEV_E_HIP, "hipStreamCreate failed");
    }
    h->stream = h->own_stream;
    const int E = c.num_envs, N = c.num_agents, K = std::max(1, c.max_npcs);
    const size_t EN = size_t(E) * size_t(N), EK = size_t(E) * size_t(K);
    mev::SimParams& p = h->sp;
    hipError_t err = hipSuccess;
    auto A = [&](auto** ptr, size_t n) { if (err == hipSuccess) err = h->alloc(ptr, n); };
    // state
    // the 4-byte fields of each SoA in one block, field k at k * stride (mev_kernels.h)
    const size_t ens = (EN + 63) & ~size_t(63), eks = (EK + 63) & ~size_t(63);
    float* eblk = nullptr;
    float* nblk = nullptr;
    A(&eblk, ens * mev::EF_COUNT);
    A(&nblk, eks * mev::NF_COUNT);
    if (err == hipSuccess) {
        float** ef[] = {&p.ego.x, &p.ego.y, &p.ego.v, &p.ego.h, &p.ego.acc, &p.ego.steer, &p.ego.prev_dist,
                        &p.ego.pa0, &p.ego.pa1, &p.ego.sx, &p.ego.sy, &p.ego.sv, &p.ego.sh};
        for (int k = 0; k < mev::EF_PIDX; ++k) *ef[k] = eblk + size_t(k) * ens;
        p.ego.pidx = reinterpret_cast<int32_t*>(eblk + size_t(mev::EF_PIDX) * ens);
        p.ego.route = reinterpret_cast<int32_t*>(eblk + size_t(mev::EF_ROUTE) * ens);
        p.ego.intent = reinterpret_cast<int32_t*>(eblk + size_t(mev::EF_INTENT) * ens);
        p.ego.stride = int64_t(ens);
        float** nf[] = {&p.npc.x, &p.npc.y, &p.npc.v, &p.npc.h, &p.npc.acc, &p.npc.steer};
        for (int k = 0; k < mev::NF_PIDX; ++k) *nf[k] = nblk + size_t(k) * eks;
        p.npc.pidx = reinterpret_cast<int32_t*>(nblk + size_t(mev::NF_PIDX) * eks);
        p.npc.route = reinterpret_cast<int32_t*>(nblk + size_t(mev::NF_ROUTE) * eks);
        p.npc.intent = reinterpret_cast<int32_t*>(nblk + size_t(mev::NF_INTENT) * eks);
        p.npc.stride = int64_t(eks);
    }
    A(&p.ego.alive, EN);
    A(&p.npc.alive, EK); A(&p.npc.count, size_t(E));
    A(&p.ego_dim, EN * 2); A(&p.npc_dim, EK * 2);  // car sizes (mev_set_car_dims), 54 x 24 until set
    A(&p.step_count, size_t(E)); A(&p.pending_reset, size_t(E)); A(&p.overflow, 3); A(&p.debug, size_t(E) * 8);
    A(&p.ob_box, size_t(E) * size_t(N + c.max_npcs)); A(&p.ob_cand, EN * 2);
    if (c.traffic_flow) {  // the fused traffic kernel's NPC-aware deal (mev_kernels.h, kDealLists)
        A(&p.deal_cnt, size_t(3) * mev::kDealRingInts);
        A(&p.deal_order, size_t(3) * mev::kDealLists * mev::kDealClasses * size_t(E));
    }
    // outputs
    A(&h->internal.obs, EN * size_t(D)); A(&h->internal.rew, EN); A(&h->internal.done, EN); A(&h->internal.status, EN);
    A(&h->internal.term, size_t(E)); A(&h->internal.trunc, size_t(E)); A(&h->internal.alive_cnt, size_t(E));
    A(&h->internal.step, size_t(E));
    // inputs & tables
    A(&h->d_actions, EN * 2); A(&h->d_spawn, size_t(E)); A(&h->d_mask, size_t(E));
    A(&h->d_paths, h->h_paths.size()); A(&h->d_rlen, h->h_len.size()); A(&h->d_pbox, h->h_pbox.size()); A(&h->d_spawn_tab, h->h_spawn.size()); A(&h->d_intent, h->h_intent.size());
    A(&h->d_rel, rel.size()); A(&h->d_traffic, size_t(h->P) * size_t(h->P));
    A(&h->d_reset_routes, size_t(h->P) * size_t(h->P));
    A(&h->d_lidar_table, size_t(256));
    A(reinterpret_cast<uint8_t**>(&h->d_sp), sizeof(mev::SimParams));
    float* d_dist = nullptr;
    if (!dist_mul_exact) A(&d_dist, dists.size());
    if (err != hipSuccess) {
        std::string m = hipGetErrorString(err);
        delete h;
        return fail(MEV_E_NOMEM, "device allocation failed: " + m);
    }
    h->internal.obs_ld = D;
    h->last = h->internal;
    // upload tables
    err = hipMemcpyAsync(h->d_paths, h->h_paths.data(), h->h_paths.size() * sizeof(float), hipMemcpyHostToDevice, h->stream);
    if (err == hipSuccess) err = hipMemcpyAsync(h->d_spawn_tab, h->h_spawn.data(), h->h_spawn.size() * sizeof(float), hipMemcpyHostToDevice, h->stream);
    if (err == hipSuccess) err = hipMemcpyAsync(h->d_pbox, h->h_pbox.data(), h->h_pbox.size() * sizeof(float), hipMemcpyHostToDevice, h->stream);
    if (err == hipSuccess) err = hipMemcpyAsync(h->d_intent, h->h_intent.data(), h->h_intent.size() * sizeof(int32_t), hipMemcpyHostToDevice, h->stream);
    if (err == hipSuccess) err = hipMemcpyAsync(h->d_rlen, h->h_len.data(), h->h_len.size() * sizeof(int32_t), hipMemcpyHostToDevice, h->stream);
    if (err == hipSuccess) err = hipMemcpyAsync(h->d_rel, rel.data(), rel.size() * sizeof(float), hipMemcpyHostToDevice, h->stream);
    if (err == hipSuccess && d_dist) err = hipMemcpyAsync(d_dist, dists.data(), dists.size() * sizeof(float), hipMemcpyHostToDevice, h->stream);
    if (err == hipSuccess)
        err = hipMemcpyAsync(h->d_lidar_table, h->h_lidar_table.data(), 256 * sizeof(float), hipMemcpyHostToDevice, h->stream);
    if (err == hipSuccess) err = hipMemcpyAsync(h->d_traffic, h->h_traffic.data(), h->h_traffic.size() * sizeof(int32_t), hipMemcpyHostToDevice, h->stream);
    // every car of the reference's default size (Car.h:19-20); p.dims stays 0 while they all are
    std::vector<float> dflt(2 * std::max(EN, EK));
    for (size_t i = 0; i < dflt.size(); i += 2) { dflt[i] = mev::CAR_LENGTH; dflt[i + 1] = mev::CAR_WIDTH; }
    if (err == hipSuccess) err = hipMemcpyAsync(p.ego_dim, dflt.data(), EN * 2 * sizeof(float), hipMemcpyHostToDevice, h->stream);
    if (err == hipSuccess) err = hipMemcpyAsync(p.npc_dim, dflt.data(), EK * 2 * sizeof(float), hipMemcpyHostToDevice, h->stream);
    // default ego routes: reference env.py:138-145 (mapping routes, cyclic)
    std::vector<int32_t> ego(EN);
    {
        const int L = c.num_lanes;
        const int (*map)[2] = (L == 2) ? kMap2 : kMap3;
        const int M = (L == 2) ? 7 : 12;
        std::vector<int32_t> valid;
        for (int k = 0; k < M; ++k) {
            const int s = map[k][0] - 1, e = 4 * L + map[k][1] - 1;
            if (map[k][0] <= 4 * L && map[k][1] <= 4 * L) valid.push_back(s * h->P + e);
        }
        if (valid.empty()) valid = h->h_traffic;
        for (size_t i = 0; i < EN; ++i) ego[i] = valid[(i % size_t(N)) % valid.size()];
    }
    if (err == hipSuccess) err = hipMemcpyAsync(p.ego.route, ego.data(), ego.size() * sizeof(int32_t), hipMemcpyHostToDevice, h->stream);
    if (err == hipSuccess) err = hipStreamSynchronize(h->stream);
    if (err != hipSuccess) {
        std::string m = hipGetErrorString(err);
        delete h;
        return fail(MEV_E_HIP, "table upload failed: " + m);
    }
    // parameters
    p.E = E; p.N = N; p.R = c.lidar_rays; p.K = c.max_npcs; p.D = D;
    p.lidar_slots = h->lidar_slots;
    p.num_lanes = c.num_lanes;
    p.irw = int(c.num_lanes * int(mev::LANE_WIDTH_PX));
    p.line_stop = int(c.num_lanes * int(mev::LANE_WIDTH_PX)) + int(mev::CORNER_RADIUS);  // LineMask.cpp:52-54
    p.rw = c.num_lanes * mev::LANE_WIDTH_PX;  // RoadGeometry.h:16
    p.use_team = c.use_team_reward;
    p.respawn = c.respawn_enabled;
    p.traffic = c.traffic_flow;
    p.max_steps = c.max_steps;
    p.k_prog = c.reward[0]; p.v_min = c.reward[1]; p.k_stuck = c.reward[2]; p.k_cv = c.reward[3];
    p.k_co = c.reward[4]; p.k_succ = c.reward[5]; p.k_sm = c.reward[6]; p.alpha = c.reward[7];
    p.max_progress = mev::hypotf(float(mev::WIDTH), float(mev::HEIGHT));  // IntersectionEnv.cpp:22
    p.lidar_max = c.lidar_max_dist;
    p.lidar_step = c.lidar_step;
    p.lidar_inv = (c.lidar_max_dist > 0.0f) ? (1.0f / c.lidar_max_dist) : 0.0f;  // Lidar.cpp:94
    p.lidar_steps = int(dists.size());
    p.ob_stride = N + c.max_npcs;
    p.dist_tab = d_dist;
    p.seed = c.seed;
    p.rt.path = h->d_paths;
    p.rt.intent = h->d_intent;
    p.rt.spawn = h->d_spawn_tab;
    p.rt.pbox = reinterpret_cast<const float4*>(h->d_pbox);
    p.rt.nroutes = h->nroutes;
    p.rt.len = h->d_rlen;
    p.rt.plen = mev::PATH_LEN;
    p.rt.row = mev::ROUTE_PTS;
    p.rt.min_len = mev::PATH_LEN;
    p.rel_angles = h->d_rel;
    p.traffic_routes = h->d_traffic;
    p.n_traffic_routes = int(h->h_traffic.size());
    p.reset_routes = h->d_reset_routes;
    p.n_reset_routes = 0;
    // initial state = a reset (the reference env.py constructor ends with reset(), env.py:136)
    const int rc = mev_reset(h, nullptr, nullptr, 0);
    if (rc != MEV_OK) {
        const std::string m = g_err;
        delete h;
        *out = nullptr;
        return fail(rc, m);
    }
    *out = h;
    return MEV_OK;
}

int mev_destroy(mev_handle* h) {
    if (!h) return MEV_OK;
    (void)hipSetDevice(h->cfg.device);
    (void)serve_stop(h);
    serve_unlist(h);
    (void)hipStreamSynchronize(h->stream);
    delete h;
    return MEV_OK;
}

int mev_get_config(const mev_handle* h, mev_config* cfg) {
    if (!h || !cfg) return fail(MEV_E_INVALID, "null argument");
    *cfg = h->cfg;
    cfg->obs_dim = h->D;
    return MEV_OK;
}

int mev_obs_dim(const mev_handle* h, int32_t* d) {
    if (!h || !d) return fail(MEV_E_INVALID, "null argument");
    *d = h->D;
    return MEV_OK;
}

int mev_set_stream(mev_handle* h, void* stream) {
    if (!h) return fail(MEV_E_INVALID, "null handle");
    HIP_TRY(hipSetDevice(h->cfg.device));
    if (int r_ = serve_stop(h)) return r_;  // (the server holds the stream)
    HIP_TRY(hipStreamSynchronize(h->stream));  // order the switch after outstanding work
    h->stream = static_cast<hipStream_t>(stream);  // NULL = the legacy default stream
    if (h->stream != h->own_stream) serve_unlist(h);  // (no server on a caller's stream: its slot goes)
    return MEV_OK;
}

int mev_use_own_stream(mev_handle* h) {
    if (!h) return fail(MEV_E_INVALID, "null handle");
    HIP_TRY(hipSetDevice(h->cfg.device));
    if (int r_ = serve_stop(h)) return r_;  // (the server holds the stream)
    HIP_TRY(hipStreamSynchronize(h->stream));
    h->stream = h->own_stream;
    return MEV_OK;
}

int mev_debug_stamps(mev_handle* h, uint64_t* out) {
    if (!h || !out) return fail(MEV_E_INVALID, "null argument");
    HIP_TRY(hipSetDevice(h->cfg.device));
    if (int r_ = serve_stop(h)) return r_;  // (the server holds the stream)
    HIP_TRY(hipMemcpyAsync(out, h->sp.debug, size_t(h->cfg.num_envs) * 8 * sizeof(uint64_t), hipMemcpyDeviceToHost, h->stream));
    HIP_TRY(hipStreamSynchronize(h->stream));
    return MEV_OK;
}

int mev_sync(mev_handle* h) {
    if (!h) return fail(MEV_E_INVALID, "null handle");
    HIP_TRY(hipSetDevice(h->cfg.device));
    if (int r_ = serve_stop(h)) return r_;  // (the server holds the stream)
    HIP_TRY(hipStreamSynchronize(h->stream));
    return MEV_OK;
}

int mev_configure(mev_handle* h, int32_t use_team, int32_t respawn, int32_t max_steps) {
    if (!h) return fail(MEV_E_INVALID, "null handle");
    h->cfg.use_team_reward = use_team;
    h->cfg.respawn_enabled = respawn;
    h->cfg.max_steps = max_steps;
    h->sp.use_team = use_team;
    h->sp.respawn = respawn;
    h->sp.max_steps = max_steps;
    return MEV_OK;
}

int mev_configure_traffic(mev_handle* h, int32_t enabled, float density) {
    if (!h) return fail(MEV_E_INVALID, "null handle");
    if (enabled && h->cfg.max_npcs == 0) return fail(MEV_E_INVALID, "traffic needs max_npcs > 0 (set at creation)");
    if (enabled && h->sp.step_kernel == 2) {
        mev::SimParams q = h->sp;
        q.traffic = 1;
        if (mev::step_kernel_for(q) == 0)
            return fail(MEV_E_INVALID, "the fused step kernel (mev_set_step_kernel 2) cannot hold this handle's NPC slots");
    }
    h->cfg.traffic_flow = enabled;
    h->deal_valid = false;
    h->cfg.traffic_density = density < 0.0f ? 0.0f : density;  // configure_traffic clamps (:56-60)
    h->sp.traffic = enabled;
    return MEV_OK;
}

int mev_set_reward(mev_handle* h, const float* rc) {
    if (!h || !rc) return fail(MEV_E_INVALID, "null argument");
    memcpy(h->cfg.reward, rc, sizeof(h->cfg.reward));
    mev::SimParams& p = h->sp;
    p.k_prog = rc[0]; p.v_min = rc[1]; p.k_stuck = rc[2]; p.k_cv = rc[3];
    p.k_co = rc[4]; p.k_succ = rc[5]; p.k_sm = rc[6]; p.alpha = rc[7];
    return MEV_OK;
}

int mev_car_update(float* kin, float throttle, float steer_input, float dt) {
    if (!kin) return fail(MEV_E_INVALID, "null argument");
    mev::Kin k{kin[0], kin[1], kin[2], kin[3], kin[4], kin[5]};
    float c, s;
    mev::car_update(k, throttle, steer_input, dt, &c, &s);
    kin[0] = k.x; kin[1] = k.y; kin[2] = k.v; kin[3] = k.h; kin[4] = k.acc; kin[5] = k.steer;
    return MEV_OK;
}

static void box_corners(const float* b, float* cx, float* cy, float* c, float* s) {
    // Car::corners (cpp/Car.cpp:86-103) with the car's own length/width
    mev::sincosf(b[2], s, c);
    const float hx = b[4] * 0.5f, hy = b[3] * 0.5f;
    const float lx[4] = {hy, hy, -hy, -hy}, ly[4] = {hx, -hx, -hx, hx};
    for (int k = 0; k < 4; ++k) {
        cx[k] = b[0] + lx[k] * *c - ly[k] * *s;
        cy[k] = b[1] + lx[k] * *s + ly[k] * *c;
    }
}

int mev_car_check_collision(const float* a, const float* b, int32_t* collide) {
    if (!a || !b || !collide) return fail(MEV_E_INVALID, "null argument");
    float ax[4], ay[4], bx[4], by[4], ca, sa, cb, sb;
    box_corners(a, ax, ay, &ca, &sa);
    box_corners(b, bx, by, &cb, &sb);
    *collide = mev::sat_collide(ax, ay, ca, sa, bx, by, cb, sb) ? 1 : 0;
    return MEV_OK;
}

int mev_num_points(const mev_handle* h, int32_t* n) {
    if (!h || !n) return fail(MEV_E_INVALID, "null argument");
    *n = h->P;
    return MEV_OK;
}

int mev_point_xy(const mev_handle* h, int32_t point, float* xy) {
    if (!h || !xy) return fail(MEV_E_INVALID, "null argument");
    if (point < 0 || point >= h->P) return fail(MEV_E_RANGE, "lane point out of range");
    xy[0] = h->pts[size_t(point)].x;
    xy[1] = h->pts[size_t(point)].y;
    return MEV_OK;
}

int mev_route_id(const mev_handle* h, int32_t s, int32_t e, int32_t* route) {
    if (!h || !route) return fail(MEV_E_INVALID, "null argument");
    if (s < 0 || s >= h->P || e < 0 || e >= h->P) return fail(MEV_E_RANGE, "lane point out of range");
    *route = s * h->P + e;
    return MEV_OK;
}

int mev_route_len(const mev_handle* h, int32_t route, int32_t* npoints) {
    if (!h || !npoints) return fail(MEV_E_INVALID, "null argument");
    if (route < 0 || route >= h->nroutes) return fail(MEV_E_RANGE, "route out of range");
    *npoints = h->h_len[size_t(route)];
    return MEV_OK;
}

int mev_route_info(const mev_handle* h, int32_t route, float* path, int32_t* intent, float* spawn) {
    if (!h) return fail(MEV_E_INVALID, "null handle");
    if (route < 0 || route >= h->nroutes) return fail(MEV_E_RANGE, "route out of range");
    if (path) {  // max(n, PATH_LEN) points: a shorter path padded with its last point
        const int n = std::max(h->h_len[size_t(route)], mev::PATH_LEN);
        memcpy(path, &h->h_paths[size_t(route) * 2 * size_t(h->row_pts)], sizeof(float) * 2 * size_t(n));
    }
    if (intent) *intent = h->h_intent[size_t(route)];
    if (spawn) memcpy(spawn, &h->h_spawn[size_t(3 * route)], sizeof(float) * 3);
    return MEV_OK;
}

int mev_add_route(mev_handle* h, const float* path, int32_t intent, int32_t* route) {
    return mev_add_route_n(h, path, mev::PATH_LEN, intent, route);
}

namespace {
// a route-table row of `plen` points: the n points, padded with the last one, then the
// last segment at plen, plen + 1 and zeros up to plen + 16 (mev_world.h)
void fill_row(float* row, const float* pts, int n, int plen) {
    for (int i = 0; i < plen; ++i) {
        const int q = i < n ? i : n - 1;
        row[2 * i] = pts[2 * q];
        row[2 * i + 1] = pts[2 * q + 1];
    }
    std::copy(pts + 2 * (n - 2), pts + 2 * n, row + 2 * plen);
    std::fill(row + 2 * (plen + 2), row + 2 * (plen + 16), 0.0f);
}
}  // namespace

int mev_add_route_n(mev_handle* h, const float* path_in, int32_t npoints, int32_t intent, int32_t* route) {
    if (!h || !path_in || !route) return fail(MEV_E_INVALID, "null argument");
    if (intent < 0 || intent > 2) return fail(MEV_E_INVALID, "intent must be 0 (straight), 1 (left) or 2 (right)");
    if (npoints < 2 || npoints > mev::MAX_PATH_LEN) return fail(MEV_E_INVALID, "a route path has 2 .. 4096 points");
    for (int i = 0; i < 2 * npoints; ++i)
        if (!(fabsf(path_in[i]) < 1.0e6f)) return fail(MEV_E_INVALID, "path points must be finite (|coordinate| < 1e6)");
    if (h->nroutes >= 32767) return fail(MEV_E_INVALID, "too many routes (the state gather format ships i16 ids)");
    if (h->comm && h->gather_fmt == MEV_GATHER_STATE)  // every rank's route ids are decoded with the root's table
        return fail(MEV_E_INVALID, "routes cannot be added while a state-format gather communicator exists");
    HIP_TRY(hipSetDevice(h->cfg.device));
    if (int r_ = serve_stop(h)) return r_;  // (the server holds the stream)
    HIP_TRY(hipStreamSynchronize(h->stream));
    const int r = h->nroutes;
    // a path longer than the rows re-lays the whole table out at the new length (rounded up to
    // 16 points, rows stay 128-B aligned); every row keeps its own n and its padding.  The
    // boxes of the other rows stay: their new padding is their last point, which their third
    // piece [110, old plen) already holds
    const int plen = npoints > h->plen ? (npoints + 15) & ~15 : h->plen;
    const int row_pts = plen + 16;
    const bool relayout = plen != h->plen;
    std::vector<float> old_paths;
    if (relayout) {
        old_paths.swap(h->h_paths);
        h->h_paths.resize(size_t(r) * 2 * size_t(row_pts));
        for (int q = 0; q < r; ++q)
            fill_row(&h->h_paths[size_t(q) * 2 * row_pts], &old_paths[size_t(q) * 2 * h->row_pts], h->h_len[size_t(q)],
                     plen);
    }
    h->h_paths.resize(size_t(r + 1) * 2 * size_t(row_pts));
    float* row = &h->h_paths[size_t(r) * 2 * row_pts];
    fill_row(row, path_in, npoints, plen);
    {  // the pieces [0, 50), [50, 110), [110, plen) of the padded row
        const int cut[4] = {0, 50, 110, plen};
        for (int q = 0; q < 3; ++q) {
            float x0 = row[2 * cut[q]], x1 = x0, y0 = row[2 * cut[q] + 1], y1 = y0;
            for (int i = cut[q]; i < cut[q + 1]; ++i) {
                x0 = std::min(x0, row[2 * i]); x1 = std::max(x1, row[2 * i]);
                y0 = std::min(y0, row[2 * i + 1]); y1 = std::max(y1, row[2 * i + 1]);
            }
            h->h_pbox.push_back(x0); h->h_pbox.push_back(x1); h->h_pbox.push_back(y0); h->h_pbox.push_back(y1);
        }
    }
    h->h_len.push_back(npoints);
    h->h_intent.push_back(intent);
    h->h_spawn.push_back(row[0]);  // add_car_with_route's spawn: the path's first point (RouteGen.cpp:111-205)
    h->h_spawn.push_back(row[1]);
    h->h_spawn.push_back(mev::spawn_heading(row));
    auto rollback = [&]() {
        if (relayout) h->h_paths.swap(old_paths);
        else h->h_paths.resize(size_t(r) * 2 * size_t(row_pts));
        h->h_len.pop_back();
        h->h_intent.pop_back();
        h->h_spawn.resize(h->h_spawn.size() - 3);
        h->h_pbox.resize(h->h_pbox.size() - 12);
    };
    // the five route tables: the new route's rows go into spare capacity; a full table (or a
    // re-laid-out one) is reallocated at twice the routes (so n added routes cost O(log n)
    // reallocations, each a hipFree that waits for the device) and uploaded whole
    const size_t per[5] = {2 * size_t(row_pts) * sizeof(float), sizeof(int32_t), 3 * sizeof(float), 12 * sizeof(float),
                           sizeof(int32_t)};
    const void* src[5] = {h->h_paths.data(), h->h_intent.data(), h->h_spawn.data(), h->h_pbox.data(), h->h_len.data()};
    const int cap = r >= h->route_cap ? std::min(32767, std::max(2 * h->route_cap, r + 1)) : h->route_cap;
    hipError_t e = hipSuccess;
    if (cap == h->route_cap && !relayout) {
        void* cur[5] = {h->d_paths, h->d_intent, h->d_spawn_tab, h->d_pbox, h->d_rlen};
        for (int k = 0; k < 5 && e == hipSuccess; ++k)
            e = hipMemcpy(static_cast<uint8_t*>(cur[k]) + size_t(r) * per[k],
                          static_cast<const uint8_t*>(src[k]) + size_t(r) * per[k], per[k], hipMemcpyHostToDevice);
        if (e != hipSuccess) {
            rollback();
            return fail(MEV_E_HIP, std::string("route table: ") + hipGetErrorString(e));
        }
    } else {
        void* np[5] = {nullptr, nullptr, nullptr, nullptr, nullptr};
        for (int k = 0; k < 5 && e == hipSuccess; ++k) {
            e = hipMalloc(&np[k], size_t(cap) * per[k]);
            if (e == hipSuccess) e = hipMemcpy(np[k], src[k], size_t(r + 1) * per[k], hipMemcpyHostToDevice);
        }
        if (e != hipSuccess) {
            for (void* q : np) if (q) (void)hipFree(q);
            rollback();
            return fail(MEV_E_NOMEM, std::string("route table: ") + hipGetErrorString(e));
        }
        void* old[5] = {h->d_paths, h->d_intent, h->d_spawn_tab, h->d_pbox, h->d_rlen};
        for (int k = 0; k < 5; ++k) {
            for (auto& a : h->allocs)
                if (a == old[k]) { (void)hipFree(a); a = np[k]; break; }
        }
        h->d_paths = static_cast<float*>(np[0]);
        h->d_intent = static_cast<int32_t*>(np[1]);
        h->d_spawn_tab = static_cast<float*>(np[2]);
        h->d_pbox = static_cast<float*>(np[3]);
        h->d_rlen = static_cast<int32_t*>(np[4]);
        h->route_cap = cap;
    }
    h->plen = plen;
    h->row_pts = row_pts;
    h->nroutes = r + 1;
    h->extend_route_hash();
    h->sp.rt.path = h->d_paths;
    h->sp.rt.intent = h->d_intent;
    h->sp.rt.spawn = h->d_spawn_tab;
    h->sp.rt.pbox = reinterpret_cast<const float4*>(h->d_pbox);
    h->sp.rt.len = h->d_rlen;
    h->sp.rt.nroutes = h->nroutes;  // (the next launch refreshes the device copy of the parameters)
    h->sp.rt.plen = plen;
    h->sp.rt.row = row_pts;
    h->sp.rt.min_len = std::min(h->sp.rt.min_len, int32_t(npoints));
    *route = r;
    return MEV_OK;
}

// ---- per-car sizes (reference Car::length / Car::width, cpp/Car.h:19-20, read-write
// through cpp/bindings.cpp:24-25): the SAT corners, the status corners and the LiDAR
// boxes of each car.  The device arrays always hold every car's size (54 x 24 until
// set); SimParams::dims says whether any differs, and only then do the steps run the
// runtime-layout kernels that read them (mev_kernels.hip, DIMS).
static bool all_default_dims(const float* d, size_t n) {
    for (size_t i = 0; i < n; ++i)
        if (d[2 * i] != mev::CAR_LENGTH || d[2 * i + 1] != mev::CAR_WIDTH) return false;
    return true;
}

int mev_set_car_dims(mev_handle* h, const float* ego_dims, const float* npc_dims) {
    if (!h) return fail(MEV_E_INVALID, "null handle");
    const size_t EN = size_t(h->cfg.num_envs) * size_t(h->cfg.num_agents);
    const size_t EK = size_t(h->cfg.num_envs) * size_t(h->cfg.max_npcs);
    for (int w = 0; w < 2; ++w) {
        const float* d = w ? npc_dims : ego_dims;
        const size_t n = 2 * (w ? EK : EN);
        if (d)
            for (size_t i = 0; i < n; ++i)
                if (!(fabsf(d[i]) <= 1.0e4f)) return fail(MEV_E_INVALID, "car length / width must be finite, |value| <= 1e4 px");
    }
    HIP_TRY(hipSetDevice(h->cfg.device));
    if (int r_ = serve_stop(h)) return r_;  // (the server holds the stream)
    if (ego_dims) HIP_TRY(hipMemcpyAsync(h->sp.ego_dim, ego_dims, EN * 2 * sizeof(float), hipMemcpyHostToDevice, h->stream));
    if (npc_dims && EK) HIP_TRY(hipMemcpyAsync(h->sp.npc_dim, npc_dims, EK * 2 * sizeof(float), hipMemcpyHostToDevice, h->stream));
    // whether any car differs from 54 x 24: the arrays given, and the device's for the other
    std::vector<float> e(ego_dims ? 0 : EN * 2), k(npc_dims ? 0 : EK * 2);
    if (!e.empty()) HIP_TRY(hipMemcpyAsync(e.data(), h->sp.ego_dim, e.size() * sizeof(float), hipMemcpyDeviceToHost, h->stream));
    if (!k.empty()) HIP_TRY(hipMemcpyAsync(k.data(), h->sp.npc_dim, k.size() * sizeof(float), hipMemcpyDeviceToHost, h->stream));
    HIP_TRY(hipStreamSynchronize(h->stream));
    const bool dflt = all_default_dims(ego_dims ? ego_dims : e.data(), EN) && all_default_dims(npc_dims ? npc_dims : k.data(), EK);
    h->sp.dims = dflt ? 0 : 1;  // (the next step refreshes the device copy of the parameters)
    h->deal_valid = false;      // (a dims handle runs another kernel: the deal restarts)
    return MEV_OK;
}

int mev_get_car_dims(mev_handle* h, float* ego_dims, float* npc_dims) {
    if (!h) return fail(MEV_E_INVALID, "null handle");
    const size_t EN = size_t(h->cfg.num_envs) * size_t(h->cfg.num_agents);
    const size_t EK = size_t(h->cfg.num_envs) * size_t(h->cfg.max_npcs);
    HIP_TRY(hipSetDevice(h->cfg.device));
    if (int r_ = serve_stop(h)) return r_;  // (the server holds the stream)
    if (ego_dims) HIP_TRY(hipMemcpyAsync(ego_dims, h->sp.ego_dim, EN * 2 * sizeof(float), hipMemcpyDeviceToHost, h->stream));
    if (npc_dims && EK) HIP_TRY(hipMemcpyAsync(npc_dims, h->sp.npc_dim, EK * 2 * sizeof(float), hipMemcpyDeviceToHost, h->stream));
    HIP_TRY(hipStreamSynchronize(h->stream));
    return MEV_OK;
}

int mev_car_dims_active(const mev_handle* h, int32_t* active) {
    if (!h || !active) return fail(MEV_E_INVALID, "null argument");
    *active = h->sp.dims;
    return MEV_OK;
}

// ---- LiDAR beam offsets (reference Lidar::rel_angles, cpp/Lidar.h:17, read-write through
// cpp/bindings.cpp:92): e.g. the first R angles of a longer beam list, which is what a
// reference Lidar whose `rays` was lowered casts (Lidar.cpp:24-25 indexes rel_angles up to
// rays).  The step's car-pair culling models the beams as rel[0] + b * (rel[R-1] - rel[0]) /
// (R - 1) with 2e-4 rad of margin (mev_kernels.hip phase 3b), so the offsets must be evenly
// spaced to 1e-5 rad; any other list is refused.
int mev_set_beam_angles(mev_handle* h, const float* rel) {
    if (!h || !rel) return fail(MEV_E_INVALID, "null argument");
    const int R = h->cfg.lidar_rays;
    for (int b = 0; b < R; ++b)
        if (!(fabsf(rel[b]) <= 1.0e3f)) return fail(MEV_E_INVALID, "beam angles must be finite, |angle| <= 1000 rad");
    h->sp.beam_cull = beam_cull_ok(rel, R);  // (any other list: no culling, SimParams::beam_cull)
    HIP_TRY(hipSetDevice(h->cfg.device));
    if (int r_ = serve_stop(h)) return r_;  // (the server holds the stream)
    HIP_TRY(hipStreamSynchronize(h->stream));
    HIP_TRY(hipMemcpy(h->d_rel, rel, size_t(R) * sizeof(float), hipMemcpyHostToDevice));
    return MEV_OK;
}

int mev_get_beam_angles(mev_handle* h, float* rel) {
    if (!h || !rel) return fail(MEV_E_INVALID, "null argument");
    HIP_TRY(hipSetDevice(h->cfg.device));
    if (int r_ = serve_stop(h)) return r_;  // (the server holds the stream)
    HIP_TRY(hipStreamSynchronize(h->stream));
    HIP_TRY(hipMemcpy(rel, h->d_rel, size_t(h->cfg.lidar_rays) * sizeof(float), hipMemcpyDeviceToHost));
    return MEV_OK;
}

int mev_set_ego_routes(mev_handle* h, const int32_t* routes) {
    if (!h || !routes) return fail(MEV_E_INVALID, "null argument");
    const size_t EN = size_t(h->cfg.num_envs) * size_t(h->cfg.num_agents);
    for (size_t i = 0; i < EN; ++i)
        if (routes[i] < 0 || routes[i] >= h->nroutes) return fail(MEV_E_RANGE, "ego route id out of range");
    HIP_TRY(hipSetDevice(h->cfg.device));
    if (int r_ = serve_stop(h)) return r_;  // (the server holds the stream)
    HIP_TRY(hipMemcpyAsync(h->sp.ego.route, routes, EN * sizeof(int32_t), hipMemcpyHostToDevice, h->stream));
    HIP_TRY(hipStreamSynchronize(h->stream));
    return MEV_OK;
}

int mev_set_traffic_routes(mev_handle* h, const int32_t* routes, int32_t count) {
    if (!h || (count > 0 && !routes)) return fail(MEV_E_INVALID, "null argument");
    if (count < 0 || count > h->P * h->P) return fail(MEV_E_INVALID, "bad traffic route count");
    for (int i = 0; i < count; ++i)
        if (routes[i] < 0 || routes[i] >= h->nroutes) return fail(MEV_E_RANGE, "traffic route id out of range");
    HIP_TRY(hipSetDevice(h->cfg.device));
    if (int r_ = serve_stop(h)) return r_;  // (the server holds the stream)
    h->h_traffic.assign(routes, routes + count);
    if (count > 0)
        HIP_TRY(hipMemcpyAsync(h->d_traffic, routes, size_t(count) * sizeof(int32_t), hipMemcpyHostToDevice, h->stream));
    HIP_TRY(hipStreamSynchronize(h->stream));
    h->sp.n_traffic_routes = count;
    return MEV_OK;
}

int mev_default_traffic_routes(const mev_handle* h, int32_t* routes, int32_t* count) {
    if (!h || !count) return fail(MEV_E_INVALID, "null argument");
    const auto d = mev::default_traffic_routes(h->cfg.num_lanes);
    if (routes) memcpy(routes, d.data(), d.size() * sizeof(int32_t));
    *count = int32_t(d.size());
    return MEV_OK;
}

static mev::Outputs resolve_outputs(mev_handle* h, float* obs, float* rew, uint8_t* done, uint8_t* status, uint8_t* term,
                                    uint8_t* trunc, int32_t* alive, int32_t* step, bool device) {
    mev::Outputs o = h->internal;
    if (device) {
        if (obs) o.obs = obs;
        if (rew) o.rew = rew;
        if (done) o.done = done;
        if (status) o.status = status;
        if (term) o.term = term;
        if (trunc) o.trunc = trunc;
        if (alive) o.alive_cnt = alive;
        if (step) o.step = step;
    }
    return o;
}

static int copy_out(mev_handle* h, const mev::Outputs& src, float* obs, float* rew, uint8_t* done, uint8_t* status,
                    uint8_t* term, uint8_t* trunc, int32_t* alive, int32_t* step, hipMemcpyKind kind) {
    const size_t E = size_t(h->cfg.num_envs), EN = E * size_t(h->cfg.num_agents);
    auto cp = [&](void* dst, const void* s, size_t bytes) -> hipError_t {
        if (!dst || dst == s) return hipSuccess;
        return hipMemcpyAsync(dst, s, bytes, kind, h->stream);
    };
    HIP_TRY(cp(obs, src.obs, EN * size_t(h->D) * sizeof(float)));
    HIP_TRY(cp(rew, src.rew, EN * sizeof(float)));
    HIP_TRY(cp(done, src.done, EN));
    HIP_TRY(cp(status, src.status, EN));
    HIP_TRY(cp(term, src.term, E));
    HIP_TRY(cp(trunc, src.trunc, E));
    HIP_TRY(cp(alive, src.alive_cnt, E * sizeof(int32_t)));
    HIP_TRY(cp(step, src.step, E * sizeof(int32_t)));
    return MEV_OK;
}

int mev_reset(mev_handle* h, const uint8_t* env_mask, float* obs, uint32_t flags) {
    if (!h) return fail(MEV_E_INVALID, "null handle");
    HIP_TRY(hipSetDevice(h->cfg.device));
    if (int r_ = serve_stop(h)) return r_;  // (the server holds the stream)
    const bool dev = (flags & MEV_DEVICE_PTRS) != 0;
    const uint8_t* d_mask = nullptr;
    if (env_mask) {
        if (dev) d_mask = env_mask;
        else {
            HIP_TRY(hipMemcpyAsync(h->d_mask, env_mask, size_t(h->cfg.num_envs), hipMemcpyHostToDevice, h->stream));
            d_mask = h->d_mask;
        }
    }
    mev::Outputs o = h->internal;
    if (dev && obs) o.obs = obs;
    h->deal_valid = false;  // NPC counts changed outside the step: the deal restarts
    HIP_TRY(mev::launch_reset(h->sp, d_mask, o, h->stream, h->rng_counter++));
    h->last.obs = o.obs;
    if (!dev) {
        if (obs) HIP_TRY(hipMemcpyAsync(obs, o.obs, size_t(h->cfg.num_envs) * size_t(h->cfg.num_agents) * size_t(h->D) * sizeof(float),
                                        hipMemcpyDeviceToHost, h->stream));
        HIP_TRY(hipStreamSynchronize(h->stream));
    }
    return MEV_OK;
}

// the pinned zero-copy block of a small handle (created at its first host-mode step)
static bool pin_ready(mev_handle* h) {
    if (h->pin) return true;
    const size_t E = size_t(h->cfg.num_envs), EN = E * size_t(h->cfg.num_agents);
    const size_t sz[10] = {EN * 2 * sizeof(float), E * sizeof(int32_t), EN * size_t(h->D) * sizeof(float),
                           EN * sizeof(float), EN, EN, E, E, E * sizeof(int32_t), E * sizeof(int32_t)};
    size_t off = 0;
    for (int k = 0; k < 10; ++k) {
        h->pin_off[k] = off;
        off += (sz[k] + 255) & ~size_t(255);
    }
    if (off - h->pin_off[2] > mev_handle::kPinMax) return false;  // large outputs: device buffers + DMA copies
    void* hp = nullptr;
    if (hipHostMalloc(&hp, off, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess) return false;
    void* dp = nullptr;
    if (hipHostGetDevicePointer(&dp, hp, 0) != hipSuccess) {
        (void)hipHostFree(hp);
        return false;
    }
    h->pin = static_cast<uint8_t*>(hp);
    h->pin_dev = static_cast<uint8_t*>(dp);
    uint8_t* d = h->pin_dev;
    h->pin_out.obs = reinterpret_cast<float*>(d + h->pin_off[2]);
    h->pin_out.rew = reinterpret_cast<float*>(d + h->pin_off[3]);
    h->pin_out.done = d + h->pin_off[4];
    h->pin_out.status = d + h->pin_off[5];
    h->pin_out.term = d + h->pin_off[6];
    h->pin_out.trunc = d + h->pin_off[7];
    h->pin_out.alive_cnt = reinterpret_cast<int32_t*>(d + h->pin_off[8]);
    h->pin_out.step = reinterpret_cast<int32_t*>(d + h->pin_off[9]);
    h->pin_out.obs_ld = h->D;
    return true;
}

// ---- the persistent step server (k_serve; protocol in mev_kernels.h ServeBox) ----
namespace {
constexpr double kServeTimeoutMs = 10000.0;  // no answer within this: the call fails

inline void cpu_relax() {
#if defined(__x86_64__)
    __builtin_ia32_pause();
#endif
}

constexpr double kServeIdleMinUs = 200.0, kServeIdleMaxUs = 2000.0;
constexpr int kServeMissLimit = 4;        // consecutive posts that found the server gone ...
constexpr uint64_t kPausedSteps = 1024;  // ... pause serving for this many host steps

// the idle limit of the next instance, in ticks of s_memrealtime (100 MHz):
// MEV_SERVE_IDLE_MS fixes it (1..1000 ms); otherwise adaptive (mev_handle::serve_gap_us)
uint32_t serve_idle_ticks(const mev_handle* h) {
    static const int fixed_ms = [] {
        const char* v = getenv("MEV_SERVE_IDLE_MS");
        if (!v) return 0;
        const int m = atoi(v);
        return m < 1 ? 1 : (m > 1000 ? 1000 : m);
    }();
    if (fixed_ms > 0) return (uint32_t)fixed_ms * 100000u;
    double us = 8.0 * h->serve_gap_us;
    us = us < kServeIdleMinUs ? kServeIdleMinUs : (us > kServeIdleMaxUs ? kServeIdleMaxUs : us);
    return (uint32_t)(us * 100.0);
}

// post a command: the line's fields are written by the caller, then cmd, then seq (release)
void serve_post(mev_handle* h, uint32_t cmd) {
    volatile mev::ServeBox* b = h->sbox;
    b->cmd = cmd;
    std::atomic_thread_fence(std::memory_order_seq_cst);
    b->seq = ++h->serve_seq;
    std::atomic_thread_fence(std::memory_order_seq_cst);
}

int serve_launch(mev_handle* h) {
    mev::ServeArgs sa{};
    sa.box = h->sbox_dev;
    sa.actions = reinterpret_cast<const float*>(h->pin_dev + h->pin_off[0]);
    sa.spawn_route = reinterpret_cast<const int32_t*>(h->pin_dev + h->pin_off[1]);
    sa.epoch = ++h->serve_epoch;
    sa.idle_ticks = serve_idle_ticks(h);
    HIP_TRY(hipEventRecord(h->serve_ev, h->stream));  // after whatever the handle's stream holds
    HIP_TRY(hipStreamWaitEvent(h->serve_stream, h->serve_ev, 0));
    HIP_TRY(mev::launch_serve(h->sp, h->d_sp, sa, h->pin_out, h->serve_stream));
    h->serve_running = true;
    h->serve_wg = h->sp.E;
    ++h->serve_launches;
    return MEV_OK;
}

// Resident servers per process are capped: their high-priority hardware queues are
// few, and a server launched behind another one's on a shared queue would wait for its
// idle exit.  Handles beyond the cap step launched (same results).  A slot belongs to
// the handle that took it -- across its server's idle exits and paused stretches --
// until the handle is closed, or has made no host step for kServeStaleMs when another
// handle asks for a slot: which handles are served does not depend on the timing of
// idle exits (a round-robin over more handles than slots serves the first ones).
constexpr int kMaxResidentServers = 2;
constexpr int64_t kServeStaleMs = 50;
std::mutex g_serve_mu;
std::vector<mev_handle*> g_serving;  // the slots' owners (<= kMaxResidentServers)

int64_t now_ns() {
    return std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now().time_since_epoch())
        .count();
}

// whether h's server is still resident (some workgroup has not yet left)
bool serve_resident(const mev_handle* h) {
    if (!h->serve_running) return false;
    const volatile mev::ServeBox* b = h->sbox;
    for (int w = 0; w < h->serve_wg; ++w)
        if (b->exited[w] != h->serve_epoch) return true;
    return false;
}

// h may keep or start a resident server: it owns a slot, or takes a free one (or
// one whose owner has stepped no host step for kServeStaleMs and has no server left)
bool serve_slot(mev_handle* h) {
    std::lock_guard<std::mutex> lk(g_serve_mu);
    for (const mev_handle* x : g_serving)
        if (x == h) return true;
    if ((int)g_serving.size() >= kMaxResidentServers) {
        const int64_t t = now_ns();
        for (size_t i = 0; i < g_serving.size(); ++i) {
            const mev_handle* x = g_serving[i];
            if (!serve_resident(x) && t - x->serve_last_ns.load(std::memory_order_relaxed) > kServeStaleMs * 1000000) {
                g_serving.erase(g_serving.begin() + long(i));
                break;
            }
        }
    }
    if ((int)g_serving.size() >= kMaxResidentServers) return false;
    g_serving.push_back(h);
    return true;
}

void serve_unlist(mev_handle* h) {
    std::lock_guard<std::mutex> lk(g_serve_mu);
    for (size_t i = 0; i < g_serving.size(); ++i)
        if (g_serving[i] == h) {
            g_serving.erase(g_serving.begin() + long(i));
            break;
        }
}

double ms_since(std::chrono::steady_clock::time_point t0) {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}
}  // namespace

// Stop a resident server (every other call on the handle does this first): post
// STOP, wait until every workgroup has left, then the stream is free.
static int serve_stop(mev_handle* h) {
    if (!h->serve_running) return MEV_OK;
    serve_post(h, mev::kServeStop);
    volatile mev::ServeBox* b = h->sbox;
    const auto t0 = std::chrono::steady_clock::now();
    for (int w = 0; w < h->serve_wg; ++w)
        while (b->exited[w] != h->serve_epoch) {
            if (ms_since(t0) > kServeTimeoutMs) return fail(MEV_E_HIP, "step server: no stop within 10 s");
            cpu_relax();
        }
    h->serve_running = false;
    HIP_TRY(hipStreamSynchronize(h->serve_stream));  // the server's grid has drained
    return MEV_OK;
}

// whether a host-mode step of h (pinned block ready) goes to the server
static bool serve_wanted(mev_handle* h) {
    static const bool off = [] { const char* v = getenv("MEV_NO_SERVE"); return v && v[0] == '1'; }();
    // (only on the handle's own non-blocking stream: a resident server would hold back
    // whatever a caller queues behind it on a stream it shares)
    if (off || h->serve_mode == 0 || !h->tev.empty() || h->stream != h->own_stream || !mev::serve_fits(h->sp))
        return false;
    if (h->serve_pause > 0) {  // repeated idle exits between posts: launched steps for a while
        --h->serve_pause;
        return false;
    }
    if (h->sbox) return true;
    if (!h->serve_stream || !h->serve_ev) {
        int lo = 0, hi = 0;
        if (hipDeviceGetStreamPriorityRange(&lo, &hi) != hipSuccess) return false;
        if (hipStreamCreateWithPriority(&h->serve_stream, hipStreamNonBlocking, hi) != hipSuccess) {
            h->serve_stream = nullptr;
            return false;
        }
        if (hipEventCreateWithFlags(&h->serve_ev, hipEventDisableTiming) != hipSuccess) {
            (void)hipStreamDestroy(h->serve_stream);
            h->serve_stream = nullptr;
            h->serve_ev = nullptr;
            return false;
        }
    }
    void* hp = nullptr;
    if (hipHostMalloc(&hp, sizeof(mev::ServeBox), hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess) return false;
    void* dp = nullptr;
    if (hipHostGetDevicePointer(&dp, hp, 0) != hipSuccess) {
        (void)hipHostFree(hp);
        return false;
    }
    memset(hp, 0, sizeof(mev::ServeBox));
    h->sbox = static_cast<mev::ServeBox*>(hp);
    h->sbox_dev = static_cast<mev::ServeBox*>(dp);
    return true;
}

// one step through the server: post it (launching an instance if none is
// resident) and wait until every workgroup has answered.  A workgroup that left
// (idle) without answering: the instance is stopped, the same step (same sid) is
// posted again and a new instance launched; workgroups that had answered skip it.
static int serve_step(mev_handle* h, const mev::StepInputs& in) {
    volatile mev::ServeBox* b = h->sbox;
    if (h->serve_running) {  // the host gap since the last answer, and whether the server waited for it
        const double gap_us = 1000.0 * ms_since(h->serve_t_answer);
        h->serve_gap_us = 0.875 * h->serve_gap_us + 0.125 * (gap_us < kServeIdleMaxUs ? gap_us : kServeIdleMaxUs);
        if (b->exited[0] != h->serve_epoch) {  // still resident: a hit
            h->serve_misses = 0;
        } else {  // it left (idle) before this post
            ++h->serve_misses_total;
            if (++h->serve_misses >= kServeMissLimit) {
                h->serve_misses = 0;
                h->serve_pause = kPausedSteps;
            }
        }
    }
    const uint32_t sid = ++h->serve_sid;
    uint32_t u;
    b->sid = sid;
    memcpy(&u, &in.dt, 4);
    b->dt = u;
    memcpy(&u, &in.spawn_prob, 4);
    b->spawn_prob = u;
    b->auto_reset = (uint32_t)in.auto_reset;
    b->spawn = in.spawn_route ? 1u : 0u;
    b->rng_lo = (uint32_t)in.rng_counter;
    b->rng_hi = (uint32_t)(in.rng_counter >> 32);
    serve_post(h, mev::kServeStep);
    if (!h->serve_running)
        if (int r = serve_launch(h)) return r;
    const auto t0 = std::chrono::steady_clock::now();
    for (int w = 0; w < h->serve_wg; ++w) {
        while (b->done[w] != sid) {
            if (b->exited[w] == h->serve_epoch) {
                std::atomic_thread_fence(std::memory_order_seq_cst);
                if (b->done[w] == sid) break;  // answered, then left
                if (int r = serve_stop(h)) return r;
                serve_post(h, mev::kServeStep);  // the same step again
                if (int r = serve_launch(h)) return r;
                w = 0;
                continue;
            }
            if (ms_since(t0) > kServeTimeoutMs) return fail(MEV_E_HIP, "step server: no answer within 10 s");
            cpu_relax();
        }
    }
    std::atomic_thread_fence(std::memory_order_seq_cst);
    ++h->serve_steps;
    h->serve_t_answer = std::chrono::steady_clock::now();
    return MEV_OK;
}

int mev_set_serve(mev_handle* h, int32_t mode) {
    if (!h) return fail(MEV_E_INVALID, "null handle");
    if (mode != 0 && mode != 1) return fail(MEV_E_INVALID, "serve mode must be 0 (off) or 1 (automatic)");
    HIP_TRY(hipSetDevice(h->cfg.device));
    if (int r = serve_stop(h)) return r;
    h->serve_mode = mode;
    if (mode == 0) serve_unlist(h);  // (its slot, if it owns one, goes to the next handle that asks)
    return MEV_OK;
}

int mev_serve_stats(const mev_handle* h, uint64_t* steps, uint64_t* launches, int32_t* running) {
    if (!h) return fail(MEV_E_INVALID, "null handle");
    if (steps) *steps = h->serve_steps;
    if (launches) *launches = h->serve_launches;
    if (running) *running = h->serve_running ? 1 : 0;
    return MEV_OK;
}

int mev_step(mev_handle* h, const mev_step_args* a) {
    if (!h || !a) return fail(MEV_E_INVALID, "null argument");
    if (!a->actions) return fail(MEV_E_INVALID, "actions required");
    const bool gather = (a->flags & MEV_GATHER_TO_ROOT) != 0;
    if (gather) {
        if (!h->comm) return fail(MEV_E_INVALID, "MEV_GATHER_TO_ROOT needs a communicator (mev_comm_init)");
        if (a->obs || a->reward || a->done || a->status || a->terminated || a->truncated)
            return fail(MEV_E_INVALID, "MEV_GATHER_TO_ROOT writes the outputs packed: pass NULL output pointers");
    }
    HIP_TRY(hipSetDevice(h->cfg.device));
    const bool dev = (a->flags & MEV_DEVICE_PTRS) != 0;
    const size_t E = size_t(h->cfg.num_envs), EN = E * size_t(h->cfg.num_agents);
    mev::StepInputs in{};
    in.dt = a->dt;
    in.auto_reset = (a->flags & MEV_AUTO_RESET) ? 1 : 0;
    in.rng_counter = h->rng_counter++;
    const bool pinned = !dev && !gather && pin_ready(h);  // zero-copy host mode (small handles)
    if (pinned) h->serve_last_ns.store(now_ns(), std::memory_order_relaxed);  // (a slot owner keeps stepping)
    const bool serve = pinned && serve_wanted(h) && serve_slot(h);  // ... answered by the resident step server
    if (!serve)
        if (int r = serve_stop(h)) return r;
    if (dev) {
        in.actions = a->actions;
        in.spawn_route = a->spawn_route;
    } else if (pinned) {
        // the previous host-mode step was synchronized: the block is free
        memcpy(h->pin + h->pin_off[0], a->actions, EN * 2 * sizeof(float));
        in.actions = reinterpret_cast<const float*>(h->pin_dev + h->pin_off[0]);
        if (a->spawn_route) {
            memcpy(h->pin + h->pin_off[1], a->spawn_route, E * sizeof(int32_t));
            in.spawn_route = reinterpret_cast<const int32_t*>(h->pin_dev + h->pin_off[1]);
        }
    } else {
        HIP_TRY(hipMemcpyAsync(h->d_actions, a->actions, EN * 2 * sizeof(float), hipMemcpyHostToDevice, h->stream));
        in.actions = h->d_actions;
        if (a->spawn_route) {
            HIP_TRY(hipMemcpyAsync(h->d_spawn, a->spawn_route, E * sizeof(int32_t), hipMemcpyHostToDevice, h->stream));
            in.spawn_route = h->d_spawn;
        }
    }
    // spawn probability, TrafficFlow.cpp:321-322 (host glibc expf, bit-identical to the reference)
    in.spawn_prob = 1.0f - expf(-h->cfg.traffic_density * a->dt);
    mev::Outputs o = pinned ? h->pin_out
                            : resolve_outputs(h, a->obs, a->reward, a->done, a->status, a->terminated, a->truncated,
                                              a->agents_alive, a->step, dev);
    const int slot = int(h->gathers & 1);
    if (gather) {
        // this rank's packed slot: on the root its own row of the gather buffer
        // (no copy), elsewhere the send buffer; step t and t+2 share a buffer
        if (h->gather_pending[slot]) HIP_TRY(hipStreamWaitEvent(h->stream, h->ev_gather[slot], 0));
        uint8_t* base = h->pk_buf[slot] + (h->rank == h->root ? size_t(h->root) * h->pk_bytes : 0);
        o.obs = reinterpret_cast<float*>(base + h->pk_off[MEV_PK_OBS]);
        o.rew = reinterpret_cast<float*>(base + h->pk_off[MEV_PK_REWARD]);
        o.done = base + h->pk_off[MEV_PK_DONE];
        o.status = base + h->pk_off[MEV_PK_STATUS];
        o.term = base + h->pk_off[MEV_PK_TERMINATED];
        o.trunc = base + h->pk_off[MEV_PK_TRUNCATED];
        if (h->gather_fmt == MEV_GATHER_STATE) {  // post-step state + one LiDAR code per beam, no heads
            o.obs = nullptr;
            o.obs_ld = 0;
            o.lidar_u8 = base + h->pk_off[MEV_PK_LIDAR];
            o.state = base + h->pk_off[MEV_PK_STATE];
            o.state_n = int64_t(h->slots) * h->cfg.num_agents;
        } else if (h->gather_fmt == MEV_GATHER_LIDAR_U8) {  // heads [slots][N][31] + one LiDAR code per beam
            o.obs_ld = mev::OBS_HEAD;
            o.lidar_u8 = base + h->pk_off[MEV_PK_LIDAR];
        }
    }
    const hipEvent_t* ev = nullptr;
    if (!h->tev.empty() && (h->t_phase++ % h->t_every) == 0) {
        if (size_t(3 * (h->tn + 1)) > h->tev.size()) HIP_TRY(h->fold_timing());
        ev = &h->tev[size_t(3 * h->tn)];
        ++h->tn;
    }
    if (!h->sp_valid || memcmp(&h->sp, &h->sp_dev, sizeof(mev::SimParams)) != 0) {
        // parameters changed (configuration calls only): stream-ordered after the
        // launches that read the previous copy; waited for, so the host copy is free
        if (int r = serve_stop(h)) return r;
        HIP_TRY(hipMemcpyAsync(h->d_sp, &h->sp, sizeof(mev::SimParams), hipMemcpyHostToDevice, h->stream));
        HIP_TRY(hipStreamSynchronize(h->stream));
        memcpy(&h->sp_dev, &h->sp, sizeof(mev::SimParams));
        h->sp_valid = true;
    }
    // the NPC-aware deal (fused traffic k_step only; mev_set_env_deal)
    const bool deal = !serve && h->sp.traffic && h->sp.deal_cnt && h->deal_on && mev::step_kernel_for(h->sp) == 2;
    // classes are NPC-slot counts the next step loads (mev_kernels.hip cars_pre): rings whose
    // ended envs were put in class 0 by an auto-resetting step are not a bound for a step
    // without the reset (the env keeps its NPCs), so such a step deals afresh
    if (h->deal_valid && h->deal_ar && !in.auto_reset) h->deal_valid = false;
    if (deal) {
        if (!h->deal_valid) {  // fresh rings: this step deals by the identity order and builds the next
            HIP_TRY(hipMemsetAsync(h->sp.deal_cnt, 0, size_t(3) * mev::kDealRingInts * sizeof(int32_t), h->stream));
            h->deal_ring = 0;
        }
        in.deal = 2 | (h->deal_valid ? 1 : 0);
        in.deal_ring = h->deal_ring;
    }
    if (serve) {
        if (int r = serve_step(h, in)) return r;
    } else {
        HIP_TRY(mev::launch_step(h->sp, h->d_sp, in, o, h->stream, ev));
    }
    h->deal_valid = deal;
    h->deal_ar = in.auto_reset != 0;
    if (deal) h->deal_ring = h->deal_ring == 2 ? 0 : h->deal_ring + 1;
    h->last = o;
    if (gather && h->world == 1) {
        ++h->gathers;  // a world of one: the root's row is written in place, nothing to move
    } else if (gather) {
        // one grouped send/recv on the communication stream, after the step
        HIP_TRY(hipEventRecord(h->ev_step[slot], h->stream));
        HIP_TRY(hipStreamWaitEvent(h->comm_stream, h->ev_step[slot], 0));
        {
            ncclResult_t nr = ncclGroupStart();
            if (h->rank == h->root) {
                for (int r = 0; r < h->world && nr == ncclSuccess; ++r)
                    if (r != h->root)
                        nr = ncclRecv(h->pk_buf[slot] + size_t(r) * h->pk_bytes, h->pk_bytes, ncclUint8, r, h->comm,
                                      h->comm_stream);
            } else {
                nr = ncclSend(h->pk_buf[slot], h->pk_bytes, ncclUint8, h->root, h->comm, h->comm_stream);
            }
            const ncclResult_t ne = ncclGroupEnd();
            if (nr == ncclSuccess) nr = ne;
            if (nr != ncclSuccess) return fail(MEV_E_HIP, std::string("RCCL gather: ") + ncclGetErrorString(nr));
        }
        HIP_TRY(hipEventRecord(h->ev_gather[slot], h->comm_stream));
        h->gather_pending[slot] = true;
        ++h->gathers;
    }
    if (pinned) {
        if (!serve) HIP_TRY(hipStreamSynchronize(h->stream));
        const size_t EN_ = EN, E_ = E;
        auto cp = [&](void* dst, int k, size_t bytes) {
            if (dst) memcpy(dst, h->pin + h->pin_off[k], bytes);
        };
        cp(a->obs, 2, EN_ * size_t(h->D) * sizeof(float));
        cp(a->reward, 3, EN_ * sizeof(float));
        cp(a->done, 4, EN_);
        cp(a->status, 5, EN_);
        cp(a->terminated, 6, E_);
        cp(a->truncated, 7, E_);
        cp(a->agents_alive, 8, E_ * sizeof(int32_t));
        cp(a->step, 9, E_ * sizeof(int32_t));
    } else if (!dev) {
        int r = copy_out(h, o, a->obs, a->reward, a->done, a->status, a->terminated, a->truncated, a->agents_alive,
                         a->step, hipMemcpyDeviceToHost);
        if (r) return r;
        HIP_TRY(hipStreamSynchronize(h->stream));
    }
    return MEV_OK;
}

static int sync_internal(mev_handle* h);  // below, with mev_device_outputs

int mev_get_outputs(mev_handle* h, float* obs, float* rew, uint8_t* done, uint8_t* status, uint8_t* term,
                    uint8_t* trunc, int32_t* alive, int32_t* step, uint32_t flags) {
    if (!h) return fail(MEV_E_INVALID, "null handle");
    HIP_TRY(hipSetDevice(h->cfg.device));
    if (int r_ = serve_stop(h)) return r_;  // (the server holds the stream)
    const bool dev = (flags & MEV_DEVICE_PTRS) != 0;
    if (h->last.lidar_u8) {  // compact gather row: decoded into the handle's buffers first
        if (int r0 = sync_internal(h)) return r0;
    }
    int r = copy_out(h, h->last, obs, rew, done, status, term, trunc, alive, step,
                     dev ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost);
    if (r) return r;
    if (!dev) HIP_TRY(hipStreamSynchronize(h->stream));
    return MEV_OK;
}

#define STATE_FIELDS(X)                                                                                    \
    X(x, ego.x, EN, float) X(y, ego.y, EN, float) X(v, ego.v, EN, float) X(heading, ego.h, EN, float)      \
    X(acc, ego.acc, EN, float) X(steering, ego.steer, EN, float) X(prev_dist, ego.prev_dist, EN, float)    \
    X(prev_a0, ego.pa0, EN, float) X(prev_a1, ego.pa1, EN, float) X(spawn_x, ego.sx, EN, float)            \
    X(spawn_y, ego.sy, EN, float) X(spawn_v, ego.sv, EN, float) X(spawn_heading, ego.sh, EN, float)        \
    X(path_index, ego.pidx, EN, int32_t) X(route, ego.route, EN, int32_t)                                  \
    X(intention, ego.intent, EN, int32_t) X(alive, ego.alive, EN, uint8_t)                                 \
    X(npc_x, npc.x, EK, float) X(npc_y, npc.y, EK, float) X(npc_v, npc.v, EK, float)                        \
    X(npc_heading, npc.h, EK, float) X(npc_acc, npc.acc, EK, float) X(npc_steering, npc.steer, EK, float)  \
    X(npc_path_index, npc.pidx, EK, int32_t) X(npc_route, npc.route, EK, int32_t)                          \
    X(npc_intention, npc.intent, EK, int32_t) X(npc_alive, npc.alive, EK, uint8_t)                         \
    X(npc_count, npc.count, E, int32_t) X(step_count, step_count, E, int32_t)

int mev_get_state(mev_handle* h, const mev_state* s) {
    if (!h || !s) return fail(MEV_E_INVALID, "null argument");
    HIP_TRY(hipSetDevice(h->cfg.device));
    if (int r_ = serve_stop(h)) return r_;  // (the server holds the stream)
    const size_t E = size_t(h->cfg.num_envs), EN = E * size_t(h->cfg.num_agents);
    const size_t EK = E * size_t(h->cfg.max_npcs);
    // Staged through pinned memory in at most six DMA copies: the 4-byte fields of the
    // ego and of the NPC SoA are one block each (field k at k * stride), then the alive
    // flags and the per-env counters; one pageable copy per field cost ~15 us each
    // (29 of them: env.py's traffic_cars read-back per step).
    void* const ego4[mev::EF_COUNT] = {s->x, s->y, s->v, s->heading, s->acc, s->steering, s->prev_dist,
                                      s->prev_a0, s->prev_a1, s->spawn_x, s->spawn_y, s->spawn_v,
                                      s->spawn_heading, s->path_index, s->route, s->intention};
    void* const npc4[mev::NF_COUNT] = {s->npc_x, s->npc_y, s->npc_v, s->npc_heading, s->npc_acc,
                                      s->npc_steering, s->npc_path_index, s->npc_route, s->npc_intention};
    bool want_e = false, want_n = false;
    for (void* q : ego4) want_e |= q != nullptr;
    for (void* q : npc4) want_n |= q != nullptr;
    const size_t es = size_t(h->sp.ego.stride) * 4, ns = size_t(h->sp.npc.stride) * 4;
    auto al = [](size_t b) { return (b + 255) & ~size_t(255); };
    const size_t o_e = 0, o_n = o_e + al(es * mev::EF_COUNT), o_ea = o_n + al(ns * mev::NF_COUNT);
    const size_t o_na = o_ea + al(EN), o_nc = o_na + al(EK), o_sc = o_nc + al(E * 4), total = o_sc + al(E * 4);
    if (h->gs_cap < total) {
        if (h->gs_pin) (void)hipHostFree(h->gs_pin);
        h->gs_pin = nullptr;
        h->gs_cap = 0;
        HIP_TRY(hipHostMalloc(reinterpret_cast<void**>(&h->gs_pin), total, hipHostMallocDefault));
        h->gs_cap = total;
    }
    uint8_t* st = h->gs_pin;
    auto d2h = [&](size_t off, const void* src, size_t bytes) -> hipError_t {
        return bytes ? hipMemcpyAsync(st + off, src, bytes, hipMemcpyDeviceToHost, h->stream) : hipSuccess;
    };
    if (want_e) HIP_TRY(d2h(o_e, h->sp.ego.x, es * mev::EF_COUNT));
    if (want_n && EK) HIP_TRY(d2h(o_n, h->sp.npc.x, ns * mev::NF_COUNT));
    if (s->alive) HIP_TRY(d2h(o_ea, h->sp.ego.alive, EN));
    if (s->npc_alive) HIP_TRY(d2h(o_na, h->sp.npc.alive, EK));
    if (s->npc_count) HIP_TRY(d2h(o_nc, h->sp.npc.count, E * 4));
    if (s->step_count) HIP_TRY(d2h(o_sc, h->sp.step_count, E * 4));
    HIP_TRY(hipStreamSynchronize(h->stream));
    for (int k = 0; k < mev::EF_COUNT; ++k)
        if (ego4[k]) memcpy(ego4[k], st + o_e + size_t(k) * es, EN * 4);
    for (int k = 0; k < mev::NF_COUNT; ++k)
        if (npc4[k] && EK) memcpy(npc4[k], st + o_n + size_t(k) * ns, EK * 4);
    if (s->alive) memcpy(s->alive, st + o_ea, EN);
    if (s->npc_alive && EK) memcpy(s->npc_alive, st + o_na, EK);
    if (s->npc_count) memcpy(s->npc_count, st + o_nc, E * 4);
    if (s->step_count) memcpy(s->step_count, st + o_sc, E * 4);
    return MEV_OK;
}

int mev_set_state(mev_handle* h, const mev_state* s) {
    if (!h || !s) return fail(MEV_E_INVALID, "null argument");
    HIP_TRY(hipSetDevice(h->cfg.device));
    if (int r_ = serve_stop(h)) return r_;  // (the server holds the stream)
    const size_t E = size_t(h->cfg.num_envs), EN = E * size_t(h->cfg.num_agents);
    const size_t EK = E * size_t(h->cfg.max_npcs);
    if (s->route)
        for (size_t i = 0; i < EN; ++i)
            if (s->route[i] < 0 || s->route[i] >= h->nroutes) return fail(MEV_E_RANGE, "route id out of range");
    if (s->npc_count)
        for (size_t e = 0; e < E; ++e)
            if (s->npc_count[e] < 0 || s->npc_count[e] > h->cfg.max_npcs) return fail(MEV_E_RANGE, "npc_count out of range");
    if (s->npc_route)
        for (size_t i = 0; i < EK; ++i)
            if (s->npc_route[i] < 0 || s->npc_route[i] >= h->nroutes) return fail(MEV_E_RANGE, "npc route id out of range");
#define SET(f, dev, n, T) \
    if (s->f) HIP_TRY(hipMemcpyAsync(h->sp.dev, s->f, (n) * sizeof(T), hipMemcpyHostToDevice, h->stream));
    STATE_FIELDS(SET)
#undef SET
    HIP_TRY(hipMemsetAsync(h->sp.pending_reset, 0, E, h->stream));
    h->deal_valid = false;
    HIP_TRY(mev::launch_observe_reset_lidar(h->sp, h->internal, h->stream));
    h->last.obs = h->internal.obs;
    HIP_TRY(hipStreamSynchronize(h->stream));
    return MEV_OK;
}

// The handle's own output buffers made to hold the last outputs: a step that wrote
// elsewhere (caller buffers, the pinned host block of a host-mode step, a packed
// gather row) is copied in, stream-ordered, and h->last points back at them.
static int sync_internal(mev_handle* h) {
    const size_t E = size_t(h->cfg.num_envs), EN = E * size_t(h->cfg.num_agents);
    const mev::Outputs& L = h->last;
    const mev::Outputs& I = h->internal;
    auto pull = [&](void* dst, const void* src, size_t bytes) -> hipError_t {
        if (!src || src == dst) return hipSuccess;
        return hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, h->stream);
    };
    if (L.state)  // a state-format gather row: rebuild the heads, decode the LiDAR codes
        HIP_TRY(mev::launch_decode_state(h->sp, L.state, L.lidar_u8, 0, int(L.state_n / h->cfg.num_agents), int(E),
                                         h->d_lidar_table, I.obs, h->stream));
    else if (L.lidar_u8)  // a compact-format gather row: decode heads + LiDAR codes into the obs rows
        HIP_TRY(mev::launch_unpack_lidar_u8(L.obs, L.lidar_u8, h->d_lidar_table, I.obs, int(EN), h->D, h->lidar_slots,
                                            h->stream));
    else
        HIP_TRY(pull(I.obs, L.obs, EN * size_t(h->D) * sizeof(float)));
    HIP_TRY(pull(I.rew, L.rew, EN * sizeof(float)));
    HIP_TRY(pull(I.done, L.done, EN));
    HIP_TRY(pull(I.status, L.status, EN));
    HIP_TRY(pull(I.term, L.term, E));
    HIP_TRY(pull(I.trunc, L.trunc, E));
    HIP_TRY(pull(I.alive_cnt, L.alive_cnt, E * sizeof(int32_t)));
    HIP_TRY(pull(I.step, L.step, E * sizeof(int32_t)));
    h->last = h->internal;
    return MEV_OK;
}

int mev_device_outputs(mev_handle* h, float** obs, float** rew, uint8_t** done, uint8_t** status, uint8_t** term,
                       uint8_t** trunc) {
    if (!h) return fail(MEV_E_INVALID, "null handle");
    HIP_TRY(hipSetDevice(h->cfg.device));
    if (int r_ = serve_stop(h)) return r_;  // (the server holds the stream)
    if (int r = sync_internal(h)) return r;
    if (obs) *obs = h->internal.obs;
    if (rew) *rew = h->internal.rew;
    if (done) *done = h->internal.done;
    if (status) *status = h->internal.status;
    if (term) *term = h->internal.term;
    if (trunc) *trunc = h->internal.trunc;
    return MEV_OK;
}

int mev_kernel_timing(mev_handle* h, int32_t enable) {
    if (!h) return fail(MEV_E_INVALID, "null handle");
    if (enable < 0) return fail(MEV_E_INVALID, "enable must be >= 0");
    HIP_TRY(hipSetDevice(h->cfg.device));
    if (int r_ = serve_stop(h)) return r_;  // (the server holds the stream)
    if (!enable) {
        HIP_TRY(hipStreamSynchronize(h->stream));
        h->free_timing();
        return MEV_OK;
    }
    if (h->tev.empty()) {
        const int ring = 4096;  // steps between host folds
        h->tev.resize(size_t(3 * ring), nullptr);
        for (auto& ev : h->tev) HIP_TRY(hipEventCreate(&ev));
    }
    h->tn = 0;
    h->t_every = enable;
    h->t_phase = 0;
    h->t_cars_ms = h->t_lidar_ms = 0.0;
    h->t_steps = 0;
    return MEV_OK;
}

int mev_kernel_times(mev_handle* h, double* cars_ms, double* lidar_ms, int64_t* steps) {
    if (!h || !cars_ms || !lidar_ms || !steps) return fail(MEV_E_INVALID, "null argument");
    if (h->tev.empty()) return fail(MEV_E_INVALID, "kernel timing is not enabled");
    HIP_TRY(hipSetDevice(h->cfg.device));
    if (int r_ = serve_stop(h)) return r_;  // (the server holds the stream)
    HIP_TRY(h->fold_timing());
    *cars_ms = h->t_cars_ms;
    *lidar_ms = h->t_lidar_ms;
    *steps = h->t_steps;
    h->t_cars_ms = h->t_lidar_ms = 0.0;
    h->t_steps = 0;
    return MEV_OK;
}

int mev_set_step_kernel(mev_handle* h, int32_t kernel) {
    if (!h) return fail(MEV_E_INVALID, "null handle");
    if (kernel < 0 || kernel > 2) return fail(MEV_E_INVALID, "step kernel must be 0 (auto), 1 (two kernels) or 2 (fused)");
    mev::SimParams q = h->sp;
    q.step_kernel = kernel;
    if (mev::step_kernel_for(q) == 0)
        return fail(MEV_E_INVALID, "the fused step kernel does not support this configuration (traffic mode or too much LDS)");
    HIP_TRY(hipSetDevice(h->cfg.device));
    if (int r_ = serve_stop(h)) return r_;  // (the server holds the stream)
    HIP_TRY(hipStreamSynchronize(h->stream));
    h->sp.step_kernel = kernel;
    return MEV_OK;
}

int mev_get_step_kernel(const mev_handle* h, int32_t* kernel) {
    if (!h || !kernel) return fail(MEV_E_INVALID, "null argument");
    *kernel = mev::step_kernel_for(h->sp);
    return MEV_OK;
}

int mev_set_step_pack(mev_handle* h, int32_t envs_per_wave) {
    if (!h) return fail(MEV_E_INVALID, "null handle");
    if (envs_per_wave != 0 && envs_per_wave != 1 && envs_per_wave != 2 && envs_per_wave != 4 && envs_per_wave != 8)
        return fail(MEV_E_INVALID, "envs per wave must be 0 (auto), 1, 2, 4 or 8");
    HIP_TRY(hipSetDevice(h->cfg.device));
    if (int r_ = serve_stop(h)) return r_;  // (the server holds the stream)
    HIP_TRY(hipStreamSynchronize(h->stream));
    h->sp.step_pack = envs_per_wave;
    return MEV_OK;
}

int mev_get_step_pack(const mev_handle* h, int32_t* envs_per_wave) {
    if (!h || !envs_per_wave) return fail(MEV_E_INVALID, "null argument");
    *envs_per_wave = mev::step_kernel_for(h->sp) == 2 ? mev::step_pack(h->sp) : 1;
    return MEV_OK;
}

int mev_set_step_split(mev_handle* h, int32_t mode) {
    if (!h) return fail(MEV_E_INVALID, "null handle");
    if (mode < 0 || mode > 3)
        return fail(MEV_E_INVALID, "split mode must be 0 (auto), 1 (off), 2 (on) or 3 (early split)");
    HIP_TRY(hipSetDevice(h->cfg.device));
    if (int r_ = serve_stop(h)) return r_;  // (the server holds the stream)
    HIP_TRY(hipStreamSynchronize(h->stream));
    h->sp.step_split = mode;
    h->deal_valid = false;  // (the traffic early split deals several envs per workgroup: restart the rings)
    return MEV_OK;
}

int mev_set_env_deal(mev_handle* h, int32_t on) {
    if (!h) return fail(MEV_E_INVALID, "null handle");
    if (on != 0 && on != 1) return fail(MEV_E_INVALID, "env deal must be 0 (off) or 1 (on)");
    h->deal_on = on != 0;
    h->deal_valid = false;  // the next step deals by the identity order (and rebuilds the rings)
    return MEV_OK;
}

int mev_get_step_split(const mev_handle* h, int32_t* split) {
    if (!h || !split) return fail(MEV_E_INVALID, "null argument");
    const bool fused = mev::step_kernel_for(h->sp) == 2;
    *split = fused && mev::step_esplit(h->sp) ? 2 : (fused && mev::step_split(h->sp) ? 1 : 0);
    return MEV_OK;
}

int mev_set_reset_routes(mev_handle* h, const int32_t* routes, int32_t count) {
    if (!h) return fail(MEV_E_INVALID, "null handle");
    if (count < 0 || count > h->P * h->P)
        return fail(MEV_E_INVALID, "count must be in [0, number of lane-layout routes]");
    if (count > 0 && !routes) return fail(MEV_E_INVALID, "null routes");
    for (int32_t i = 0; i < count; ++i)
        if (routes[i] < 0 || routes[i] >= h->nroutes) return fail(MEV_E_RANGE, "route id out of range");
    HIP_TRY(hipSetDevice(h->cfg.device));
    if (int r_ = serve_stop(h)) return r_;  // (the server holds the stream)
    if (count > 0) {
        HIP_TRY(hipMemcpyAsync(h->d_reset_routes, routes, size_t(count) * sizeof(int32_t), hipMemcpyHostToDevice, h->stream));
        HIP_TRY(hipStreamSynchronize(h->stream));
    }
    h->sp.n_reset_routes = count;
    return MEV_OK;
}

// ---- device snapshots: header + every state field + the last outputs, each
// field [E][bytes per env] at a 256-B aligned offset
namespace {
struct SnapField {
    uint8_t* live;     // device field (state, or the outputs the snapshot reads)
    uint8_t* restore;  // where mev_restore writes it
    size_t bpe;        // bytes per env
};
struct SnapHeader {
    uint32_t magic, version;
    int32_t E, N, K, D, R, nfields;
    uint64_t rng_counter, total_bytes;
    int32_t dims;     // SimParams::dims of the snapshot's handle (some car not 54 x 24)
    int32_t nroutes;  // its route table's size (route ids must name the same routes on restore)
    uint64_t route_hash;  // mev_handle::route_hash[nroutes]
};
constexpr uint32_t kSnapVersion = 2;  // 2: car sizes, dims flag and route count
static_assert(sizeof(SnapHeader) == 64, "snapshot header");
constexpr uint32_t kSnapMagic = 0x5356454du;  // "MEVS"

static std::vector<SnapField> snap_fields(mev_handle* h) {
    const size_t N = size_t(h->cfg.num_agents), K = size_t(h->cfg.max_npcs), D = size_t(h->D);
    std::vector<SnapField> f;
    auto add = [&](void* live, void* restore, size_t bpe) {
        if (bpe) f.push_back({static_cast<uint8_t*>(live), static_cast<uint8_t*>(restore), bpe});
    };
#define SNAP(name, dev, n, T) add(h->sp.dev, h->sp.dev, (std::string(#n) == "EN" ? N : std::string(#n) == "EK" ? K : 1) * sizeof(T));
    STATE_FIELDS(SNAP)
#undef SNAP
    add(h->sp.pending_reset, h->sp.pending_reset, 1);
    add(h->sp.ego_dim, h->sp.ego_dim, N * 2 * sizeof(float));  // car sizes (mev_set_car_dims)
    add(h->sp.npc_dim, h->sp.npc_dim, K * 2 * sizeof(float));
    const mev::Outputs& L = h->last;
    const mev::Outputs& I = h->internal;
    add(L.obs ? L.obs : I.obs, I.obs, N * D * sizeof(float));
    add(L.rew ? L.rew : I.rew, I.rew, N * sizeof(float));
    add(L.done ? L.done : I.done, I.done, N);
    add(L.status ? L.status : I.status, I.status, N);
    add(L.term ? L.term : I.term, I.term, 1);
    add(L.trunc ? L.trunc : I.trunc, I.trunc, 1);
    add(L.alive_cnt ? L.alive_cnt : I.alive_cnt, I.alive_cnt, sizeof(int32_t));
    add(L.step ? L.step : I.step, I.step, sizeof(int32_t));
    return f;
}

size_t snap_offsets(const std::vector<SnapField>& f, size_t E, std::vector<size_t>* off) {
    size_t o = sizeof(SnapHeader);
    for (const SnapField& x : f) {
        o = (o + 255) & ~size_t(255);
        if (off) off->push_back(o);
        o += x.bpe * E;
    }
    return o;
}
}  // namespace

int mev_snapshot_size(mev_handle* h, uint64_t* bytes) {
    if (!h || !bytes) return fail(MEV_E_INVALID, "null argument");
    *bytes = snap_offsets(snap_fields(h), size_t(h->cfg.num_envs), nullptr);
    return MEV_OK;
}

int mev_snapshot(mev_handle* h, void* dst, uint32_t flags) {
    if (!h || !dst) return fail(MEV_E_INVALID, "null argument");
    HIP_TRY(hipSetDevice(h->cfg.device));
    if (int r_ = serve_stop(h)) return r_;  // (the server holds the stream)
    const bool dev = (flags & MEV_DEVICE_PTRS) != 0;
    const size_t E = size_t(h->cfg.num_envs);
    if (h->last.lidar_u8) {  // compact gather row: the snapshot stores plain obs rows
        if (int r0 = sync_internal(h)) return r0;
    }
    const std::vector<SnapField> f = snap_fields(h);
    std::vector<size_t> off;
    const size_t total = snap_offsets(f, E, &off);
    SnapHeader hd{};
    hd.magic = kSnapMagic; hd.version = kSnapVersion;
    hd.dims = h->sp.dims; hd.nroutes = h->nroutes; hd.route_hash = h->route_hash[size_t(h->nroutes)];
    hd.E = h->cfg.num_envs; hd.N = h->cfg.num_agents; hd.K = h->cfg.max_npcs; hd.D = h->D; hd.R = h->cfg.lidar_rays;
    hd.nfields = int32_t(f.size()); hd.rng_counter = h->rng_counter; hd.total_bytes = total;
    uint8_t* d = static_cast<uint8_t*>(dst);
    const hipMemcpyKind kind = dev ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost;
    if (dev) HIP_TRY(hipMemcpyAsync(d, &hd, sizeof(hd), hipMemcpyHostToDevice, h->stream));
    else memcpy(d, &hd, sizeof(hd));
    for (size_t i = 0; i < f.size(); ++i) HIP_TRY(hipMemcpyAsync(d + off[i], f[i].live, f[i].bpe * E, kind, h->stream));
    // the header copy reads host memory: always wait before returning in device mode too
    HIP_TRY(hipStreamSynchronize(h->stream));
    return MEV_OK;
}

int mev_restore(mev_handle* h, const void* src, const uint8_t* env_mask, uint32_t flags) {
    if (!h || !src) return fail(MEV_E_INVALID, "null argument");
    HIP_TRY(hipSetDevice(h->cfg.device));
    if (int r_ = serve_stop(h)) return r_;  // (the server holds the stream)
    const bool dev = (flags & MEV_DEVICE_PTRS) != 0;
    const size_t E = size_t(h->cfg.num_envs);
    SnapHeader hd{};
    if (dev) {
        HIP_TRY(hipMemcpyAsync(&hd, src, sizeof(hd), hipMemcpyDeviceToHost, h->stream));
        HIP_TRY(hipStreamSynchronize(h->stream));
    } else {
        memcpy(&hd, src, sizeof(hd));
    }
    {  // validate before touching the handle: a mismatched snapshot leaves it unchanged
        const mev::Outputs save_last = h->last;
        h->last = h->internal;  // the field table of a restore (its targets are the internal buffers)
        const std::vector<SnapField> f0 = snap_fields(h);
        h->last = save_last;
        const size_t total0 = snap_offsets(f0, E, nullptr);
        if (hd.magic == kSnapMagic && hd.version == 1)  // (no car sizes, no route count / hash to check ids by)
            return fail(MEV_E_INVALID, "snapshot format 1 is no longer supported (format 2 adds car sizes and the "
                                       "route table's hash): take the snapshot again with this library");
        if (hd.magic != kSnapMagic || hd.version != kSnapVersion || hd.E != h->cfg.num_envs || hd.N != h->cfg.num_agents ||
            hd.K != h->cfg.max_npcs || hd.D != h->D || hd.nfields != int32_t(f0.size()) || hd.total_bytes != total0)
            return fail(MEV_E_INVALID, "snapshot does not match this handle");
        // the snapshot's route ids index its handle's route table (lane-layout routes, then
        // mev_add_route's): a handle with fewer routes would read past the end of its tables
        if (hd.nroutes < 0 || hd.nroutes > h->nroutes || hd.route_hash != h->route_hash[size_t(hd.nroutes)])
            return fail(MEV_E_INVALID, "snapshot's routes differ from this handle's (mev_add_route)");
        if (env_mask && f0.size() > size_t(mev::kMaxRestoreFields)) return fail(MEV_E_INVALID, "too many snapshot fields");
    }
    // the live outputs are restored into the handle's own buffers; envs a masked
    // restore leaves alone keep their current outputs, so bring those in first
    if (env_mask) {
        if (int r = sync_internal(h)) return r;
    }
    h->last = h->internal;
    h->deal_valid = false;
    const std::vector<SnapField> f = snap_fields(h);
    std::vector<size_t> off;
    const size_t total = snap_offsets(f, E, &off);
    const uint8_t* s = static_cast<const uint8_t*>(src);
    if (!env_mask) {
        const hipMemcpyKind kind = dev ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice;
        for (size_t i = 0; i < f.size(); ++i) HIP_TRY(hipMemcpyAsync(f[i].restore, s + off[i], f[i].bpe * E, kind, h->stream));
        h->rng_counter = hd.rng_counter;
        h->sp.dims = hd.dims;
    } else {
        const uint8_t* dsrc = s;
        const uint8_t* dmask = env_mask;
        if (!dev) {  // stage the snapshot and the mask on the device
            if (h->snap_stage_bytes < total) {
                if (h->d_snap_stage) {
                    HIP_TRY(hipStreamSynchronize(h->stream));
                    HIP_TRY(hipFree(h->d_snap_stage));
                    h->d_snap_stage = nullptr;
                    h->snap_stage_bytes = 0;
                }
                HIP_TRY(hipMalloc(reinterpret_cast<void**>(&h->d_snap_stage), total));
                h->snap_stage_bytes = total;
            }
            HIP_TRY(hipMemcpyAsync(h->d_snap_stage, s, total, hipMemcpyHostToDevice, h->stream));
            HIP_TRY(hipMemcpyAsync(h->d_mask, env_mask, E, hipMemcpyHostToDevice, h->stream));
            dsrc = h->d_snap_stage;
            dmask = h->d_mask;
        }
        mev::RestoreTab tab{};
        tab.n = int32_t(f.size());
        for (size_t i = 0; i < f.size(); ++i) {
            tab.dst[i] = f[i].restore;
            tab.src_off[i] = off[i];
            tab.bpe[i] = int32_t(f[i].bpe);
        }
        HIP_TRY(mev::launch_restore(tab, dsrc, dmask, h->cfg.num_envs, h->stream));
        h->sp.dims = h->sp.dims || hd.dims;  // (the sizes arrays hold valid entries either way)
    }
    if (!dev) HIP_TRY(hipStreamSynchronize(h->stream));
    return MEV_OK;
}

// ---- multi-GPU gather (include/marlenv.h) ----------------
int mev_packed_layout(int32_t slots, int32_t num_agents, int32_t obs_dim, uint64_t* offsets, uint64_t* bytes) {
    if (!offsets || !bytes) return fail(MEV_E_INVALID, "null argument");
    if (slots < 1 || num_agents < 1 || obs_dim < 1) return fail(MEV_E_INVALID, "slots, agents and obs_dim must be >= 1");
    const uint64_t C = uint64_t(slots), N = uint64_t(num_agents), D = uint64_t(obs_dim);
    const uint64_t sizes[MEV_PK_COUNT] = {C * N * D * 4, C * N * 4, C * N, C * N, C, C};
    uint64_t off = 0;
    for (int f = 0; f < MEV_PK_COUNT; ++f) {
        off = (off + 255) & ~uint64_t(255);
        offsets[f] = off;
        off += sizes[f];
    }
    *bytes = (off + 255) & ~uint64_t(255);
    return MEV_OK;
}

int mev_packed_layout2(int32_t slots, int32_t num_agents, int32_t obs_dim, int32_t lidar_slots, int32_t format,
                       uint64_t* offsets, uint64_t* bytes) {
    if (!offsets || !bytes) return fail(MEV_E_INVALID, "null argument");
    if (slots < 1 || num_agents < 1 || obs_dim < mev::OBS_HEAD || lidar_slots < 0 || lidar_slots > obs_dim - mev::OBS_HEAD)
        return fail(MEV_E_INVALID, "slots and agents must be >= 1, obs_dim >= 31, 0 <= lidar_slots <= obs_dim - 31");
    if (format != MEV_GATHER_F32 && format != MEV_GATHER_LIDAR_U8 && format != MEV_GATHER_STATE)
        return fail(MEV_E_INVALID, "unknown gather format");
    const uint64_t C = uint64_t(slots), N = uint64_t(num_agents);
    const bool codes = format != MEV_GATHER_F32, st = format == MEV_GATHER_STATE;
    const uint64_t row = st ? 0 : (codes ? uint64_t(mev::OBS_HEAD) : uint64_t(obs_dim));
    const uint64_t sizes[MEV_PK_FIELDS] = {C * N * row * 4, C * N * 4, C * N, C * N, C, C,
                                           codes ? C * N * uint64_t(lidar_slots) : 0,
                                           st ? C * N * uint64_t(mev::kStateBytesPerAgent) : 0};
    uint64_t off = 0;
    for (int f = 0; f < MEV_PK_FIELDS; ++f) {
        off = (off + 255) & ~uint64_t(255);
        offsets[f] = off;
        off += sizes[f];
    }
    *bytes = (off + 255) & ~uint64_t(255);
    return MEV_OK;
}

int mev_set_gather_format(mev_handle* h, int32_t format) {
    if (!h) return fail(MEV_E_INVALID, "null handle");
    if (format != MEV_GATHER_F32 && format != MEV_GATHER_LIDAR_U8 && format != MEV_GATHER_STATE)
        return fail(MEV_E_INVALID, "unknown gather format");
    if (h->comm) return fail(MEV_E_INVALID, "set the gather format before mev_comm_init");
    if (format != MEV_GATHER_F32 && h->sp.lidar_steps + 1 >= mev::kLidarCodeDead)
        return fail(MEV_E_INVALID, "the compact gather formats need at most 253 LiDAR march probes");
    if (format == MEV_GATHER_STATE && (h->cfg.traffic_flow || h->cfg.num_agents > 64))
        return fail(MEV_E_INVALID, "the state gather format is for handles without traffic (N <= 64)");
    h->gather_fmt = format;
    return MEV_OK;
}

int mev_lidar_decode_table(const mev_handle* h, float* table) {
    if (!h || !table) return fail(MEV_E_INVALID, "null argument");
    memcpy(table, h->h_lidar_table.data(), 256 * sizeof(float));
    return MEV_OK;
}

int mev_comm_unique_id(uint8_t* id) {
    if (!id) return fail(MEV_E_INVALID, "null argument");
    static_assert(sizeof(ncclUniqueId) == MEV_COMM_ID_BYTES, "unique id size");
    ncclUniqueId u;
    const ncclResult_t r = ncclGetUniqueId(&u);
    if (r != ncclSuccess) return fail(MEV_E_HIP, std::string("ncclGetUniqueId: ") + ncclGetErrorString(r));
    memcpy(id, &u, sizeof(u));
    return MEV_OK;
}

int mev_comm_init(mev_handle* h, const uint8_t* id, int32_t world, int32_t rank, int32_t root, int32_t slots) {
    if (!h || !id) return fail(MEV_E_INVALID, "null argument");
    if (h->comm) return fail(MEV_E_INVALID, "the handle already has a communicator");
    if (world < 1 || rank < 0 || rank >= world || root < 0 || root >= world)
        return fail(MEV_E_INVALID, "bad world / rank / root");
    if (slots <= 0) slots = h->cfg.num_envs;
    if (slots < h->cfg.num_envs) return fail(MEV_E_INVALID, "slots must be >= num_envs");
    HIP_TRY(hipSetDevice(h->cfg.device));
    if (int r_ = serve_stop(h)) return r_;  // (the server holds the stream)
    HIP_TRY(hipStreamSynchronize(h->stream));
    int rc = mev_packed_layout2(slots, h->cfg.num_agents, h->D, h->lidar_slots, h->gather_fmt, h->pk_off, &h->pk_bytes);
    if (rc) return rc;
    // the check buffer before the communicator: once ncclCommInitRank returned, every rank
    // must reach the exchange below (a rank that left early would hang its peers in it)
    constexpr int kChk = 5;  // nroutes, route hash, gather format, packed bytes, ok
    uint64_t* dchk = nullptr;
    if (world > 1) HIP_TRY(hipMalloc(reinterpret_cast<void**>(&dchk), size_t(world + 1) * kChk * sizeof(uint64_t)));
    ncclUniqueId u;
    memcpy(&u, id, sizeof(u));
    ncclComm_t comm = nullptr;
    const ncclResult_t nr = ncclCommInitRank(&comm, world, u, rank);
    if (nr != ncclSuccess) {
        if (dchk) (void)hipFree(dchk);
        return fail(MEV_E_HIP, std::string("ncclCommInitRank: ") + ncclGetErrorString(nr));
    }
    h->comm = comm;
    h->world = world; h->rank = rank; h->root = root; h->slots = slots; h->gathers = 0;
    hipError_t e = hipStreamCreateWithFlags(&h->comm_stream, hipStreamNonBlocking);
    if (world > 1) {
        // Every rank, whatever its format or local errors: the packed layout (format and
        // bytes per rank) must agree, and with the state format the route tables too (the
        // root rebuilds every rank's observation heads from route ids with ITS table:
        // mev_add_route in the same order everywhere).  Local failures travel as ok = 0, so
        // every rank returns the same verdict.
        const uint64_t mine[kChk] = {uint64_t(h->nroutes), h->route_hash[size_t(h->nroutes)], uint64_t(h->gather_fmt),
                                     uint64_t(h->pk_bytes), e == hipSuccess ? 1u : 0u};
        std::vector<uint64_t> all(size_t(world) * kChk, 0);
        hipError_t ce = hipMemcpy(dchk, mine, sizeof(mine), hipMemcpyHostToDevice);
        const ncclResult_t ar = ncclAllGather(dchk, dchk + kChk, kChk, ncclUint64, comm, h->stream);
        if (ar == ncclSuccess) {
            const hipError_t se = hipStreamSynchronize(h->stream);
            if (ce == hipSuccess) ce = se;
            if (ce == hipSuccess) ce = hipMemcpy(all.data(), dchk + kChk, all.size() * sizeof(uint64_t), hipMemcpyDeviceToHost);
        }
        (void)hipFree(dchk);
        if (ar != ncclSuccess) {
            h->free_comm();
            return fail(MEV_E_HIP, std::string("RCCL layout check: ") + ncclGetErrorString(ar));
        }
        if (ce != hipSuccess) {
            h->free_comm();
            return fail(MEV_E_HIP, std::string("layout check: ") + hipGetErrorString(ce));
        }
        for (int r = 0; r < world; ++r) {
            const uint64_t* o = &all[size_t(r) * kChk];
            const char* why = nullptr;
            if (o[4] != 1) why = "a rank failed to create its communication stream";
            else if (o[2] != mine[2] || o[3] != mine[3])
                why = "the ranks' gather layouts differ (mev_set_gather_format, num_agents, obs_dim, slots)";
            else if (h->gather_fmt == MEV_GATHER_STATE && (o[0] != mine[0] || o[1] != mine[1]))
                why = "the ranks' route tables differ (mev_add_route): the state gather format decodes every "
                      "rank's route ids with the root's table";
            if (why) {
                h->free_comm();
                return fail(MEV_E_INVALID, why);
            }
        }
    }
    const size_t per = (rank == root) ? size_t(world) * h->pk_bytes : h->pk_bytes;
    for (int b = 0; b < 2 && e == hipSuccess; ++b) {
        e = hipMalloc(reinterpret_cast<void**>(&h->pk_buf[b]), per);
        if (e == hipSuccess) e = hipMemsetAsync(h->pk_buf[b], 0, per, h->stream);  // unused slot tails stay 0
        if (e == hipSuccess) e = hipEventCreateWithFlags(&h->ev_step[b], hipEventDisableTiming);
        if (e == hipSuccess) e = hipEventCreateWithFlags(&h->ev_gather[b], hipEventDisableTiming);
    }
    if (e == hipSuccess) e = hipStreamSynchronize(h->stream);
    if (e != hipSuccess) {
        h->free_comm();
        return fail(MEV_E_NOMEM, std::string("gather buffers: ") + hipGetErrorString(e));
    }
    return MEV_OK;
}

int mev_comm_destroy(mev_handle* h) {
    if (!h) return fail(MEV_E_INVALID, "null handle");
    HIP_TRY(hipSetDevice(h->cfg.device));
    if (int r_ = serve_stop(h)) return r_;  // (the server holds the stream)
    HIP_TRY(hipStreamSynchronize(h->stream));
    if (h->comm_stream) HIP_TRY(hipStreamSynchronize(h->comm_stream));
    h->free_comm();
    return MEV_OK;
}

int mev_gather_result(mev_handle* h, void** stacked, uint64_t* bytes_per_rank, int32_t* world) {
    if (!h || !stacked || !bytes_per_rank || !world) return fail(MEV_E_INVALID, "null argument");
    if (!h->comm) return fail(MEV_E_INVALID, "no communicator (mev_comm_init)");
    if (h->rank != h->root) return fail(MEV_E_INVALID, "the gather result lives on the root rank");
    if (h->gathers == 0) return fail(MEV_E_INVALID, "no step has been gathered yet");
    HIP_TRY(hipSetDevice(h->cfg.device));
    if (int r_ = serve_stop(h)) return r_;  // (the server holds the stream)
    const int b = int((h->gathers - 1) & 1);
    if (h->gather_pending[b]) HIP_TRY(hipStreamWaitEvent(h->stream, h->ev_gather[b], 0));
    *stacked = h->pk_buf[b];
    *bytes_per_rank = h->pk_bytes;
    *world = h->world;
    return MEV_OK;
}

int mev_unpack_gathered(mev_handle* h, const void* stacked, int32_t world, float* obs) {
    if (!h || !stacked || !obs) return fail(MEV_E_INVALID, "null argument");
    if (!h->comm) return fail(MEV_E_INVALID, "no communicator (mev_comm_init): the layout is the handle's");
    if (world < 1 || world > h->world) return fail(MEV_E_INVALID, "world must be in [1, the communicator's world]");
    HIP_TRY(hipSetDevice(h->cfg.device));
    if (int r_ = serve_stop(h)) return r_;  // (the server holds the stream)
    const uint8_t* sb = static_cast<const uint8_t*>(stacked);
    const size_t C = size_t(h->slots), N = size_t(h->cfg.num_agents), D = size_t(h->D);
    const size_t rows = C * N;
    for (int r = 0; r < world; ++r) {
        const uint8_t* m = sb + size_t(r) * h->pk_bytes;
        float* o = obs + size_t(r) * rows * D;
        if (h->gather_fmt == MEV_GATHER_F32)
            HIP_TRY(hipMemcpyAsync(o, m + h->pk_off[MEV_PK_OBS], rows * D * sizeof(float), hipMemcpyDeviceToDevice,
                                   h->stream));
        else if (h->gather_fmt == MEV_GATHER_LIDAR_U8)
            HIP_TRY(mev::launch_unpack_lidar_u8(reinterpret_cast<const float*>(m + h->pk_off[MEV_PK_OBS]),
                                                m + h->pk_off[MEV_PK_LIDAR], h->d_lidar_table, o, int(rows), h->D,
                                                h->lidar_slots, h->stream));
    }
    if (h->gather_fmt == MEV_GATHER_STATE)  // one launch over every rank's envs
        HIP_TRY(mev::launch_decode_state(h->sp, sb + h->pk_off[MEV_PK_STATE], sb + h->pk_off[MEV_PK_LIDAR], h->pk_bytes,
                                         int(C), int(C) * world, h->d_lidar_table, obs, h->stream));
    return MEV_OK;
}

// A failed or stuck gather: abort the communicator (its kernels exit), then
// release the gather resources as free_comm does, without ncclCommDestroy; the
// outputs of later queries come from the handle's own buffers again.
static void abort_comm(mev_handle* h) {
    (void)ncclCommAbort(h->comm);
    h->comm = nullptr;
    if (h->last.obs != h->internal.obs) h->last = h->internal;  // h->last pointed into a packed row
    h->free_comm();
}

int mev_gather_wait(mev_handle* h, int32_t timeout_ms) {
    if (!h) return fail(MEV_E_INVALID, "null handle");
    if (!h->comm) return fail(MEV_E_INVALID, "no communicator (mev_comm_init)");
    HIP_TRY(hipSetDevice(h->cfg.device));
    if (int r_ = serve_stop(h)) return r_;  // (the server holds the stream)
    const auto t0 = std::chrono::steady_clock::now();
    for (int b = 0; b < 2; ++b) {
        if (!h->gather_pending[b]) continue;
        for (;;) {
            const hipError_t q = hipEventQuery(h->ev_gather[b]);
            if (q == hipSuccess) break;
            if (q != hipErrorNotReady) return fail(MEV_E_HIP, std::string("gather: ") + hipGetErrorString(q));
            ncclResult_t ae = ncclSuccess;
            if (ncclCommGetAsyncError(h->comm, &ae) == ncclSuccess && ae != ncclSuccess && ae != ncclInProgress) {
                abort_comm(h);
                return fail(MEV_E_HIP, std::string("RCCL gather failed: ") + ncclGetErrorString(ae));
            }
            const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
            if (timeout_ms > 0 && ms > double(timeout_ms)) {
                abort_comm(h);  // a lost peer must not hang the caller
                return fail(MEV_E_HIP, "RCCL gather timed out (communicator aborted)");
            }
            std::this_thread::sleep_for(std::chrono::microseconds(50));
        }
        h->gather_pending[b] = false;
    }
    return MEV_OK;
}

// ---- DLPack export of the internal output buffers ---------------------------
namespace {
struct DlBox {
    mev_dl_managed m;
    int64_t shape[3];
};
void dl_delete(mev_dl_managed* m) { delete reinterpret_cast<DlBox*>(m); }
}  // namespace

int mev_output_dlpack(mev_handle* h, int32_t which, mev_dl_managed** out) {
    if (!h || !out) return fail(MEV_E_INVALID, "null argument");
    const int64_t E = h->cfg.num_envs, N = h->cfg.num_agents, D = h->D;
    void* data = nullptr;
    int nd = 1;
    int64_t sh[3] = {E, 0, 0};
    mev_dl_dtype dt{1, 8, 1};  // u8
    HIP_TRY(hipSetDevice(h->cfg.device));
    if (int r_ = serve_stop(h)) return r_;  // (the server holds the stream)
    if (which != MEV_OUT_GATHERED) {
        if (int r = sync_internal(h)) return r;
    }
    const mev::Outputs& I = h->internal;
    switch (which) {
        case MEV_OUT_OBS: data = I.obs; nd = 3; sh[1] = N; sh[2] = D; dt = {2, 32, 1}; break;
        case MEV_OUT_REWARD: data = I.rew; nd = 2; sh[1] = N; dt = {2, 32, 1}; break;
        case MEV_OUT_DONE: data = I.done; nd = 2; sh[1] = N; break;
        case MEV_OUT_STATUS: data = I.status; nd = 2; sh[1] = N; break;
        case MEV_OUT_TERMINATED: data = I.term; break;
        case MEV_OUT_TRUNCATED: data = I.trunc; break;
        case MEV_OUT_AGENTS_ALIVE: data = I.alive_cnt; dt = {0, 32, 1}; break;
        case MEV_OUT_STEP: data = I.step; dt = {0, 32, 1}; break;
        case MEV_OUT_GATHERED:
            if (!h->comm || h->rank != h->root) return fail(MEV_E_INVALID, "the gather buffer lives on the root rank");
            {
                const int b = h->gathers > 0 ? int((h->gathers - 1) & 1) : 0;
                // as mev_gather_result: the handle's stream waits for the RCCL receives into it
                if (h->gather_pending[b]) HIP_TRY(hipStreamWaitEvent(h->stream, h->ev_gather[b], 0));
                data = h->pk_buf[b];
            }
            nd = 2; sh[0] = h->world; sh[1] = int64_t(h->pk_bytes);
            break;
        default: return fail(MEV_E_INVALID, "unknown output");
    }
    auto* box = new DlBox();
    for (int k = 0; k < 3; ++k) box->shape[k] = sh[k];
    mev_dl_tensor& t = box->m.dl_tensor;
    t.data = data;
    t.device = {10, h->cfg.device};  // kDLROCM
    t.ndim = nd;
    t.dtype = dt;
    t.shape = box->shape;
    t.strides = nullptr;
    t.byte_offset = 0;
    box->m.manager_ctx = nullptr;
    box->m.deleter = dl_delete;
    *out = &box->m;
    return MEV_OK;
}

int mev_npc_overflow(mev_handle* h, int64_t* count) {
    if (!h || !count) return fail(MEV_E_INVALID, "null argument");
    HIP_TRY(hipSetDevice(h->cfg.device));
    if (int r_ = serve_stop(h)) return r_;  // (the server holds the stream)
    unsigned long long v = 0;
    HIP_TRY(hipMemcpyAsync(&v, h->sp.overflow, sizeof(v), hipMemcpyDeviceToHost, h->stream));
    HIP_TRY(hipStreamSynchronize(h->stream));
    *count = int64_t(v);
    return MEV_OK;
}

int mev_npc_stats(mev_handle* h, int64_t* overflow, int64_t* sequential_turns) {
    if (!h || !overflow || !sequential_turns) return fail(MEV_E_INVALID, "null argument");
    HIP_TRY(hipSetDevice(h->cfg.device));
    if (int r_ = serve_stop(h)) return r_;  // (the server holds the stream)
    unsigned long long v[2] = {0, 0};
    HIP_TRY(hipMemcpyAsync(v, h->sp.overflow, sizeof(v), hipMemcpyDeviceToHost, h->stream));
    HIP_TRY(hipStreamSynchronize(h->stream));
    *overflow = int64_t(v[0]);
    *sequential_turns = int64_t(v[1]);
    return MEV_OK;
}

int mev_decode_errors(mev_handle* h, int64_t* count) {
    if (!h || !count) return fail(MEV_E_INVALID, "null argument");
    HIP_TRY(hipSetDevice(h->cfg.device));
    if (int r_ = serve_stop(h)) return r_;  // (the server holds the stream)
    unsigned long long v[3] = {0, 0, 0};
    HIP_TRY(hipMemcpyAsync(v, h->sp.overflow, sizeof(v), hipMemcpyDeviceToHost, h->stream));
    HIP_TRY(hipStreamSynchronize(h->stream));
    *count = int64_t(v[2]);
    return MEV_OK;
}

}  // extern "C"
