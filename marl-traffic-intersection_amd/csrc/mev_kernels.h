// mev_kernels.h — device-side data layout and kernel launchers of the
// batched intersection environment (gfx950).
//
// HBM layout (structure of arrays; env e, agent i, NPC slot k):
//   ego field f      : f[e*N + i]            (x, y, v, heading, acc, steering, prev_dist,
//                                             prev_a0, prev_a1, spawn_x/y/v/heading: f32;
//                                             path_index, route, intention: i32; alive: u8)
//   npc field f      : f[e*K + k]  K = max_npcs, live slots are a prefix of length npc_count[e]
//   per-env          : step_count, npc_count (i32), pending_reset (u8)
//   outputs          : obs[(e*N + i)*D + c] f32 (D = obs_dim), reward/done/status [e*N+i],
//                      terminated/truncated/agents_alive/step [e]
//   constant tables  : route paths [P*P][160][2] f32 (P = 8L lane points), route intent /
//                      spawn (x, y, heading) / success axis, LiDAR beam offsets [R] f32,
//                      NPC route list [M] i32
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mev {

// The 4-byte fields of each SoA live in ONE allocation, field k at base +
// k * stride (x first): kernels address them from the x pointer and the stride
// so they hold one base address in SGPRs instead of one pointer per field.
struct EgoSoA {
    float *x, *y, *v, *h, *acc, *steer, *prev_dist, *pa0, *pa1, *sx, *sy, *sv, *sh;
    int32_t *pidx, *route, *intent;
    uint8_t* alive;
    int64_t stride;  // elements between consecutive fields (>= E*N)
};
enum EgoField { EF_X, EF_Y, EF_V, EF_H, EF_ACC, EF_STEER, EF_PREV_DIST, EF_PA0, EF_PA1, EF_SX, EF_SY, EF_SV, EF_SH,
                EF_PIDX, EF_ROUTE, EF_INTENT, EF_COUNT };

struct NpcSoA {
    float *x, *y, *v, *h, *acc, *steer;
    int32_t *pidx, *route, *intent;
    uint8_t* alive;
    int32_t* count;
    int64_t stride;  // elements between consecutive fields (>= E*K)
};
enum NpcField { NF_X, NF_Y, NF_V, NF_H, NF_ACC, NF_STEER, NF_PIDX, NF_ROUTE, NF_INTENT, NF_COUNT };

struct RouteTab {
    const float* path;      // [nroutes][row][2]: plen points, the last segment, zeros (mev_world.h)
    const int32_t* intent;  // [nroutes]
    const float* spawn;     // [nroutes][3]  x, y, heading
    // [nroutes][3] bounding boxes (min x, max x, min y, max y) of each route's three
    // pieces -- points [0, 50), [50, 110), [110, plen) (RouteGen.cpp:160-237) -- for
    // the NPC ghost scan's prefilter
    const float4* pbox;
    const int32_t* len;     // [nroutes] each path's own length (Car.path.size())
    int32_t nroutes;
    int32_t plen;           // points per path in the rows (PATH_LEN, or the longest path rounded up to 16)
    int32_t row;            // points per row (plen + 16; ROUTE_PTS for plen = PATH_LEN)
    int32_t min_len;        // the shortest path's length (an index below it is inside every path)
};

struct Outputs {
    float* obs;
    float* rew;
    uint8_t* done;
    uint8_t* status;
    uint8_t* term;
    uint8_t* trunc;
    int32_t* alive_cnt;
    int32_t* step;
    // floats per observation row in `obs`: D, or OBS_HEAD when lidar_u8 is set (the
    // compact gather format: the LiDAR block goes to lidar_u8 as one code per beam,
    // [E*N][lidar_slots]: 0 = no hit (max_dist), k + 1 = hit at march probe k, 255 =
    // dead agent (0.0); decoded through mev_lidar_decode_table; padding columns
    // beyond 31 + lidar_slots are not written)
    int32_t obs_ld;
    uint8_t* lidar_u8;
    // The state gather format (MEV_GATHER_STATE; obs == nullptr, lidar_u8 set): no
    // observation head is written; instead every agent's post-step state, from which
    // the root rebuilds the head (launch_decode_state), as SoA arrays of state_n
    // elements at `state` (layout: kStateBytesPerAgent).  Agent a = e * N + i.
    uint8_t* state;
    int64_t state_n;
};
// the LiDAR code of a dead agent's beam in the compact gather formats
constexpr int kLidarCodeDead = 255;
// decode the compact format's rows: obs [n][D] from heads [n][31] and codes [n][slots]
hipError_t launch_unpack_lidar_u8(const float* head, const uint8_t* codes, const float* table, float* obs, int n,
                                  int D, int slots, hipStream_t s);
// The state format's per-agent arrays, n elements each: x, y, v, heading f32 at
// byte offsets 0, 4n, 8n, 12n; route, path index i16 at 16n, 18n; intention,
// alive u8 at 20n, 21n -- 22 bytes per agent.
constexpr int kStateBytesPerAgent = 22;
struct SimParams;
// Rebuild the float observation rows of state-format messages (no traffic): n_env
// envs, env g in message g / C (messages `stride` bytes apart), slot g % C; each
// message's state arrays (C * N elements) at state0 and LiDAR codes [C*N][lidar_slots]
// at codes0 (+ the message offset); obs [n_env][N][D] -- the rows the plain step
// writes, bit for bit (write_obs_head_tg + the decode table).
hipError_t launch_decode_state(const SimParams& p, const uint8_t* state0, const uint8_t* codes0, size_t stride, int C,
                               int n_env, const float* table, float* obs, hipStream_t s);

struct SimParams {
    int32_t E, N, R, K, D;   // envs, agents, beams, npc slots, obs_dim
    int32_t lidar_slots;     // min(R, D - 31)
    int32_t num_lanes;
    int32_t irw;             // road half width in px (L*42)
    int32_t line_stop;       // LineMask stop offset int(L*42) + 84
    float rw;                // road half width (float)
    int32_t use_team, respawn, traffic, max_steps;
    float k_prog, v_min, k_stuck, k_cv, k_co, k_succ, k_sm, alpha;
    float max_progress;      // hypot(750, 750)
    float lidar_max, lidar_step, lidar_inv;
    int32_t lidar_steps;      // S = number of march probes (dist < max_dist)
    const float* dist_tab;    // [S] accumulated probe distances, or null when dist_k == k*step exactly
    uint64_t seed;
    EgoSoA ego;
    NpcSoA npc;
    RouteTab rt;
    const float* rel_angles;  // [R]
    const int32_t* traffic_routes;  // [M] route ids
    int32_t n_traffic_routes;
    int32_t* step_count;      // [E]
    uint8_t* pending_reset;   // [E]
    unsigned long long* overflow;  // [3]: dropped spawns, sequential NPC turns (npc_phase), undecodable route ids (k_decode_state)
    unsigned long long* debug;     // diagnostic builds only (MEV_STAMPS): [E*8]
    // LiDAR hand-off k_cars -> k_lidar (L2-resident, rewritten every step)
    int4* ob_box;                  // [E][ob_stride] integer pixel AABB (x0, x1, y0, y1)
    unsigned long long* ob_cand;   // [E*N][2] candidate obstacle bits per agent
    int32_t ob_stride;             // N + max_npcs
    // route pool drawn per agent at every reset (n_reset_routes == 0: routes stay fixed)
    const int32_t* reset_routes;
    int32_t n_reset_routes;
    // step kernel choice (host side): 0 auto, 1 k_cars + k_lidar, 2 fused k_step
    int32_t step_kernel;
    // envs per fused k_step wave (host side): 0 auto, 1, 2 or 4 (reduced to fit 8 agent slots)
    int32_t step_pack;
    // two waves per fused workgroup (host side): 0 auto (<= 2048 workgroups), 1 off, 2 on
    int32_t step_split;
    // NPC-aware env deal of the fused traffic kernel (see kDealLists): per (ring, list,
    // class) counters, each on its own 128-B line, and per (ring, list, class) env orders
    int32_t* deal_cnt;    // [3][kDealLists][kDealClasses][kDealPad]
    int32_t* deal_order;  // [3][kDealLists][kDealClasses][E]: rings like the counters
    // Car sizes (Car::length / Car::width, cpp/Car.h:19-20), (length, width) per car: ego
    // [E*N][2], NPC [E*K][2] (moved with the NPCs).  Always valid: every entry is 54, 24 until
    // mev_set_car_dims.  The kernels that can run a handle with other sizes (k_cars, k_reset,
    // k_step<NM = 0>) read and keep them; dims: some car differs from 54 x 24, so the steps
    // run those kernels (the compile-time layouts assume the reference's size).  Last in the
    // struct: the other fields keep their offsets.
    float* ego_dim;
    float* npc_dim;
    int32_t dims;
    // LiDAR phase 3b culls each obstacle box to the beams its angular span covers with a
    // linear model of the offsets: rel[b] = rel[0] + b*d, d > 0, (R-1)*d <= 2*pi (every list
    // Lidar() / add_car_with_route makes with fov > 0).  0 for any other list (descending,
    // constant, uneven or wider than a revolution; a written Lidar.rel_angles): every beam
    // is then resolved against every candidate box -- the same probes, no culling.
    int32_t beam_cull;
};

// The fused traffic k_step deals envs to workgroups by their NPC count: every env
// stays in logical list x (the workgroups b with b % 8 == x, i.e. one XCD), and
// within a list the workgroups take its envs heaviest first (the i-th workgroup of
// list x, b = 8 i + x, the i-th env in descending NPC class), so that the first
// workgroups the dispatcher places -- one per SIMD -- hold the heaviest envs and
// every SIMD's four wave slots get one env from each quarter of the NPC-count
// order.  At the end of its step each env appends itself to the class list of
// step t+1 (a counter atomic per (list, class)); rings of three counter sets and
// three order sets: step t reads ring t % 3, fills ring (t+1) % 3 and clears the
// counters of ring (t+2) % 3.  (With one order set, step t's early envs would
// overwrite entries that workgroups starting later still have to read.)
constexpr int kDealLists = 8;
constexpr int kDealClasses = 8;  // NPC counts 0..6, 7 and more
constexpr int kDealPad = 32;     // ints per counter (128 B)
constexpr int kDealRingInts = kDealLists * kDealClasses * kDealPad;

struct StepInputs {
    const float* actions;      // [E*N*2]
    const int32_t* spawn_route;  // [E] or null
    float dt;
    float spawn_prob;          // 1 - expf(-density * dt) computed on host with glibc
    int32_t auto_reset;
    uint64_t rng_counter;      // handle-wide step counter (Philox counter for NPC spawns)
    // NPC-aware deal (fused traffic k_step): bit 0 take envs from ring deal_ring's
    // lists (else the XCD-aware identity order), bit 1 build ring deal_ring + 1
    int32_t deal;
    int32_t deal_ring;
};

// The kernels launch_step will use for p: 1 = k_cars + k_lidar, 2 = the fused
// k_step (one wave per env); 0 when p.step_kernel == 2 but k_step cannot run p
// (traffic mode, or a pool that does not fit a wave's LDS budget).
int step_kernel_for(const SimParams& p);
// envs per k_step wave the fused path uses for p (1, 2 or 4)
int step_pack(const SimParams& p);
// whether the fused path runs two waves per workgroup (car part / LiDAR overlap)
bool step_split(const SimParams& p);
bool step_esplit(const SimParams& p);
int esplit_pack(const SimParams& p);
// ev (nullable): three events recorded before k_cars, between k_cars and k_lidar, after k_lidar
// (with k_step: before it, and twice after it)
// dp: a device copy of p (k_step reads its parameters through it)
hipError_t launch_step(const SimParams& p, const SimParams* dp, const StepInputs& in, const Outputs& out,
                       hipStream_t s, const hipEvent_t* ev = nullptr);
hipError_t launch_reset(const SimParams& p, const uint8_t* env_mask, const Outputs& out, hipStream_t s,
                        uint64_t rng_counter);
// recompute the observation rows from the current state with LiDAR = max (after set_state)
hipError_t launch_observe_reset_lidar(const SimParams& p, const Outputs& out, hipStream_t s);

// Persistent step server (k_serve) of a small host-mode handle: the mailbox in
// host-coherent pinned memory.  A posting writes the command line's fields, then
// seq (release).  STEP carries a step number sid (a re-post after a relaunch keeps
// it); workgroup b answers done[b] = sid once its outputs are in the pinned block,
// and answers a sid it has served before with nothing.  STOP writes only cmd and
// seq.  Every workgroup publishes exited[b] = its instance's epoch when it leaves
// (STOP, or no posting for ServeArgs::idle_ticks).
constexpr int kServeMaxWG = 64;
constexpr int kServeLine = 9;  // words of the command line
constexpr uint32_t kServeStep = 1, kServeStop = 2;
struct ServeBox {
    uint32_t seq, cmd, sid;     // host -> device: posting number, kind, step number
    uint32_t dt, spawn_prob;    // f32 bits
    uint32_t auto_reset, spawn;  // spawn: spawn_route holds this step's routes
    uint32_t rng_lo, rng_hi;    // StepInputs::rng_counter
    uint32_t pad0[23];
    uint32_t done[kServeMaxWG];    // device -> host
    uint32_t exited[kServeMaxWG];  // device -> host
};
struct ServeArgs {
    ServeBox* box;               // device address of the mailbox
    const float* actions;        // device address of the pinned actions
    const int32_t* spawn_route;  // device address of the pinned spawn routes
    uint32_t epoch;
    uint32_t idle_ticks;         // 100 MHz ticks
};
// whether the handle's step can run as k_serve (fused, one workgroup per env, <= 64 envs)
bool serve_fits(const SimParams& p);
hipError_t launch_serve(const SimParams& p, const SimParams* dp, const ServeArgs& sa, const Outputs& out,
                        hipStream_t s);

// masked per-env copy of snapshot fields (mev_restore)
constexpr int kMaxRestoreFields = 48;
struct RestoreTab {
    int32_t n;
    uint8_t* dst[kMaxRestoreFields];
    unsigned long long src_off[kMaxRestoreFields];
    int32_t bpe[kMaxRestoreFields];  // bytes per env
};
hipError_t launch_restore(const RestoreTab& tab, const uint8_t* src, const uint8_t* env_mask, int E, hipStream_t s);

}  // namespace mev
