// mev_kernels.hip — the hot path: one fused step of E intersection envs on gfx950.
//
// Mapping: one 64-lane wavefront == one workgroup == one env.  Per-env state
// (<= 64 egos, <= 64 NPCs) is staged in LDS; lanes take agents for the
// per-car phases, (agent, beam) pairs for the LiDAR march, ghost-path points
// for the NPC conflict scan and car pairs for SAT collision.  The reference's
// order-dependent loops (greedy collision marking, Gauss-Seidel NPC control,
// order-preserving NPC erase) are kept exact with 64-bit lane masks
// (ballot / popcount) instead of serial loops over cars.
//
// Reference: cpp/IntersectionEnv.cpp:133-392 (step), :418-520 (observations),
// cpp/TrafficFlow.cpp:22-196, 317-367 (NPCs), cpp/Car.cpp (kinematics, SAT),
// cpp/Lidar.cpp:16-90 (ray march).  Compiled with -ffp-contract=off.
#include <type_traits>

#include <cstdlib>

#include "mev_kernels.h"
#include "mev_world.h"
#include "mev_nsort.h"

namespace mev {

constexpr int WAVE = 64;

// Diagnostic builds only, never compiled into the product library:
//  -DMEV_STAMPS: per-env phase timestamps (s_memtime) into SimParams::debug[e*8 + k]
//   (tools/phase_profile.py);
//  -DMEV_STAMPS -DMEV_STAMPS_R: a wall-clock (s_memrealtime, 100 MHz) timeline of
//   each wave -- entry, after the loads, end, and where it ran (tools/simd_balance.py);
//   MEV_STAMPS_POSTEND=1 moves slot 2 to the end of cars_post;
//  -DMEV_STAMPS_N: the NPC phase's parts (tools/npc_profile.py --parts);
//  -DMEV_EXP_STOP=n: timing-only builds stopped after part n of k_step (phase budgets,
//   tools/phase_budget.sh).
// Experiment variants measured and rejected in earlier rounds are recorded in
// DESIGN.md §9 and live in git history (before round 4), not here.
#ifdef MEV_STAMPS
#define STAMP_RAW(k)                                                     \
    do {                                                                 \
        __builtin_amdgcn_wave_barrier();                                 \
        if (threadIdx.x == 0) p.debug[e * 8 + (k)] = __builtin_amdgcn_s_memtime(); \
    } while (0)
#if defined(MEV_STAMPS_R)
#undef STAMP_RAW
#define STAMP_RAW(k)                                                     \
    do {                                                                 \
        __builtin_amdgcn_wave_barrier();                                 \
        if (threadIdx.x == 0) p.debug[e * 8 + (k)] = __builtin_amdgcn_s_memrealtime(); \
    } while (0)
#ifndef MEV_STAMPS_POSTEND  // slot 2: end of cars_pre (0) or of cars_post (1: the split kernel's car wave end)
#define MEV_STAMPS_POSTEND 0
#endif
#define STAMP(k) do { if ((k) == 0) STAMP_RAW(1); if ((k) == (MEV_STAMPS_POSTEND ? 6 : 5)) STAMP_RAW(2); } while (0)
#else
#define STAMP(k) STAMP_RAW(k)
#endif
#elif defined(MEV_STAMPS_Q)
// -DMEV_STAMPS_Q: s_memtime at eight points of the fused step kept in LDS (no global store,
// no wave barrier; lane 0 of single-wave workgroups), written to SimParams::debug[e*8 + k]
// at the end of the kernel: 0 entry, 1 loads consumed, 2 NPC phase done, 3 phase 1 done,
// 4 cars_pre done, 5 cars_post before the observation head, 6 cars_post done, 7 kernel end
// (tools/qstamp_profile.py)
__shared__ unsigned long long mev_qst[8 * 8];  // (per wave of the workgroup)
#define QSTAMP(k) do { if ((threadIdx.x & 63) == 0) mev_qst[(threadIdx.x >> 6) * 8 + (k)] = __builtin_amdgcn_s_memtime(); } while (0)
#define STAMP(k) do { if ((k) == 0) QSTAMP(1); if ((k) == 1) QSTAMP(2); if ((k) == 2) QSTAMP(3); \
                      if ((k) == 5) QSTAMP(4); if ((k) == 6) QSTAMP(6); } while (0)
#else
#define STAMP(k) do {} while (0)
#endif
#ifndef QSTAMP
#define QSTAMP(k) do {} while (0)
#endif
constexpr int MAXN = 64;
constexpr int MAXK = 64;

// k_step's issue priorities (s_setprio), falling as a wave's remaining work
// shrinks: the four waves of a SIMD start together and the hardware otherwise
// favours the oldest, so the wave with the most work left -- the one that sets
// the SIMD's finish -- would be served last.  Cars and the first quarter of
// LiDAR phase 1: 3, the rest of phase 1: 2, phase 2 (march): 1, phase 3 and the
// block writes: 0 (measured +11 % over cars 1 / LiDAR 0).  k_lidar
// (two-kernel path) runs the LiDAR phases' levels too (54.4 -> 50.7 us/step).
constexpr int kPrioCars = 3;
constexpr int kPrioLidar = 3;
constexpr int kPrioP1B = 2;  // LiDAR phase 1 after the first quarter of its agents
constexpr int kPrioP2 = 1;
constexpr int kPrioP3 = 0;

// With traffic: issue priority of the NPC controller by the NPCs an env has to
// control (level = NPCs / kNpcPrio, capped at 3).  The env with the most NPCs is
// the kernel's critical path (config 4: k_cars 53.9 -> 48.3 us).
#ifndef MEV_NPC_PRIO
#define MEV_NPC_PRIO 2
#endif
constexpr int kNpcPrio = MEV_NPC_PRIO;

// --------------------------------------------------------------- helpers ---
// A pointer the kernel reads through SimParams as a global-memory pointer.  The
// compiler cannot tell where a pointer loaded from memory points, so it would emit
// FLAT loads and stores, which count on lgkmcnt like LDS operations: every later
// s_waitcnt lgkmcnt for an LDS read would then also wait for them (a path load in
// flight could not overlap the LDS work after it).  Every array in SimParams is a
// device (global) allocation.
template <class T>
__device__ __forceinline__ __attribute__((address_space(1))) T* gmem(T* q) {
    return (__attribute__((address_space(1))) T*)q;
}
typedef float f2v __attribute__((ext_vector_type(2)));
typedef float f4v __attribute__((ext_vector_type(4)));
// float2 / float4 arrays in global memory (HIP's vector classes cannot be accessed
// through an address-space-qualified pointer; their native vector types can)
struct GF2 {
    const __attribute__((address_space(1))) f2v* q;
    __device__ __forceinline__ float2 operator[](int i) const {
        const f2v v = q[i];
        return make_float2(v.x, v.y);
    }
};
struct GF4 {
    const __attribute__((address_space(1))) f4v* q;
    __device__ __forceinline__ float4 operator[](int i) const {
        const f4v v = q[i];
        return make_float4(v.x, v.y, v.z, v.w);
    }
};
__device__ __forceinline__ GF2 gf2(const float* base) { return GF2{(const __attribute__((address_space(1))) f2v*)base}; }
__device__ __forceinline__ GF4 gf4(const float4* base) { return GF4{(const __attribute__((address_space(1))) f4v*)base}; }
// SoA field k of the ego / NPC blocks (one base pointer + stride, see EgoSoA)
__device__ inline __attribute__((address_space(1))) float* egof(const SimParams& p, int k) {
    return gmem(p.ego.x + p.ego.stride * k);
}
__device__ inline __attribute__((address_space(1))) int32_t* egoi(const SimParams& p, int k) {
    return gmem(reinterpret_cast<int32_t*>(p.ego.x + p.ego.stride * k));
}
// Element i of a global array addressed as base + 32-bit unsigned byte offset: the
// global_load saddr form (wave-uniform base in SGPRs, one offset VGPR shared by all
// the fields of an agent) instead of a 64-bit VGPR address per load.
template <class T>
__device__ __forceinline__ T ldu(const __attribute__((address_space(1))) T* base, uint32_t i) {
    typedef const __attribute__((address_space(1))) char gchar;
    return *(const __attribute__((address_space(1))) T*)((gchar*)base + i * (uint32_t)sizeof(T));
}
__device__ inline __attribute__((address_space(1))) float* npcf(const SimParams& p, int k) {
    return gmem(p.npc.x + p.npc.stride * k);
}
__device__ inline __attribute__((address_space(1))) int32_t* npci(const SimParams& p, int k) {
    return gmem(reinterpret_cast<int32_t*>(p.npc.x + p.npc.stride * k));
}
__device__ inline unsigned long long ballot(bool p) { return __ballot(p); }
// lanes below this one with their bit set in mask
__device__ inline int lane_rank(unsigned long long mask) {
    return (int)__builtin_amdgcn_mbcnt_hi((unsigned)(mask >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)mask, 0u));
}

// atan2f for wave code: the branch-free atan2f_bf unless a lane of the wave has a
// zero / infinite / NaN operand (then fdlibm's atan2f for the wave); bit-identical
// either way (mev_math.h).  The branchy form runs every range and quadrant the
// wave's lanes fall into one after another.
__device__ inline float atan2f_wave(float y, float x) {
    if (ballot(atan2f_special(y, x))) return atan2f(y, x);
    return atan2f_bf(y, x);
}

// LDS visibility between the lanes of one wave.  k_cars, k_reset and the NPC
// phase run as single-wave workgroups and k_lidar's waves are independent, so
// no s_barrier is needed -- and unlike __syncthreads() this does not wait for
// outstanding global stores.
__device__ inline void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// The same for LDS written by this wave's own ds_write instructions only (not by
// LDS DMA): one wave's LDS operations are processed in order, so a compiler
// barrier that keeps the reads after the writes is enough.
__device__ inline void wave_lds_order() {
    __builtin_amdgcn_wave_barrier();
}

// Inclusive add / max scans over the 64 lanes with DPP row shifts and row
// broadcasts (VALU only, no LDS permute round trips).  wave_scan_max assumes
// values >= 0 (0 is the identity the shifted-in lanes read).
template <class Op>
__device__ inline int wave_scan_dpp(int v, Op op) {
    v = op(v, __builtin_amdgcn_update_dpp(0, v, 0x111, 0xf, 0xf, true));  // row_shr:1
    v = op(v, __builtin_amdgcn_update_dpp(0, v, 0x112, 0xf, 0xf, true));  // row_shr:2
    v = op(v, __builtin_amdgcn_update_dpp(0, v, 0x114, 0xf, 0xf, true));  // row_shr:4
    v = op(v, __builtin_amdgcn_update_dpp(0, v, 0x118, 0xf, 0xf, true));  // row_shr:8
    v = op(v, __builtin_amdgcn_update_dpp(0, v, 0x142, 0xa, 0xf, false));  // row_bcast:15 -> rows 1, 3
    v = op(v, __builtin_amdgcn_update_dpp(0, v, 0x143, 0xc, 0xf, false));  // row_bcast:31 -> rows 2, 3
    return v;
}
// a 64-bit value of lane l (wave-uniform result)
__device__ inline unsigned long long readlane64(unsigned long long v, int l) {
    return ((unsigned long long)(unsigned)__builtin_amdgcn_readlane((int)(v >> 32), l) << 32) |
           (unsigned)__builtin_amdgcn_readlane((int)(unsigned)v, l);
}

// one DPP lane move of a float (ctrl: quad_perm / row_half_mirror ...; every lane reads a valid lane)
#define dpp_f(v, ctrl) __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), (ctrl), 0xf, 0xf, false))

__device__ inline int wave_scan_add(int v) {
    return wave_scan_dpp(v, [](int a, int b) { return a + b; });
}
__device__ inline int wave_scan_max(int v) {
    return wave_scan_dpp(v, [](int a, int b) { return a > b ? a : b; });
}

__device__ inline float wave_min(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const float w = __shfl_xor(v, o);
        v = (w < v) ? w : v;
    }
    return v;
}

// argmin over lanes of (d, i), ties -> smaller i; NaN treated as +inf.
__device__ inline int wave_argmin_first(float d, int i) {
    if (d != d) d = __builtin_inff();
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const float d2 = __shfl_xor(d, o);
        const int i2 = __shfl_xor(i, o);
        if (d2 < d || (d2 == d && i2 < i)) { d = d2; i = i2; }
    }
    return i;
}

// Philox4x32-10 (Salmon et al. 2011), counter (a, b, c, 0), key seed.
__device__ inline void philox(uint32_t c0, uint32_t c1, uint32_t c2, uint64_t seed, uint32_t* r0, uint32_t* r1) {
    uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
    uint32_t x0 = c0, x1 = c1, x2 = c2, x3 = 0x9e3779b9u;
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        const uint64_t p0 = (uint64_t)0xD2511F53u * x0;
        const uint64_t p1 = (uint64_t)0xCD9E8D57u * x2;
        const uint32_t y0 = (uint32_t)(p1 >> 32) ^ x1 ^ k0;
        const uint32_t y2 = (uint32_t)(p0 >> 32) ^ x3 ^ k1;
        x1 = (uint32_t)p1;
        x3 = (uint32_t)p0;
        x0 = y0;
        x2 = y2;
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
    *r0 = x0;
    *r1 = x1;
}

__device__ inline float u01(uint32_t r) { return (float)(r >> 8) * 0x1p-24f; }

// Route of agent i of env e at a reset: fixed (reference env.py) unless a reset
// route pool is set, then drawn uniformly per (reset, env, agent) with Philox,
// like the reference test.py's random.choice(all_routes) on every reset.
__device__ inline int reset_route(const SimParams& p, uint64_t ctr, int e, int i, int fixed) {
    if (p.n_reset_routes <= 0) return fixed;
    uint32_t r0, r1;
    philox((uint32_t)ctr, (uint32_t)(ctr >> 32) ^ 0x9E3779B9u, (uint32_t)e * 64u + (uint32_t)i, p.seed, &r0, &r1);
    return gmem(p.reset_routes)[(int)(((uint64_t)r0 * (uint32_t)p.n_reset_routes) >> 32)];
}

// dist of march probe k: the reference accumulates `dist += step_size` in
// float (Lidar.cpp:33); when that sum equals k*step exactly (checked on the
// host, e.g. step 4) we multiply, otherwise read the host-accumulated table.
// TAB: the handle's probe distances are not exactly k*step (they accumulate
// dist += step like Lidar.cpp:33), read them from the table
template <bool TAB>
__device__ inline float march_dist(const SimParams& p, int k) {
    if constexpr (TAB) return gmem(p.dist_tab)[k];
    else return (float)k * p.lidar_step;
}

// XCD-aware env order: the dispatcher deals workgroups round-robin over the 8
// XCDs (block b -> XCD b % 8), and each XCD has its own L2.  An env's SoA
// slices are 4 B x N per field (32 B at N = 8), so four consecutive envs share
// every 128-B line; mapping block b to env (b % 8) * (E / 8) + b / 8 keeps
// consecutive envs -- and their shared lines, and the partial lines between
// their observation rows -- on one XCD instead of fetching/merging them in
// four L2s.  (Placement is a performance hint only: any bijection is correct.)
__device__ inline int xcd_env(int b, int E) {
    const int q = E >> 3;
    return b < 8 * q ? (b & 7) * q + (b >> 3) : b;
}

// The env of workgroup b under the NPC-aware deal (kDealLists in mev_kernels.h):
// list x = b % 8 (the XCD the dispatcher sends b to), rank i = b / 8 in that list's
// descending NPC-class order, from the counts and orders step t - 1 built.
// (k envs per workgroup, the traffic early split (kTsplitEnvs): workgroup b takes
// ranks k (b / 8) + j, j < k, of its list; every list holds E / 8 envs whichever
// kernel built it, so any E divisible by 8 k keeps the deal a bijection)
// cls (optional): the env's NPC class in the deal, i.e. its NPC count after the previous
// step (kDealClasses - 1: that many or more)
__device__ inline int deal_env(const SimParams& p, int ring, int b, int k = 1, int j = 0, int* cls = nullptr) {
    const int x = b & (kDealLists - 1);
    int i = (b >> 3) * k + j;
    const __attribute__((address_space(1))) int32_t* cnt =
        gmem(p.deal_cnt) + (size_t)ring * kDealRingInts + x * kDealClasses * kDealPad;
    int n[kDealClasses];
#pragma unroll
    for (int c = 0; c < kDealClasses; ++c) n[c] = __builtin_amdgcn_readfirstlane(cnt[c * kDealPad]);
    int c = kDealClasses - 1;
#pragma unroll
    for (int k = kDealClasses - 1; k > 0; --k) {  // heaviest class first
        if (c == k && i >= n[k]) { i -= n[k]; c = k - 1; }
    }
    i = i < p.E - 1 ? i : p.E - 1;  // (the host keeps the rings consistent; never out of bounds)
    if (cls) *cls = c;
    const size_t ring_off = (size_t)ring * kDealLists * kDealClasses * (size_t)p.E;
    return __builtin_amdgcn_readfirstlane(gmem(p.deal_order)[ring_off + ((size_t)x * kDealClasses + c) * p.E + i]);
}

// -------------------------------------------------------- shared state ---
struct EgoLDS {
    float x[MAXN], y[MAXN], v[MAXN], h[MAXN], c[MAXN], s[MAXN];
    float cx[MAXN][4], cy[MAXN][4];
    int32_t pidx[MAXN], intent[MAXN];
    uint8_t alive[MAXN], done[MAXN], status[MAXN];
    float rew[MAXN];
    unsigned long long col[MAXN];
    uint8_t colnpc[MAXN];
};

// capacity KM NPC slots (k_cars / k_reset: MAXK; the fused k_step: the smallest
// of 32 / 64 that holds the handle's max_npcs, so that the NPC arrays leave room
// in the wave's LDS for a LiDAR pool).  DIMS: with each NPC's length / width (last).
template <int KM, bool DIMS = false>
struct NpcLDST {
    static constexpr bool kDims = DIMS;
    static constexpr int kCap = KM;
    float x[KM], y[KM], v[KM], h[KM], c[KM], s[KM], acc[KM], steer[KM];
    int32_t pidx[KM], route[KM], intent[KM];
    uint8_t alive[KM];
    union {
        struct {  // the car corners (collision phase, after the controller)
            float cx[KM][4], cy[KM][4];
        };
        struct {  // the controller's round-A states (npc_phase part 2), dead once committed
            float xn[KM], yn[KM], vn[KM], hn[KM], accn[KM], steern[KM], cn[KM], sn[KM];
            float mdcn[KM];  // the round-A state's distance to the centre
        };
    };
    unsigned long long col[KM];
    // the controller's parallel rounds: throttles of round A / B, ghost-scan candidates
    // (others that passed the filters) and which of them k must yield to, new path index
    float thr_a[KM], thr_b[KM];
    unsigned long long em[KM], ym[KM];      // this round's filtered others / yields (scans)
    unsigned long long em_a[KM], ym_a[KM];  // round A's
    float mc_a[KM];                         // round A's conflict distance (< 0: none)
    int32_t pidxn[KM];
    // the controller's per-NPC terms that depend on its own start-of-step state only
    int32_t pidx0[KM];          // after the first update_path_index of its turn
    float nsteer[KM], ntan[KM];  // Car::update's new steering angle and its tangent
    float accb[KM], mdc[KM];  // cruise throttle, distance to the centre
    float endx[KM], endy[KM];  // the route's last point (arrival test)
    // Per-NPC length / width (Car::length / Car::width), after every other array: only in
    // the kernels that can run a handle with per-car sizes (k_cars, k_reset, k_step<NM =
    // 0>); zero-length elsewhere, so the compile-time layouts keep their size
    float len[DIMS ? KM : 0], wid[DIMS ? KM : 0];
};
using NpcLDS = NpcLDST<MAXK, true>;

// the size of NPC k (the reference's constant 54 x 24 px unless the handle has cars of
// other sizes: dims)
template <class NL>
__device__ __forceinline__ float npc_len(const NL& nl, int k, bool dims) {
    if constexpr (NL::kDims) return dims ? nl.len[k] : CAR_LENGTH;
    else return CAR_LENGTH;
}
template <class NL>
__device__ __forceinline__ float npc_wid(const NL& nl, int k, bool dims) {
    if constexpr (NL::kDims) return dims ? nl.wid[k] : CAR_WIDTH;
    else return CAR_WIDTH;
}

// One NPC slot's state in the registers of lane = slot, loaded together with the
// ego state (one round of loads) and handed to npc_phase.
struct NpcRegs {
    float x, y, v, h, acc, steer;
    int32_t pidx, route, intent;
    uint8_t alive;
    float len, wid;  // (dims handles only)
};


// --------------------------------------------------- NPC traffic phase ---
// update_traffic_flow, cpp/TrafficFlow.cpp:317-367, for env e.  Egos (positions
// in LDS) are read for spawn blocking but not moved.  On return NpcLDS holds the compacted NPCs.
template <bool DIMS>
__device__ __forceinline__ NpcRegs npc_load(const SimParams& p, int e, int lane, int kload) {
    NpcRegs r{};
    if (lane < kload) {  // (kload <= K: the slots that can hold an NPC)
        const int g = e * p.K + lane;
        r.x = npcf(p, NF_X)[g]; r.y = npcf(p, NF_Y)[g]; r.v = npcf(p, NF_V)[g]; r.h = npcf(p, NF_H)[g];
        r.acc = npcf(p, NF_ACC)[g]; r.steer = npcf(p, NF_STEER)[g];
        r.pidx = npci(p, NF_PIDX)[g]; r.route = npci(p, NF_ROUTE)[g]; r.intent = npci(p, NF_INTENT)[g];
        r.alive = gmem(p.npc.alive)[g];
        if constexpr (DIMS) {
            r.len = gmem(p.npc_dim)[2 * g];
            r.wid = gmem(p.npc_dim)[2 * g + 1];
        }
    }
    return r;
}

// (d, i) pairs: the minimum d over the wave, ties to the smaller i (DPP within
// each 16-lane row, then the four row results compared as scalars); wave-uniform
__device__ inline int wave_argmin_dpp(float d, int i) {
    auto take = [&](float od, int oi) {
        if (od < d || (od == d && oi < i)) { d = od; i = oi; }
    };
    take(dpp_f(d, 0xB1), __builtin_amdgcn_mov_dpp(i, 0xB1, 0xf, 0xf, false));    // quad_perm [1,0,3,2]
    take(dpp_f(d, 0x4E), __builtin_amdgcn_mov_dpp(i, 0x4E, 0xf, 0xf, false));    // quad_perm [2,3,0,1]
    take(dpp_f(d, 0x141), __builtin_amdgcn_mov_dpp(i, 0x141, 0xf, 0xf, false));  // row_half_mirror
    take(dpp_f(d, 0x140), __builtin_amdgcn_mov_dpp(i, 0x140, 0xf, 0xf, false));  // row_mirror
    float bd = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(d), 0));
    int bi = __builtin_amdgcn_readlane(i, 0);
#pragma unroll
    for (int r = 16; r < WAVE; r += 16) {
        const float od = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(d), r));
        const int oi = __builtin_amdgcn_readlane(i, r);
        if (od < bd || (od == bd && oi < bi)) { bd = od; bi = oi; }
    }
    return bi;
}

// Diagnostic build only (-DMEV_STAMPS_N): cycles spent in each part of the NPC
// phase, accumulated over the turns and written to SimParams::debug[e*8 + part]
// (tools/npc_profile.py --parts); never compiled into the product library.
#ifdef MEV_STAMPS_N
#define NT(k)                                                                  \
    do {                                                                       \
        __builtin_amdgcn_wave_barrier();                                       \
        const unsigned long long t_ = __builtin_amdgcn_s_memtime();            \
        nt_acc[k] += t_ - nt_prev;                                             \
        nt_prev = t_;                                                          \
    } while (0)
#else
#define NT(k) do {} while (0)
#endif

// One (NPC k, other NPC j) pair of plan_npc_action_tf's longitudinal tests:
// f30 / f50 -- j is a front car closer than 30 / 50 (get_front_car_dist_tf,
// TrafficFlow.cpp:22-47, used as front < 30 / < 50 at :72-73); pok -- j passes
// the ghost-scan filters (:97-154); yfar -- k yields to j (:156-181).  k's own
// terms: pose, speed, cos/sin of its heading, distance to the centre.  The
// front-car and ghost-scan tests need only these thresholds, so a turn's plan
// is ballots over j, not reductions.
struct NpcPair {
    bool f30, f50, pok, yfar;
};
// odcj: j's distance to the centre, hypotf(oxj - 375, oyj - 375) (precomputed per NPC)
__device__ __forceinline__ NpcPair npc_pair(int k, float x, float y, float h, float v, float ck, float sk,
                                            float my_dist_to_center, bool jvalid, int j, float oxj, float oyj,
                                            float ohj, float ovj, float ocj, float osj, float odcj) {
    NpcPair r{false, false, false, false};
    const float vx = ck, vy = -sk;
    // |wrap(h - h_j)| and the distance to j: shared by the front-car test and the
    // ghost-scan filters (the same expressions in the reference, :37/:101/:107)
    const float dxj = oxj - x;
    const float dyj = oyj - y;
    const float dist_j = hypotf(dxj, dyj);
    const float adiff_j = fabs_f(wrap_angle(h - ohj));
    if (jvalid) {
        const float dist = dist_j;
        if (!(dist > 80.0f)) {
            const float dot = (dxj * vx + dyj * vy) / (dist + 1e-5f);
            if (dot > 0.8f) {
                if (adiff_j < (45.0f * PI_F / 180.0f)) { r.f30 = dist < 30.0f; r.f50 = dist < 50.0f; }
            }
        }
    }
    bool pok = false, yfar = false;
    if (jvalid) {
        const float angle_diff = adiff_j;
        pok = true;
        if (angle_diff < (60.0f * PI_F / 180.0f)) pok = false;
        if (pok) {
            const float dxo = dxj;
            const float dyo = dyj;
            const float dist_o = dist_j;
            if (dist_o > 1e-5f) {
                const float mdx = ck, mdy = -sk;
                const float two_pi_m = 2.0f * PI_F - angle_diff;
                const float adn = (two_pi_m < angle_diff) ? two_pi_m : angle_diff;
                const bool parallel = (adn < (30.0f * PI_F / 180.0f)) || (adn > (150.0f * PI_F / 180.0f));
                if (parallel) {
                    const float lon = dxo * mdx + dyo * mdy;
                    float lsq = dist_o * dist_o - lon * lon;
                    lsq = (0.0f < lsq) ? lsq : 0.0f;  // std::max(0, .)
                    const float lat = __builtin_sqrtf(lsq);
                    const bool sideways = fabs_f(lat) < (LANE_WIDTH_PX * 1.5f);
                    const bool near_lon = fabs_f(lon) < (CAR_LENGTH * 2.0f);
                    if (sideways && near_lon) {
                        const float fdist = 20.0f;
                        const float mfx = x + mdx * fdist;
                        const float mfy = y + mdy * fdist;
                        const float odx = ocj, ody = -osj;
                        const float ofx = oxj + odx * fdist;
                        const float ofy = oyj + ody * fdist;
                        const float fdx = ofx - mfx;
                        const float fdy = ofy - mfy;
                        const float fmag = hypotf(fdx, fdy);
                        if (fmag > 1e-5f) {
                            const float flon = fdx * mdx + fdy * mdy;
                            float flsq = fmag * fmag - flon * flon;
                            flsq = (0.0f < flsq) ? flsq : 0.0f;
                            const float flat = __builtin_sqrtf(flsq);
                            const float change = fabs_f(flat - lat);
                            if (change < (LANE_WIDTH_PX * 0.5f)) pok = false;  // side by side: skip
                        }
                    }
                }
            }
        }
        if (pok) {
            const float odc = odcj;
            if (v < 1.0f && ovj > 3.0f && odc < my_dist_to_center + 25.0f) yfar = true;
            else if (odc < my_dist_to_center - 5.0f) yfar = true;
            else if (fabs_f(odc - my_dist_to_center) <= 5.0f) yfar = k < j;  // address order
        }
    }
    r.pok = pok;
    r.yfar = yfar;
    return r;
}

// The ghost scan's end min(g0 + 120, path.size()) (TrafficFlow.cpp:88-89).  A row holds
// plen points, a shorter path padded with its last point, which repeats that point's
// verdict: so plen serves while g0 lies inside the path.  Past a path's end (an index
// written through set_state; the window searches keep it there) the reference's scan is
// empty.  Only an index at or beyond the table's shortest path can be there (one compare
// on every other).
__device__ __forceinline__ int npc_scan_end(const SimParams& p, int route, int g0) {
    int g1 = g0 + 120 < p.rt.plen ? g0 + 120 : p.rt.plen;
    if (__builtin_expect(g0 >= p.rt.min_len, 0)) {
        if (g0 >= gmem(p.rt.len)[route]) g1 = g0;
    }
    return g1;
}

// The ghost path scan of NPC k (:157-188) with its path points path[idx0 + lane]
// (ga) and path[idx0 + 64 + lane] (gb): the first point, in path order, within
// SAFE of an other in em (k's filtered others; lane o holds other o's position)
// that k yields to there (ym, or the point is within 15 of k) is the conflict;
// its distance to k is the minimum (:183-188).  Returns the conflict distance,
// or -1 without a conflict.
__device__ __forceinline__ float npc_ghost_scan(int g_start, int g_end, float x, float y, float2 ga, float2 gb,
                                                unsigned long long em, unsigned long long ym, float oxj, float oyj,
                                                int lane) {
    const float SAFE = CAR_WIDTH * 2.0f;
    const float SAFE_SQ = SAFE * SAFE;
#pragma unroll
    for (int c = 0; c < 2; ++c) {
        if (g_start + c * WAVE >= g_end) break;
        const float2 gp = c ? gb : ga;
        const bool gv = g_start + c * WAVE + lane < g_end;
        const float dtc = hypotf(gp.x - x, gp.y - y);
        bool hit = false;
        for (unsigned long long mm = em; mm; mm &= mm - 1ull) {
            const int o = __builtin_ctzll(mm);
            const float ox = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(oxj), o));
            const float oy = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(oyj), o));
            const float dxg = ox - gp.x;
            const float dyg = oy - gp.y;
            if (dxg * dxg + dyg * dyg < SAFE_SQ && (dtc < 15.0f || ((ym >> o) & 1ull))) hit = true;
        }
        const unsigned long long m = ballot(gv && hit);
        if (m) return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(dtc), __builtin_ctzll(m)));
    }
    return -1.0f;
}

// compose (:190-195): the longitudinal throttle after the front-car rules (acc_thr)
// and the ghost scan's conflict distance (< 0: none)
__device__ __forceinline__ float npc_throttle(float acc_thr, float min_conflict) {
    float thr = acc_thr;
    if (min_conflict >= 0.0f) {
        if (min_conflict < 35.0f) thr = -1.0f;
        else if (min_conflict < 60.0f) thr = -0.8f;
        else thr = (0.0f < thr) ? 0.0f : thr;
    }
    return thr;
}

// the surviving NPCs' state back to HBM (npc_phase's result, in nl)
template <class NL>
__device__ __forceinline__ void npc_writeback(const SimParams& p, int e, const NL& nl, int newcnt, int lane) {
    const int K = p.K;
    if (lane < newcnt) {
        const int g = e * K + lane;
        npcf(p, NF_X)[g] = nl.x[lane]; npcf(p, NF_Y)[g] = nl.y[lane]; npcf(p, NF_V)[g] = nl.v[lane]; npcf(p, NF_H)[g] = nl.h[lane];
        npcf(p, NF_ACC)[g] = nl.acc[lane]; npcf(p, NF_STEER)[g] = nl.steer[lane]; npci(p, NF_PIDX)[g] = nl.pidx[lane];
        npci(p, NF_ROUTE)[g] = nl.route[lane]; npci(p, NF_INTENT)[g] = nl.intent[lane]; gmem(p.npc.alive)[g] = 1;
        if constexpr (NL::kDims) {
            gmem(p.npc_dim)[2 * g] = nl.len[lane];
            gmem(p.npc_dim)[2 * g + 1] = nl.wid[lane];
        }
    }
    if (lane == 0) gmem(p.npc.count)[e] = newcnt;
}

// The NPC state goes back to HBM at the end of the phase (measured against a
// write-back at the end of k_step: config 4 33.1 vs 33.4 us, r3_ab_deferwb.txt).
template <class NL>
__device__ int npc_phase(const SimParams& p, const StepInputs& in, int e, int cnt, NL& nl, int lane,
                          const float* ego_x, const float* ego_y, const NpcRegs& nr) {
    const int K = p.K;
    // per-NPC sizes (Car::length / width in the SAT and the LiDAR boxes): kernels that can
    // run a handle with cars of other sizes keep them (every entry is 54 x 24 unless p.dims)
    constexpr bool dims = NL::kDims;
    const int plen = p.rt.plen;
#ifdef MEV_STAMPS_N
    unsigned long long nt_acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    unsigned long long nt_prev = __builtin_amdgcn_s_memtime();
#endif
    // state -> LDS (loaded with the ego state)
    if (lane < cnt) {
        nl.x[lane] = nr.x; nl.y[lane] = nr.y; nl.v[lane] = nr.v; nl.h[lane] = nr.h;
        nl.acc[lane] = nr.acc; nl.steer[lane] = nr.steer;
        nl.pidx[lane] = nr.pidx; nl.route[lane] = nr.route; nl.intent[lane] = nr.intent; nl.alive[lane] = nr.alive;
        if constexpr (NL::kDims) { nl.len[lane] = nr.len; nl.wid[lane] = nr.wid; }
    }
    // -- spawn (TrafficFlow.cpp:320-329, try_spawn_traffic_car :275-315)
    int r = -1;
    if (in.spawn_route) {
        r = in.spawn_route[e];
        if (r >= p.n_traffic_routes) r = -1;
    } else if (p.n_traffic_routes > 0) {
        uint32_t a0, a1;
        philox((uint32_t)in.rng_counter, (uint32_t)(in.rng_counter >> 32), (uint32_t)e, p.seed, &a0, &a1);
        if (u01(a0) < in.spawn_prob) {
            r = (int)(((uint64_t)a1 * (uint32_t)p.n_traffic_routes) >> 32);
        }
    }
    if (r >= 0) {
        const int rid = gmem(p.traffic_routes)[r];
        const float sx = gmem(p.rt.spawn)[3 * rid], sy = gmem(p.rt.spawn)[3 * rid + 1];
        const float min_dist = CAR_LENGTH * 2.5f;
        const float min_d2 = min_dist * min_dist;
        // is_spawn_blocked (:240-259): every ego (alive or not) and every NPC
        bool blk = false;
        for (int base = 0; base < p.N; base += WAVE) {
            const int i = base + lane;
            bool b = false;
            if (i < p.N) {
                const float dx = ego_x[i] - sx;
                const float dy = ego_y[i] - sy;
                b = dx * dx + dy * dy < min_d2;
            }
            blk |= ballot(b) != 0ull;
        }
        {
            bool b = false;
            if (lane < cnt) {
                const float dx = nl.x[lane] - sx;
                const float dy = nl.y[lane] - sy;
                b = dx * dx + dy * dy < min_d2;
            }
            blk |= ballot(b) != 0ull;
        }
        if (!blk) {
            if (cnt < K) {
                if (lane == 0) {
                    nl.x[cnt] = sx;
                    nl.y[cnt] = sy;
                    nl.v[cnt] = 0.0f;
                    nl.h[cnt] = gmem(p.rt.spawn)[3 * rid + 2];
                    nl.acc[cnt] = 0.0f;
                    nl.steer[cnt] = 0.0f;
                    nl.pidx[cnt] = 0;
                    nl.route[cnt] = rid;
                    nl.intent[cnt] = gmem(p.rt.intent)[rid];
                    nl.alive[cnt] = 1;
                    if constexpr (NL::kDims) { nl.len[cnt] = CAR_LENGTH; nl.wid[cnt] = CAR_WIDTH; }  // a new Car
                }
                ++cnt;
            } else if (lane == 0) {
                atomicAdd(p.overflow, 1ull);
            }
        }
    }
    wave_lds_sync();
    if (lane < cnt) {
        float s, c;
        sincosf(nl.h[lane], &s, &c);
        nl.s[lane] = s;
        nl.c[lane] = c;
    }
    wave_lds_sync();

    NT(0);  // state -> LDS, spawn
    // -- controller (:331-344): update_path_index, plan_npc_action_tf, Car::update,
    // update_path_index per NPC in vector order, each NPC planning against the
    // others' CURRENT states (Gauss-Seidel: the ones before it already moved).
    // Everything a turn needs from the NPC's own start-of-step state -- which no
    // earlier turn changes -- is computed first for all NPCs at once (part 1), and
    // the second update_path_index, which no later turn reads, after the loop
    // (part 3); the sequential loop keeps only what depends on the others.
    const float CXf = WIDTH * 0.5f, CYf = HEIGHT * 0.5f;
    const int grp = lane >> 3, sub = lane & 7;
    // path_index_update (Car.cpp:47-74) for NPCs k0 .. k0 + 7 at once (8 lanes
    // each, 8 window points per lane, first minimum wins); returns the new index
    // and leaves the 64-point window in pt
    auto npc_window = [&](int kk, int idx, float x, float y, float2* pt, int& start_i) -> int {
        const GF2 P = gf2(p.rt.path + (size_t)nl.route[kk] * (2 * p.rt.row));
        start_i = idx < 0 ? 0 : idx;
        const int wcnt = (start_i + 50 > plen) ? plen - start_i : 50;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int q = start_i + sub * 8 + j;
            pt[j] = P[q < plen ? q : plen - 1];
        }
        float bd = __builtin_inff();
        int bi = 0x7fffffff;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int off = sub * 8 + j;
            if (off < wcnt) {
                const float dx = pt[j].x - x, dy = pt[j].y - y;
                const float d = dx * dx + dy * dy;
                if (d < bd) { bd = d; bi = start_i + off; }
            }
        }
        auto take = [&](float od, int oi) {
            if (od < bd || (od == bd && oi < bi)) { bd = od; bi = oi; }
        };
        take(dpp_f(bd, 0xB1), __builtin_amdgcn_mov_dpp(bi, 0xB1, 0xf, 0xf, false));    // quad_perm [1,0,3,2]
        take(dpp_f(bd, 0x4E), __builtin_amdgcn_mov_dpp(bi, 0x4E, 0xf, 0xf, false));    // quad_perm [2,3,0,1]
        take(dpp_f(bd, 0x141), __builtin_amdgcn_mov_dpp(bi, 0x141, 0xf, 0xf, false));  // row_half_mirror
        return bi == 0x7fffffff ? start_i : bi;
    };
    // part 1: the first path index, the steering command towards path[idx + 12]
    // (:50-63) and Car::update's steering part with its tangent (Car.cpp:11-23;
    // the steering input is known before the throttle), the cruise throttle
    // (:66-70) and the distance to the centre (:83).
    for (int k0 = 0; k0 < cnt; k0 += 8) {
        const int k = k0 + grp;
        const bool act = k < cnt;
        const int kk = act ? k : 0;  // idle groups mirror NPC 0 so every lane reaches the DPP moves
        const float x = nl.x[kk], y = nl.y[kk];
        float2 pt[8];
        int start_i;
        const int pidx0 = npc_window(kk, nl.pidx[kk], x, y, pt, start_i);
        // the look-ahead point min(pidx0 + 12, plen - 1) lies in the 64-point window; an index
        // at or past the row's end (a written one) has a window of copies of path.back()
        const int tidx = pidx0 + 12 < plen - 1 ? pidx0 + 12 : plen - 1;
        const int toff = tidx < start_i ? 0 : tidx - start_i;
        if (act && sub == (toff >> 3)) {
            float2 t = pt[0];
#pragma unroll
            for (int j = 1; j < 8; ++j) t = ((toff & 7) == j) ? pt[j] : t;
            const float h = nl.h[k], v = nl.v[k];
            const float tdx = t.x - x;
            const float tdy = t.y - y;
            const float heading_err = wrap_angle(atan2f_wave(-tdy, tdx) - h);
            float steer_cmd = heading_err * 3.0f;
            steer_cmd = (1.0f < steer_cmd) ? 1.0f : steer_cmd;    // std::min(1, .)
            steer_cmd = (steer_cmd < -1.0f) ? -1.0f : steer_cmd;  // std::max(-1, .)
            const float ns = car_steer(nl.steer[k], steer_cmd);
            nl.nsteer[k] = ns;
            nl.ntan[k] = tanf(ns);
            const float target_speed = PHYSICS_MAX_SPEED * 0.4f;
            nl.accb[k] = (v < target_speed) ? 0.5f : ((v > target_speed + 1.0f) ? -0.1f : 0.0f);
            nl.mdc[k] = hypotf(x - CXf, y - CYf);
            nl.pidx0[k] = pidx0;
        }
        if (act && sub == 7) {  // the route's end point, for the arrival test after the turns
            const float2 pe = gf2(p.rt.path + (size_t)nl.route[k] * (2 * p.rt.row))[plen - 1];
            nl.endx[k] = pe.x;
            nl.endy[k] = pe.y;
        }
    }
    wave_lds_sync();
    NT(1);  // part 1
    // part 2: the turns in vector order (Gauss-Seidel: NPC k plans against the
    // others' CURRENT states -- the NPCs before it have already moved).  A turn's
    // plan is one throttle value; the steering, Car::update and the path indices
    // are k's own.  So the turns run as parallel rounds, not one after another:
    //   round A: every NPC plans against the start-of-step states (Jacobi) and moves;
    //   round B: every NPC re-plans against the round-A states of the NPCs before
    //            it and the start states of the NPCs after it.
    // If round B reproduces every round-A throttle, the round-A moves ARE the
    // sequential result (induction over k: NPC 0 has no predecessor; when NPCs < k
    // planned as in sequence, round B gave NPC k exactly its sequential inputs).
    // Otherwise the first NPC k* that differs takes its round-B throttle (its
    // inputs were right) and the NPCs after it run the sequential turns.
    const unsigned long long alive_k = ballot(lane < cnt && nl.alive[lane < cnt ? lane : 0] != 0);
    {  // the env with the most NPCs to control sets the kernel's end: serve it first
        const int lvl = __popcll(alive_k) / kNpcPrio;
        if (lvl >= 3) __builtin_amdgcn_s_setprio(3);
        else if (lvl == 2) __builtin_amdgcn_s_setprio(2);
        else if (lvl == 1) __builtin_amdgcn_s_setprio(1);
        else __builtin_amdgcn_s_setprio(0);
    }
    // NPC kk's ghost points path[idx0 + lane] and path[idx0 + 64 + lane] (clamped;
    // only indices below min(idx0 + 120, plen) are used)
    auto fetch_ghost = [&](int kk, float2& a, float2& b) {
        const GF2 P = gf2(p.rt.path + (size_t)nl.route[kk] * (2 * p.rt.row));
        const int i0 = nl.pidx0[kk] + lane, i1 = i0 + WAVE;
        a = P[i0 < plen ? i0 : plen - 1];
        b = P[i1 < plen ? i1 : plen - 1];
    };
    // the ghost points of NPC kk in the scan layout: lane t of its 16 holds
    // path[idx0 + 8t .. idx0 + 8t + 7] (clamped; only indices below min(idx0 + 120,
    // plen) are used)
    auto load_ghost8 = [&](int kk, float2* gp) {
        const GF2 P = gf2(p.rt.path + (size_t)nl.route[kk] * (2 * p.rt.row));
        const int q0 = nl.pidx0[kk] + 8 * (lane & 15);
#pragma unroll
        for (int i = 0; i < 8; ++i) gp[i] = P[q0 + i < plen ? q0 + i : plen - 1];
    };
    // plan every alive NPC (mixed: round B) into thr.  Lane = (NPC k of the chunk,
    // other j) over Kp = 8 / 16 / 32 / 64 others.  Then the ghost scans, four NPCs
    // per pass (16 lanes x 8 path points each); round B reuses round A's scan of
    // an NPC whose filtered others are the same and all come after it (unmoved).
    auto plan_all = [&](bool mixed, float* thr) {
        const int lk = cnt <= 8 ? 3 : (cnt <= 16 ? 4 : (cnt <= 32 ? 5 : 6));
        const int Kp = 1 << lk;
        const int kpc = WAVE >> lk;  // NPCs per chunk
        const int jl = lane & (Kp - 1), kl = lane >> lk;
        const unsigned long long seg = Kp == WAVE ? ~0ull : ((1ull << Kp) - 1ull);
        unsigned long long scan_m = 0ull;
#pragma nounroll
        for (int k0 = 0; k0 < cnt; k0 += kpc) {
            const int k = k0 + kl;
            const int kk = k < cnt ? k : 0;
            const bool kact = k < cnt && ((alive_k >> kk) & 1ull);
            const int j = jl;
            const int jj = j < cnt ? j : 0;
            const bool jvalid = kact && j < cnt && j != k && ((alive_k >> jj) & 1ull);
            const bool newj = mixed && j < k;  // j has moved before k's turn
            const float oxj = newj ? nl.xn[jj] : nl.x[jj], oyj = newj ? nl.yn[jj] : nl.y[jj];
            const float ohj = newj ? nl.hn[jj] : nl.h[jj], ovj = newj ? nl.vn[jj] : nl.v[jj];
            const float ocj = newj ? nl.cn[jj] : nl.c[jj], osj = newj ? nl.sn[jj] : nl.s[jj];
            const float odcj = newj ? nl.mdcn[jj] : nl.mdc[jj];
            // k's route pieces (bounding boxes), in flight during the pair tests
            const GF4 PB = gf4(p.rt.pbox + (size_t)nl.route[kk] * 3);
            const float4 pb0 = PB[0], pb1 = PB[1], pb2 = PB[2];
            const NpcPair pr = npc_pair(k, nl.x[kk], nl.y[kk], nl.h[kk], nl.v[kk], nl.c[kk], nl.s[kk], nl.mdc[kk],
                                        jvalid, j, oxj, oyj, ohj, ovj, ocj, osj, odcj);
            // prefilter of the ghost scan: j can only stop k's scan if it lies within
            // SAFE of one of k's scanned path points path[idx0, idx0 + 120); the points
            // of each route piece lie in its bounding box, so j farther than SAFE + 0.01
            // (beyond any float rounding of the squared distance) from every box the
            // scan window overlaps never hits, and leaves the scan's candidates
            bool reach = false;
            if (pr.pok) {
                const int g0 = nl.pidx0[kk], g1 = npc_scan_end(p, nl.route[kk], g0);
                const float R2 = (CAR_WIDTH * 2.0f + 0.01f) * (CAR_WIDTH * 2.0f + 0.01f);
                auto near_box = [&](float4 b) {
                    const float dx = fmaxf(fmaxf(b.x - oxj, oxj - b.y), 0.0f);
                    const float dy = fmaxf(fmaxf(b.z - oyj, oyj - b.w), 0.0f);
                    return dx * dx + dy * dy < R2;
                };
                reach = g0 < g1 && ((g0 < 50 && near_box(pb0)) || (g0 < 110 && g1 > 50 && near_box(pb1)) ||
                                    (g1 > 110 && near_box(pb2)));
            }
            const unsigned long long b30 = ballot(pr.f30), b50 = ballot(pr.f50);
            const unsigned long long bok = ballot(reach), byf = ballot(pr.yfar);
            const int sh = kl << lk;
            float acc_thr = nl.accb[kk];
            if ((b30 >> sh) & seg) acc_thr = -1.0f;
            else if ((b50 >> sh) & seg) acc_thr = (-0.2f < acc_thr) ? -0.2f : acc_thr;
            const unsigned long long em = (bok >> sh) & seg, ym = (byf >> sh) & seg;
            bool scan = em != 0ull;
            float t = acc_thr;
            if (mixed && scan) {
                const unsigned long long before = k == 0 ? 0ull : (k >= 64 ? ~0ull : (~0ull >> (64 - k)));
                if (em == nl.em_a[kk] && ym == nl.ym_a[kk] && !(em & before)) {
                    t = npc_throttle(acc_thr, nl.mc_a[kk]);  // the same scan as in round A
                    scan = false;
                }
            }
            if (kact && jl == 0) {
                thr[k] = t;
                nl.em[k] = em;
                nl.ym[k] = ym;
                if (!mixed) { nl.em_a[k] = em; nl.ym_a[k] = ym; nl.mc_a[k] = -1.0f; }
            }
            for (unsigned long long sb = ballot(kact && jl == 0 && scan); sb; sb &= sb - 1ull)
                scan_m |= 1ull << (k0 + (__builtin_ctzll(sb) >> lk));
        }
        wave_lds_sync();
        if (mixed) NT(4); else NT(2);  // the pair pass
        // ghost scans (:88-188), four NPCs per pass: NPC ks[u] on lanes u*16 ..
        // u*16 + 15, lane t of them testing path points idx0 + 8t .. idx0 + 8t + 7;
        // the first point in path order with a yielding conflict ends the scan, its
        // distance is the minimum
        const float SAFE = CAR_WIDTH * 2.0f;
        const float SAFE_SQ = SAFE * SAFE;
        // the next (up to) four NPCs of scan_m: ks, their count, this lane's NPC
        auto next_batch = [&](int* ksv, int& nbv) {
            nbv = 0;
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                ksv[u] = scan_m ? __builtin_ctzll(scan_m) : 0;
                if (scan_m) { scan_m &= scan_m - 1ull; ++nbv; }
            }
        };
        auto lane_npc = [&](const int* ksv) {
            const int u = lane >> 4;
            return u == 0 ? ksv[0] : (u == 1 ? ksv[1] : (u == 2 ? ksv[2] : ksv[3]));
        };
        int ks[4], nb = scan_m ? 1 : 0;  // (the loop picks its batch itself)
        while (nb) {
#ifdef MEV_STAMPS_N
            nt_acc[5] += 1;  // scan passes
#endif
            float2 gp[8];
            next_batch(ks, nb);
            load_ghost8(lane_npc(ks), gp);
            const int u = lane >> 4;
            const int k = lane_npc(ks);
            const bool act = u < nb;
            const int g_start = nl.pidx0[k];
            const int g_end = npc_scan_end(p, nl.route[k], g_start);
            const int q0 = g_start + 8 * (lane & 15);
            const float x = nl.x[k], y = nl.y[k];
            const unsigned long long em = act ? nl.em[k] : 0ull, ym = nl.ym[k];
            // per point: some filtered other within SAFE (near), one of them yielded to (near_y)
            unsigned near = 0u, near_y = 0u;
            for (unsigned long long mm = em; mm; mm &= mm - 1ull) {
                const int o = __builtin_ctzll(mm);
                const bool newo = mixed && o < k;
                const float ox = newo ? nl.xn[o] : nl.x[o], oy = newo ? nl.yn[o] : nl.y[o];
                const unsigned yo = (unsigned)((ym >> o) & 1ull);
#pragma unroll
                for (int i = 0; i < 8; ++i) {
                    const float dxg = ox - gp[i].x;
                    const float dyg = oy - gp[i].y;
                    const unsigned c = (q0 + i < g_end && dxg * dxg + dyg * dyg < SAFE_SQ) ? 1u : 0u;
                    near |= c << i;
                    near_y |= (c & yo) << i;
                }
            }
            // a near point is a conflict if k yields there: to a yielded-to other, or
            // to anyone when the point is within 15 of k (dist_to_crash, :158-161)
            unsigned hits = near_y;
            unsigned close = 0u, unsure = 0u;  // dist_to_crash < 15 surely / too close to 15 to tell in f32
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                const float dx = gp[i].x - x, dy = gp[i].y - y;
                const float d2 = dx * dx + dy * dy;  // within a few ulp of the double sum hypotf rounds
                close |= (d2 < 224.0f ? 1u : 0u) << i;
                unsure |= (d2 >= 224.0f && d2 <= 226.0f ? 1u : 0u) << i;
            }
            hits |= near & close;
            for (unsigned m = near & ~hits & unsure; m; m &= m - 1u) {  // exact test only near 15
                const int i = __builtin_ctz(m);
                float2 g = gp[0];
#pragma unroll
                for (int v = 1; v < 8; ++v) g = i == v ? gp[v] : g;
                if (hypotf(g.x - x, g.y - y) < 15.0f) hits |= 1u << i;
            }
            float fd = 0.0f;  // the first conflict's distance to k
            if (hits) {
                const int i = __builtin_ctz(hits);
                float2 g = gp[0];
#pragma unroll
                for (int v = 1; v < 8; ++v) g = i == v ? gp[v] : g;
                fd = hypotf(g.x - x, g.y - y);
            }
            const unsigned long long hb = ballot(act && hits != 0u);
            float mc = -1.0f;  // lane u < nb: the conflict distance of NPC ks[u]
#pragma unroll
            for (int v = 0; v < 4; ++v) {
                const unsigned sg = (unsigned)(hb >> (16 * v)) & 0xffffu;
                const float mv = sg ? __int_as_float(__builtin_amdgcn_readlane(__float_as_int(fd), 16 * v + __builtin_ctz(sg)))
                                    : -1.0f;
                mc = lane == v ? mv : mc;
            }
            wave_lds_sync();  // every lane has read this batch's LDS inputs
            if (lane < nb) {
                const int kq = lane == 0 ? ks[0] : (lane == 1 ? ks[1] : (lane == 2 ? ks[2] : ks[3]));
                thr[kq] = npc_throttle(thr[kq], mc);
                if (!mixed) nl.mc_a[kq] = mc;
            }
            wave_lds_sync();
            nb = scan_m ? 1 : 0;
        }
        NT(6);  // the ghost scans
    };
    // move the NPCs in `which` with the throttles thr into the round-A arrays
    // (xn .. sn, pidxn): Car::update with the steering from part 1 (Car.cpp:9-40)
    // and the second update_path_index (:343) over path[idx0, idx0 + 50), 8 lanes
    // per NPC (7 window points each, first minimum wins)
    auto load_window = [&](int kk, float2* w) {
        const GF2 P = gf2(p.rt.path + (size_t)nl.route[kk] * (2 * p.rt.row));
        const int pidx0 = nl.pidx0[kk];
#pragma unroll
        for (int t = 0; t < 7; ++t) {
            const int q = pidx0 + sub * 7 + t;
            w[t] = P[q < plen ? q : plen - 1];
        }
    };
    auto move_all = [&](const float* thr, unsigned long long which) {
        for (int k0 = 0; k0 < cnt; k0 += 8) {
            const int k = k0 + grp;
            const int kk = k < cnt ? k : 0;
            const bool act = k < cnt && ((which >> kk) & 1ull);
            float2 w[7];
            load_window(kk, w);
            const int pidx0 = nl.pidx0[kk];
            Kin kin{nl.x[kk], nl.y[kk], nl.v[kk], nl.h[kk], nl.acc[kk], nl.steer[kk]};
            float cn, sn;
            car_update_steered(kin, thr[kk], nl.nsteer[kk], nl.ntan[kk], in.dt, &cn, &sn);
            float bd = __builtin_inff();
            int bi = 0x7fffffff;
#pragma unroll
            for (int t = 0; t < 7; ++t) {
                const int off = sub * 7 + t;
                if (off < 50 && pidx0 + off < plen) {
                    const float wdx = w[t].x - kin.x, wdy = w[t].y - kin.y;
                    const float d = wdx * wdx + wdy * wdy;
                    if (d < bd) { bd = d; bi = pidx0 + off; }
                }
            }
            auto take = [&](float od, int oi) {
                if (od < bd || (od == bd && oi < bi)) { bd = od; bi = oi; }
            };
            take(dpp_f(bd, 0xB1), __builtin_amdgcn_mov_dpp(bi, 0xB1, 0xf, 0xf, false));    // quad_perm [1,0,3,2]
            take(dpp_f(bd, 0x4E), __builtin_amdgcn_mov_dpp(bi, 0x4E, 0xf, 0xf, false));    // quad_perm [2,3,0,1]
            take(dpp_f(bd, 0x141), __builtin_amdgcn_mov_dpp(bi, 0x141, 0xf, 0xf, false));  // row_half_mirror
            if (act && sub == 0) {
                nl.xn[k] = kin.x; nl.yn[k] = kin.y; nl.vn[k] = kin.v; nl.hn[k] = kin.h;
                nl.accn[k] = kin.acc; nl.steern[k] = kin.steer; nl.cn[k] = cn; nl.sn[k] = sn;
                nl.mdcn[k] = hypotf(kin.x - CXf, kin.y - CYf);
                nl.pidxn[k] = bi == 0x7fffffff ? (pidx0 < 0 ? 0 : pidx0) : bi;
            }
        }
        wave_lds_sync();
    };
    if (__popcll(alive_k) >= 2) {
        plan_all(false, nl.thr_a);
    } else if (lane < cnt) {
        nl.thr_a[lane] = nl.accb[lane];  // no other NPC to plan against: the cruise throttle
        wave_lds_sync();
    }
    NT(2);  // round A: plans (pairs)
    move_all(nl.thr_a, alive_k);
    NT(3);  // round A: moves
    unsigned long long done_m = alive_k;  // NPCs whose round-A move is final
    int kseq = cnt;                       // the first NPC left to the sequential turns
#if defined(MEV_EXP_NOROUNDB)  // timing-only (wrong results): round A's moves taken as final
    if (false) {
#else
    if (__popcll(alive_k) >= 2) {
#endif
        plan_all(true, nl.thr_b);
        const bool differs = lane < cnt && ((alive_k >> lane) & 1ull) &&
                             __float_as_uint(nl.thr_a[lane < cnt ? lane : 0]) !=
                                 __float_as_uint(nl.thr_b[lane < cnt ? lane : 0]);
        const unsigned long long diff = ballot(differs);
        if (diff) {
            const int ks = __builtin_ctzll(diff);
            move_all(nl.thr_b, 1ull << ks);  // its inputs were the sequential ones
            if (lane == 0) atomicAdd(p.overflow + 1, (unsigned long long)(cnt - ks - 1));  // diagnostics
            done_m = alive_k & ((ks == 63 ? ~0ull : ((2ull << ks) - 1ull)));
            kseq = ks + 1;
        }
    }
    NT(3);  // round B's re-move
    // commit the final moves
    if (lane < cnt && ((done_m >> lane) & 1ull)) {
        nl.x[lane] = nl.xn[lane]; nl.y[lane] = nl.yn[lane]; nl.v[lane] = nl.vn[lane]; nl.h[lane] = nl.hn[lane];
        nl.acc[lane] = nl.accn[lane]; nl.steer[lane] = nl.steern[lane]; nl.c[lane] = nl.cn[lane];
        nl.s[lane] = nl.sn[lane]; nl.pidx[lane] = nl.pidxn[lane];
    }
    wave_lds_sync();
    // the sequential turns after a round-B disagreement (lane j = other NPC j)
    float2 ga = make_float2(0.0f, 0.0f), gb = ga;
    if (kseq < cnt) fetch_ghost(kseq, ga, gb);
    for (int k = kseq; k < cnt; ++k) {
        float2 na = ga, nb = gb;
        if (k + 1 < cnt) fetch_ghost(k + 1, na, nb);  // in flight while NPC k is controlled
        if (nl.alive[k]) {
            const float x = nl.x[k], y = nl.y[k], h = nl.h[k], v = nl.v[k];
            const int j = lane;
            const bool jvalid = j < cnt && j != k && nl.alive[j < cnt ? j : 0];
            float oxj = 0, oyj = 0, ohj = 0, ovj = 0, ocj = 0, osj = 0;
            if (j < cnt) {
                oxj = nl.x[j]; oyj = nl.y[j]; ohj = nl.h[j]; ovj = nl.v[j]; ocj = nl.c[j]; osj = nl.s[j];
            }
            const NpcPair pr = npc_pair(k, x, y, h, v, nl.c[k], nl.s[k], nl.mdc[k], jvalid, j, oxj, oyj, ohj, ovj,
                                        ocj, osj, hypotf(oxj - CXf, oyj - CYf));
            float acc_thr = nl.accb[k];
            if (ballot(pr.f30)) acc_thr = -1.0f;
            else if (ballot(pr.f50)) acc_thr = (-0.2f < acc_thr) ? -0.2f : acc_thr;
            const unsigned long long em = ballot(pr.pok), ym = ballot(pr.yfar);
            const float mc = em ? npc_ghost_scan(nl.pidx0[k], npc_scan_end(p, nl.route[k], nl.pidx0[k]), x, y, ga, gb,
                                                 em, ym, oxj, oyj, lane)
                                : -1.0f;
            const float thr = npc_throttle(acc_thr, mc);
            Kin kin{x, y, v, h, nl.acc[k], nl.steer[k]};
            float cn, sn;
            car_update_steered(kin, thr, nl.nsteer[k], nl.ntan[k], in.dt, &cn, &sn);
            // the second update_path_index (:343) over path[idx0, idx0 + 50): lane i holds
            // path[idx0 + i] among the ghost points; no later turn reads it
            const int pidx0 = nl.pidx0[k];
            const bool wv = lane < 50 && pidx0 + lane < plen;
            const float wdx = ga.x - kin.x, wdy = ga.y - kin.y;
            const int best = wave_argmin_dpp(wv ? wdx * wdx + wdy * wdy : __builtin_inff(),
                                             wv ? pidx0 + lane : 0x7fffffff);
            const int pidx_new = best == 0x7fffffff ? (pidx0 < 0 ? 0 : pidx0) : best;
            wave_lds_sync();  // every lane has read this turn's states
            if (lane == 0) {
                nl.x[k] = kin.x; nl.y[k] = kin.y; nl.v[k] = kin.v; nl.h[k] = kin.h;
                nl.acc[k] = kin.acc; nl.steer[k] = kin.steer;
                nl.c[k] = cn; nl.s[k] = sn;
                nl.pidx[k] = pidx_new;
            }
            wave_lds_sync();
        }
        ga = na;
        gb = nb;
    }
    NT(3);  // sequential turns (with the moves)
    // -- NPC-NPC collision: greedy i<j, both removed (:347-356)
    if (lane < cnt) {
        car_corners_d(nl.x[lane], nl.y[lane], nl.c[lane], nl.s[lane], npc_len(nl, lane, dims),
                      npc_wid(nl, lane, dims), nl.cx[lane], nl.cy[lane]);
        nl.col[lane] = 0ull;
    }
    wave_lds_sync();
    unsigned long long alive_m = ballot(lane < cnt && nl.alive[lane < cnt ? lane : 0]);
    if (cnt >= 2) {  // (one NPC cannot collide)
        for (int pbase = 0; pbase < cnt * cnt; pbase += WAVE) {
            const int pi = pbase + lane;
            // (a, b) = (pi / cnt, pi % cnt); lane = 8a + b without the integer division when cnt <= 8
            const int a = cnt <= 8 ? (lane >> 3) : pi / cnt, b = cnt <= 8 ? (lane & 7) : pi % cnt;
            const int aa = a < cnt ? a : 0, bb = b < cnt ? b : 0;
            const float cdx = nl.x[aa] - nl.x[bb], cdy = nl.y[aa] - nl.y[bb];
            // circumcircles (cars_pre); cars of other sizes: every pair runs the SAT
            const bool close = !(cdx * cdx + cdy * cdy > 3600.0f) || (dims && p.dims);
            if ((cnt <= 8 ? (a < cnt && b < cnt) : pi < cnt * cnt) && a < b && close &&
                sat_collide(nl.cx[a], nl.cy[a], nl.c[a], nl.s[a], nl.cx[b], nl.cy[b], nl.c[b], nl.s[b]))
                atomicOr(&nl.col[a], 1ull << b);
        }
        wave_lds_sync();
        // greedy in (i, j) order on the masks, lane i holding col[i] (only j > i)
        const unsigned long long colv = lane < cnt ? nl.col[lane] : 0ull;
        if (ballot(colv != 0ull)) {
            for (int i = 0; i < cnt; ++i) {
                if (!((alive_m >> i) & 1ull)) continue;
                const unsigned long long hits = readlane64(colv, i) & alive_m;
                if (hits) alive_m &= ~(hits | (1ull << i));
            }
        }
    }
    // -- erase dead / arrived / out-of-screen, order preserving (:359-366)
    bool keep = false;
    if (lane < cnt && ((alive_m >> lane) & 1ull)) {
        const float gx = nl.endx[lane], gy = nl.endy[lane];
        const bool arrived = hypotf(nl.x[lane] - gx, nl.y[lane] - gy) < 20.0f;
        const float x = nl.x[lane], y = nl.y[lane];
        const float m = 100.0f;
        const bool oos = x < -m || x > float(WIDTH) + m || y < -m || y > float(HEIGHT) + m;
        keep = !arrived && !oos;
    }
    const unsigned long long keep_m = ballot(keep);
    const int newcnt = __builtin_popcountll(keep_m);
    // (most steps erase nothing: the survivors already are the prefix 0 .. cnt - 1)
    if (keep_m != (cnt >= 64 ? ~0ull : ((1ull << cnt) - 1ull))) {
        const int dst = __builtin_popcountll(keep_m & ((1ull << lane) - 1ull));
        float kx = 0, ky = 0, kv = 0, kh = 0, ka = 0, ks = 0, kc = 0, ksn = 0, kl = 0, kw = 0;
        int kp = 0, kr = 0, ki = 0;
        if (keep) {
            kx = nl.x[lane]; ky = nl.y[lane]; kv = nl.v[lane]; kh = nl.h[lane]; ka = nl.acc[lane]; ks = nl.steer[lane];
            kc = nl.c[lane]; ksn = nl.s[lane]; kp = nl.pidx[lane]; kr = nl.route[lane]; ki = nl.intent[lane];
            kl = npc_len(nl, lane, dims); kw = npc_wid(nl, lane, dims);
        }
        wave_lds_sync();
        if (keep) {
            nl.x[dst] = kx; nl.y[dst] = ky; nl.v[dst] = kv; nl.h[dst] = kh; nl.acc[dst] = ka; nl.steer[dst] = ks;
            nl.c[dst] = kc; nl.s[dst] = ksn; nl.pidx[dst] = kp; nl.route[dst] = kr; nl.intent[dst] = ki; nl.alive[dst] = 1;
            if constexpr (NL::kDims) { nl.len[dst] = kl; nl.wid[dst] = kw; }
        }
        wave_lds_sync();
    }
    // store back + corners of the survivors (for ego-NPC SAT)
    npc_writeback(p, e, nl, newcnt, lane);
    if (lane < newcnt)
        car_corners_d(nl.x[lane], nl.y[lane], nl.c[lane], nl.s[lane], npc_len(nl, lane, dims),
                      npc_wid(nl, lane, dims), nl.cx[lane], nl.cy[lane]);
    wave_lds_sync();
#ifdef MEV_STAMPS_N
    NT(7);  // collisions, erase, store
    if (lane == 0)
        for (int q = 0; q < 8; ++q) p.debug[e * 8 + q] = nt_acc[q];
#endif
    return newcnt;
}

// ---------------------------------------------------- observation rows ---
// get_observations (cpp/IntersectionEnv.cpp:418-520) minus the LiDAR block:
// ego features, path look-ahead, 5 nearest alive neighbours (egos first, then
// NPCs) in std::sort's order (:490).  The per-lane pass keeps the stable top 5,
// which is std::sort's whenever there are at most 16 candidates (libstdc++ then
// runs only its insertion sort) or no two of the nearest share a distance.
// Otherwise it writes no neighbour slot and returns true, with *dlim = the
// fifth-smallest distance, and the caller's wave runs obs_exact_neighbours for
// the agent (mev_nsort.h).  A tie among the nearest always shows as a candidate
// equal to a kept one when it arrives: of two equal candidates a (first) and b
// with d <= the final fifth distance, either a is still kept when b arrives, or a
// was pushed out by a strictly nearer one, and then the kept fifth equals d.
template <bool TRAFFIC, class EL, class NL>
__device__ __forceinline__ bool write_obs_head_tg(const SimParams& p, int i, const EL& el, const NL* nl, int ncnt, float tx,
                                  float ty, float* row, bool pad = true, float* dlim = nullptr) {
    const float x = el.x[i], y = el.y[i], v = el.v[i], h = el.h[i];
    row[0] = x / float(WIDTH);
    row[1] = y / float(HEIGHT);
    row[2] = v / PHYSICS_MAX_SPEED;
    row[3] = h / PI_F;
    const float dxd = tx - x;  // path[min(path_index + 10, 159)] (:444-452)
    const float dyd = ty - y;
    row[4] = __builtin_sqrtf(dxd * dxd + dyd * dyd) / float(WIDTH);
    row[5] = wrap_angle(atan2f(-dyd, dxd) - h) / PI_F;
    // top-5 insertion (stable)
    float bd[NEIGHBOR_COUNT];
    int bi[NEIGHBOR_COUNT];
    int nb = 0, cnt = 0;
    bool tie = false;
    const int ncand = p.N + (TRAFFIC ? ncnt : 0);
    for (int j = 0; j < ncand; ++j) {
        float ox, oy;
        if (j < p.N) {
            if (j == i || !el.alive[j]) continue;
            ox = el.x[j]; oy = el.y[j];
        } else {
            const int k = j - p.N;
            if (!nl->alive[k]) continue;
            ox = nl->x[k]; oy = nl->y[k];
        }
        ++cnt;
        const float dx = ox - x;
        const float dy = oy - y;
        const float d = __builtin_sqrtf(dx * dx + dy * dy);
        // stable insertion into the first 5 slots
        int pos = nb;
        while (pos > 0 && bd[pos - 1] > d) --pos;
        tie = tie || (pos > 0 && bd[pos - 1] == d);
        if (pos >= NEIGHBOR_COUNT) continue;
        const int last = nb < NEIGHBOR_COUNT ? nb : NEIGHBOR_COUNT - 1;
        for (int q = last; q > pos; --q) { bd[q] = bd[q - 1]; bi[q] = bi[q - 1]; }
        bd[pos] = d;
        bi[pos] = j < p.N ? j : MAXN + (j - p.N);
        if (nb < NEIGHBOR_COUNT) ++nb;
    }
    if (cnt > 16 && tie) {  // std::sort's order: obs_exact_neighbours
        *dlim = bd[NEIGHBOR_COUNT - 1];
        if (pad)
            for (int c = OBS_HEAD + p.lidar_slots; c < p.D; ++c) row[c] = 0.0f;
        return true;
    }
    for (int q = 0; q < NEIGHBOR_COUNT; ++q) {
        float* o = row + 6 + 5 * q;
        if (q < nb) {
            const int id = bi[q];
            float ox, oy, ov, oh;
            int oi;
            if (id < MAXN) { ox = el.x[id]; oy = el.y[id]; ov = el.v[id]; oh = el.h[id]; oi = el.intent[id]; }
            else { const int k = id - MAXN; ox = nl->x[k]; oy = nl->y[k]; ov = nl->v[k]; oh = nl->h[k]; oi = nl->intent[k]; }
            o[0] = (ox - x) / float(WIDTH);
            o[1] = (oy - y) / float(HEIGHT);
            o[2] = (ov - v) / PHYSICS_MAX_SPEED;
            o[3] = wrap_angle(oh - h) / PI_F;
            o[4] = float(oi);
        } else {
            o[0] = o[1] = o[2] = o[3] = o[4] = 0.0f;
        }
    }
    if (pad)
        for (int c = OBS_HEAD + p.lidar_slots; c < p.D; ++c) row[c] = 0.0f;
    return false;
}

template <bool TRAFFIC, class EL, class NL>
__device__ __forceinline__ bool write_obs_head(const SimParams& p, int i, const EL& el, const NL* nl, int ncnt,
                               const float* path, int pidx, float* row, float* dlim) {
    int tidx = pidx + 10;
    if (tidx > p.rt.plen - 1) tidx = p.rt.plen - 1;
    return write_obs_head_tg<TRAFFIC>(p, i, el, nl, ncnt, path[2 * tidx], path[2 * tidx + 1], row, true, dlim);
}

// The 64 lanes as the array of std::sort (mev_nsort.h): position q at lane q & 63 of
// d0/i0 (q < 64) or d1/i1; every index is wave-uniform, so a get is a readlane into
// SGPRs and a set one compare-and-select per register.
// TWO: positions 64 .. 127 too (more than 64 candidates possible: up to 63 other egos and
// 64 NPCs); one half otherwise (no NPCs, or one ego and <= 64 NPC slots), half the code.
template <bool TWO>
struct WaveNRefs {
    float d0, d1;
    int i0, i1;
    int lane;
    // (both registers read and written, selected by value: a field chosen by q would be
    // a pointer select, which keeps the struct out of registers)
    __device__ __forceinline__ NRef get(int q) const {
        const int l = q & (WAVE - 1);
        const float e0 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(d0), l));
        const int j0 = __builtin_amdgcn_readlane(i0, l);
        if constexpr (!TWO) return NRef{e0, j0};
        const float e1 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(d1), l));
        const int j1 = __builtin_amdgcn_readlane(i1, l);
        return q < WAVE ? NRef{e0, j0} : NRef{e1, j1};
    }
    __device__ __forceinline__ void set(int q, NRef r) {
        const bool here = lane == (q & (WAVE - 1));
        const bool h0 = TWO ? (here && q < WAVE) : here, h1 = here && q >= WAVE;
        d0 = h0 ? r.d : d0;
        i0 = h0 ? r.id : i0;
        if constexpr (TWO) {
            d1 = h1 ? r.d : d1;
            i1 = h1 ? r.id : i1;
        }
    }
};
struct WaveStack {
    int v = 0, n = 0, lane = 0;
    __device__ __forceinline__ void push(int w) { v = lane == n ? w : v; ++n; }
    __device__ __forceinline__ int pop() { --n; return __builtin_amdgcn_readlane(v, n); }
    __device__ __forceinline__ int size() const { return n; }
};

// position of the k-th (0-based) set bit of m (k < popcount(m); otherwise some bit in 0..63)
__device__ __forceinline__ int select_bit(unsigned long long m, int k) {
    int pos = 0;
#pragma unroll
    for (int w = 32; w >= 1; w >>= 1) {
        const int c = __builtin_popcountll((m >> pos) & ((1ull << w) - 1ull));
        if (c <= k) { k -= c; pos += w; }
    }
    return pos;
}

// the lexicographic minimum of (d, position) over the wave's two slots per lane; d >= +0
// (a distance), so its bit pattern orders like its value.  Returns the position.
__device__ __forceinline__ int wave_argmin_dq(float d0, float d1, bool v0, bool v1, int lane) {
    const unsigned long long k0 = v0 ? ((unsigned long long)__float_as_uint(d0) << 32) | (unsigned)lane : ~0ull;
    const unsigned long long k1 = v1 ? ((unsigned long long)__float_as_uint(d1) << 32) | (unsigned)(lane + WAVE) : ~0ull;
    unsigned long long k = k0 < k1 ? k0 : k1;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const unsigned long long w = ((unsigned long long)(unsigned)__shfl_xor((int)(k >> 32), o) << 32) |
                                     (unsigned)__shfl_xor((int)(unsigned)k, o);
        k = w < k ? w : k;
    }
    return (int)(unsigned)__builtin_amdgcn_readfirstlane((int)(unsigned)k);
}

// Ego i's neighbour slots in std::sort's order (IntersectionEnv.cpp:466-507), by the whole
// wave (every lane, wave-uniform i): the candidates in push order -- the other alive
// egos, then the alive NPCs -- compacted into the lanes, libstdc++'s partitions over
// them (ns_introsort, pruned at dlim), then the stable first five of that permutation
// (its final insertion sort).  Rare: only when write_obs_head_tg found more than 16
// candidates and an exact tie among the nearest.
template <bool TRAFFIC, bool TWO, class EL, class NL>
__device__ __forceinline__ void obs_exact_neighbours(const SimParams& p, int i, const EL& el, const NL* nl, int ncnt,
                                                  float dlim, float* row) {
    const int lane = (int)(threadIdx.x & (WAVE - 1));
    const float x = el.x[i], y = el.y[i], v = el.v[i], h = el.h[i];
    const bool ve = lane < p.N && lane != i && el.alive[lane] != 0;
    float de = 0.0f;
    if (ve) {
        const float dx = el.x[lane] - x, dy = el.y[lane] - y;
        de = __builtin_sqrtf(dx * dx + dy * dy);
    }
    bool vn = false;
    float dn = 0.0f;
    if constexpr (TRAFFIC) {
        vn = lane < ncnt && nl->alive[lane] != 0;
        if (vn) {
            const float dx = nl->x[lane] - x, dy = nl->y[lane] - y;
            dn = __builtin_sqrtf(dx * dx + dy * dy);
        }
    }
    const unsigned long long me = ballot(ve), mn = ballot(vn);
    const int ne = __builtin_popcountll(me), n = ne + __builtin_popcountll(mn);
    // position q of the push order: ego select_bit(me, q) or NPC select_bit(mn, q - ne)
    WaveNRefs<TWO> a;
    a.lane = lane;
    a.d1 = 0.0f;
    a.i1 = 0;
    {
        const int q = lane;
        const int s = q < ne ? select_bit(me, q) : select_bit(mn, q - ne);
        const float fe = __int_as_float(__builtin_amdgcn_ds_bpermute(s << 2, __float_as_int(de)));
        const float fn = __int_as_float(__builtin_amdgcn_ds_bpermute(s << 2, __float_as_int(dn)));
        a.d0 = q < ne ? fe : fn;
        a.i0 = q < ne ? s : MAXN + s;
    }
    if constexpr (TWO) {
        const int q = lane + WAVE;
        const int s = q < ne ? select_bit(me, q) : select_bit(mn, q - ne);
        const float fe = __int_as_float(__builtin_amdgcn_ds_bpermute(s << 2, __float_as_int(de)));
        const float fn = __int_as_float(__builtin_amdgcn_ds_bpermute(s << 2, __float_as_int(dn)));
        a.d1 = q < ne ? fe : fn;
        a.i1 = q < ne ? s : MAXN + s;
    }
    WaveStack st;
    st.lane = lane;
    ns_introsort(a, n, dlim, st);
    // the stable first five of the permutation: smallest (d, position), five times
    bool v0 = lane < n, v1 = TWO && lane + WAVE < n;
    int ids[NEIGHBOR_COUNT];
#pragma unroll
    for (int q = 0; q < NEIGHBOR_COUNT; ++q) {
        const int pos = wave_argmin_dq(a.d0, a.d1, v0, v1, lane);
        ids[q] = a.get(pos).id;
        v0 = v0 && pos != lane;
        v1 = v1 && pos != lane + WAVE;
    }
    int id = ids[0];
#pragma unroll
    for (int q = 1; q < NEIGHBOR_COUNT; ++q) id = lane == q ? ids[q] : id;
    if (lane < NEIGHBOR_COUNT) {  // n > 16: five neighbours (the arithmetic of write_obs_head_tg)
        float ox, oy, ov, oh;
        int oi;
        if (id < MAXN) { ox = el.x[id]; oy = el.y[id]; ov = el.v[id]; oh = el.h[id]; oi = el.intent[id]; }
        else { const int k = id - MAXN; ox = nl->x[k]; oy = nl->y[k]; ov = nl->v[k]; oh = nl->h[k]; oi = nl->intent[k]; }
        float* o = row + 6 + 5 * lane;
        o[0] = (ox - x) / float(WIDTH);
        o[1] = (oy - y) / float(HEIGHT);
        o[2] = (ov - v) / PHYSICS_MAX_SPEED;
        o[3] = wrap_angle(oh - h) / PI_F;
        o[4] = float(oi);
    }
}

// every lane of the wave: the agents whose write_obs_head_tg returned true (bit a of m:
// agent a, its fifth distance in lane a of dl, its row at rows + a * ld)
// (inlined: as a real call -- a kernel with a call sets up a stack -- configs 3 and 4 ran
// 41 us per step instead of 33 / 28, profiles/r6_ab_exact_call_cfg3.txt, _cfg4.txt)
// (TWO: more than 64 candidates possible, WaveNRefs)
template <bool TRAFFIC, bool TWO, class EL, class NL>
__device__ __forceinline__ void obs_exact_pass(const SimParams& p, unsigned long long m, float dl, const EL& el,
                                               const NL* nl, int ncnt, float* rows, size_t ld) {
    while (m) {
        const int a = __builtin_ctzll(m);
        m &= m - 1ull;
        const float dlim = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(dl), a));
        obs_exact_neighbours<TRAFFIC, TWO>(p, a, el, nl, ncnt, dlim, rows + (size_t)a * ld);
    }
}

// ------------------------------------------------------------- the step ---

// Dynamic LDS of k_cars, carved for the handle's N egos and K NPC slots.
// s_waitcnt vmcnt(0) (gfx9 encoding: expcnt and lgkmcnt left at their maximum)
constexpr int kWaitVmcnt0 = 0x0F70;
// LDS path windows of the car part's first pass (k_step, no traffic): 4 x 1 KB + 1 KB
constexpr int kWinBytes = 5 * 1024;

struct CarsLDS {
    float *x, *y, *v, *h, *c, *s, *acc, *steer, *prev_dist, *pa0, *pa1;
    float *sx, *sy, *sv, *sh, *rew, *a0, *a1, *tgx, *tgy, *t10x, *t10y;
    float4 *cx, *cy;  // corners (Car::corners order)
    int32_t *pidx, *intent, *route;
    uint8_t *alive, *done, *status, *colnpc;
    unsigned long long* col;
    int4* box;  // obstacle AABBs, integer pixels
    float *px, *py, *ph;
    unsigned long long* cand;  // [N][2]: boxes each agent's beams can reach
    // k_step only (null in k_cars): the staged observation heads [N][31], the
    // LiDAR beam offsets [R] and the env's flags (terminated, truncated,
    // agents_alive, step, pending reset, reset this step), all written to HBM
    // at the end of the kernel
    float* head;
    float* rel;
    int32_t* envw;
    // k_step without traffic (null otherwise): 5 KB for the LDS path windows of the car
    // part's first pass, inside the LiDAR pool's region (free until the LiDAR runs)
    float4* win;
    // dims handles only (null otherwise): each ego's length / width (Car::length / width)
    float *len, *wid;
};

__host__ __device__ constexpr size_t lds_al(size_t b) { return (b + 15) & ~size_t(15); }

// NPC slots that need obstacle entries in k_cars' LDS (none without traffic)
__host__ __device__ inline int cars_k(const SimParams& p) { return p.traffic ? p.K : 0; }

// dims: the handle has cars of other sizes (two more per-ego arrays at the end)
__host__ __device__ constexpr size_t cars_lds_bytes(int N, int K, bool dims = false) {
    const size_t n = (size_t)N, ob = (size_t)(N + K);
    return 22 * lds_al(n * 4) + 2 * lds_al(n * 16) + 3 * lds_al(n * 4) + 4 * lds_al(n) + lds_al(n * 8) +
           lds_al(ob * 16) + 3 * lds_al(ob * 4) + lds_al(n * 16) + (dims ? 2 * lds_al(n * 4) : 0);
}

__device__ inline CarsLDS carve_cars_lds(unsigned char* base, int N, int K, bool dims = false) {
    const size_t n = (size_t)N, ob = (size_t)(N + K);
    CarsLDS L;
    unsigned char* q = base;
    auto take = [&](size_t bytes) { unsigned char* r = q; q += lds_al(bytes); return r; };
    float** f[22] = {&L.x, &L.y, &L.v, &L.h, &L.c, &L.s, &L.acc, &L.steer, &L.prev_dist, &L.pa0, &L.pa1,
                     &L.sx, &L.sy, &L.sv, &L.sh, &L.rew, &L.a0, &L.a1, &L.tgx, &L.tgy, &L.t10x, &L.t10y};
#pragma unroll
    for (int k = 0; k < 22; ++k) *f[k] = reinterpret_cast<float*>(take(n * 4));
    L.cx = reinterpret_cast<float4*>(take(n * 16));
    L.cy = reinterpret_cast<float4*>(take(n * 16));
    L.pidx = reinterpret_cast<int32_t*>(take(n * 4));
    L.intent = reinterpret_cast<int32_t*>(take(n * 4));
    L.route = reinterpret_cast<int32_t*>(take(n * 4));
    L.alive = take(n);
    L.done = take(n);
    L.status = take(n);
    L.colnpc = take(n);
    L.col = reinterpret_cast<unsigned long long*>(take(n * 8));
    L.box = reinterpret_cast<int4*>(take(ob * 16));
    L.px = reinterpret_cast<float*>(take(ob * 4));
    L.py = reinterpret_cast<float*>(take(ob * 4));
    L.ph = reinterpret_cast<float*>(take(ob * 4));
    L.cand = reinterpret_cast<unsigned long long*>(take(n * 16));
    L.len = nullptr;
    L.wid = nullptr;
    if (dims) {
        L.len = reinterpret_cast<float*>(take(n * 4));
        L.wid = reinterpret_cast<float*>(take(n * 4));
    }
    L.head = nullptr;
    L.rel = nullptr;
    L.envw = nullptr;
    L.win = nullptr;
    return L;
}


// the final ego state of the wave's N agent slots back to HBM (lane = slot; agent
// slot i is global agent e * NE + i); spawn poses, intent, alive and route only
// for envs reset this step (do_reset: the lane's env)
__device__ __forceinline__ void ego_writeback(const SimParams& p, int e, int NE, int N, const CarsLDS& el,
                                              bool do_reset, int tid, bool dims = false) {
    for (int i = tid; i < N; i += WAVE) {
        const int g = e * NE + i;
        egof(p, EF_X)[g] = el.x[i]; egof(p, EF_Y)[g] = el.y[i]; egof(p, EF_V)[g] = el.v[i]; egof(p, EF_H)[g] = el.h[i];
        egof(p, EF_ACC)[g] = el.acc[i]; egof(p, EF_STEER)[g] = el.steer[i]; egoi(p, EF_PIDX)[g] = el.pidx[i];
        egof(p, EF_PREV_DIST)[g] = el.prev_dist[i]; egof(p, EF_PA0)[g] = el.pa0[i]; egof(p, EF_PA1)[g] = el.pa1[i];
        if (do_reset) {
            egof(p, EF_SX)[g] = el.sx[i]; egof(p, EF_SY)[g] = el.sy[i]; egof(p, EF_SV)[g] = el.sv[i]; egof(p, EF_SH)[g] = el.sh[i];
            egoi(p, EF_INTENT)[g] = el.intent[i]; gmem(p.ego.alive)[g] = el.alive[i]; egoi(p, EF_ROUTE)[g] = el.route[i];
            if (dims) {  // reset + add_car_with_route: new Cars of the default size (Car.h:19-20)
                gmem(p.ego_dim)[2 * g] = CAR_LENGTH;
                gmem(p.ego_dim)[2 * g + 1] = CAR_WIDTH;
            }
        }
    }
}

// What the two halves of the car part share (cars_pre -> cars_post).
struct CarsCtx {
    int step_no;    // step counter after this step
    bool do_reset;  // the env was auto-reset at the start of this step
    int ncnt;       // NPCs alive after the traffic phase
    bool ended;     // (set by cars_post, PK == 1) terminated or truncated this step
};

// Phase 1 of the car part for agent i of el on lane group (grp, sub): kinematics
// (IntersectionEnv.cpp:151-163), path index, base reward (:15-46), status (:165-290).
// cars_pre runs it over its agents 8 per pass; the traffic early split's LiDAR wave
// runs it for its envs' egos, one env per lane group (el then differs per group).
// (EARLY: eroute .. ga1 are the group-layout registers of the state round, see cars_pre)
template <bool EARLY, bool DIMS>
__device__ __forceinline__ void ego_phase1(const SimParams& p, const StepInputs& in, const CarsLDS& el, const int i,
                                           const bool act, const int ii, const int grp, const int sub,
                                           const unsigned long long gmask, const int eroute, const int epidx,
                                           const Kin& gk, const uint8_t galive_b, const float ga0, const float ga1) {
    constexpr bool early = EARLY;
    constexpr bool dims = DIMS;
    const int plen = p.rt.plen;
    const GF2 P = gf2(p.rt.path + (size_t)(early ? eroute : el.route[ii]) * (2 * p.rt.row));
    const int pidx0 = early ? epidx : el.pidx[ii];
    const int start_i = pidx0 < 0 ? 0 : pidx0;
    const int cnt = (start_i + 50 > plen) ? plen - start_i : 50;
    // the window's first point: start_i, or (early: the LDS window of round B)
    // start_i rounded down to even; the 50-point window and the look-ahead target
    // lie in [w0, w0 + 64): 8 points per lane
    const int w0 = early ? (start_i & ~1) : start_i;
    float2 pt[8];
    float2 pend, pprev, p10;
    if (!early) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int q = start_i + sub * 8 + j;
            pt[j] = P[q < plen ? q : plen - 1];
        }
        pend = P[plen + 1]; pprev = P[plen]; p10 = P[10];  // the row's last segment (mev_world.h)
    }
    Kin k = early ? gk : Kin{el.x[ii], el.y[ii], el.v[ii], el.h[ii], el.acc[ii], el.steer[ii]};
    const bool alive = act && (early ? galive_b : el.alive[ii]) != 0;
    const float a0_i = early ? ga0 : el.a0[ii], a1_i = early ? ga1 : el.a1[ii];
    float cH, sH;
    {
        // every lane runs the update; a dead agent keeps its state (one sincosf)
        Kin ku = k;
        car_update_heading(ku, a0_i, a1_i, in.dt);
        sincosf(alive ? ku.h : k.h, &sH, &cH);
        car_update_move(ku, cH, sH);
        if (alive) k = ku;
    }
    if (early) {  // round B's window: wait for the LDS DMA, then 4 aligned 16-B reads per lane
        __builtin_amdgcn_s_waitcnt(kWaitVmcnt0);
        const float4* wl = reinterpret_cast<const float4*>(reinterpret_cast<const char*>(el.win) + grp * 128 + sub * 16);
#pragma unroll
        for (int m = 0; m < 4; ++m) {
            const float4 q = wl[m * 64];  // + m KB
            pt[2 * m] = make_float2(q.x, q.y);
            pt[2 * m + 1] = make_float2(q.z, q.w);
        }
        // lane (grp, 0): the row's last segment (points plen, plen + 1); lane (grp, 1): points 10, 11
        const float4* wx = reinterpret_cast<const float4*>(reinterpret_cast<const char*>(el.win) + 4096 + grp * 128);
        const float4 ends = wx[0], ten = wx[1];
        pprev = make_float2(ends.x, ends.y);
        pend = make_float2(ends.z, ends.w);
        p10 = make_float2(ten.x, ten.y);
    }
    // Car::update_path_index (Car.cpp:47-74): first minimum over the window, in order
    float bd = __builtin_inff();
    int bi = 0x7fffffff;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const int q = w0 + sub * 8 + j;  // the point's path index
        if (q >= start_i && q < start_i + cnt) {
            const float dx = pt[j].x - k.x, dy = pt[j].y - k.y;
            const float d = dx * dx + dy * dy;
            if (d < bd) { bd = d; bi = q; }
        }
    }
    // minimum over the 8 lanes of the group (first index on ties): DPP swaps
    // within quads, then the mirror within each half-row (VALU, no LDS)
    auto take = [&](float od, int oi) {
        if (od < bd || (od == bd && oi < bi)) { bd = od; bi = oi; }
    };
    take(dpp_f(bd, 0xB1), __builtin_amdgcn_mov_dpp(bi, 0xB1, 0xf, 0xf, false));    // quad_perm [1,0,3,2]
    take(dpp_f(bd, 0x4E), __builtin_amdgcn_mov_dpp(bi, 0x4E, 0xf, 0xf, false));    // quad_perm [2,3,0,1]
    take(dpp_f(bd, 0x141), __builtin_amdgcn_mov_dpp(bi, 0x141, 0xf, 0xf, false));  // row_half_mirror
    const int pidx = alive ? (bi == 0x7fffffff ? start_i : bi) : pidx0;
    // look-ahead point of the observation (:444-452), picked from the window
    {
        const int tidx = pidx + 10 < plen - 1 ? pidx + 10 : plen - 1;
        const int toff = tidx - w0;
        if (act && toff >= 0 && toff < 64 && sub == (toff >> 3)) {
            float2 t = pt[0];
#pragma unroll
            for (int j = 1; j < 8; ++j) t = ((toff & 7) == j) ? pt[j] : t;
            el.tgx[i] = t.x;
            el.tgy[i] = t.y;
        } else if (act && (toff < 0 || toff >= 64) && sub == 0) {
            el.tgx[i] = P[tidx].x;
            el.tgy[i] = P[tidx].y;
        }
    }
    float rew = 0.0f, cur = 0.0f, an = 0.0f, sn = 0.0f;
    bool succ = false;
    float ccx[4], ccy[4];
    car_corners_d(k.x, k.y, cH, sH, (dims ? el.len[ii] : CAR_LENGTH), (dims ? el.wid[ii] : CAR_WIDTH), ccx, ccy);
    {  // (branch-free: every lane evaluates the terms, a dead agent's are zeroed)
        // compute_progress / compute_stuck / compute_smooth (:15-46)
        cur = hypotf(k.x - pend.x, k.y - pend.y);
        const float prev = el.prev_dist[ii];
        float r_prog = 0.0f;
        if (prev > 0.0f) {
            const float progress = prev - cur;
            const float normalized = (p.max_progress > 0.0f) ? (progress / p.max_progress) : 0.0f;
            r_prog = p.k_prog * normalized;
        }
        const float speed_ms = (k.v * FPS) / SCALE;
        const float r_stuck = (speed_ms < p.v_min) ? p.k_stuck : 0.0f;
        an = k.acc / MAX_ACC;
        sn = k.steer / MAX_STEERING_ANGLE;
        const float d0 = an - el.pa0[ii];
        const float d1 = sn - el.pa1[ii];
        const float r_smooth = p.k_sm * (d0 * d0 + d1 * d1);
        rew = r_prog + r_stuck + r_smooth;
        // SUCCESS by the last path segment's axis
        const float dxr = pend.x - pprev.x, dyr = pend.y - pprev.y;
        const bool sx_ = fabs_f(k.y - pend.y) < 15.0f && fabs_f(k.x - pend.x) < 40.0f;
        const bool sy_ = fabs_f(k.x - pend.x) < 15.0f && fabs_f(k.y - pend.y) < 40.0f;
        succ = fabs_f(dxr) > fabs_f(dyr) ? sx_ : sy_;
        if (!alive) { rew = 0.0f; cur = 0.0f; an = 0.0f; sn = 0.0f; succ = false; }
    }
    // corner tests, one per lane: sub 0-3 corner q (screen margin, road, yellow line,
    // line mask), sub 4-7 edge midpoint q (line mask)
    bool oos_q = false, off_q = false, line_q = false;
    {
        // lane sub < 4: corner q (screen margin, road, yellow line, line mask);
        // sub >= 4: the midpoint of edge (q, q + 1) (line mask only)
        const int q = sub & 3;
        float qx = ccx[0], qy = ccy[0], rx = ccx[1], ry = ccy[1];
#pragma unroll
        for (int u = 1; u < 4; ++u) {
            if (q == u) { qx = ccx[u]; qy = ccy[u]; rx = ccx[(u + 1) & 3]; ry = ccy[(u + 1) & 3]; }
        }
        const bool corner = sub < 4;
        const float px_ = corner ? qx : 0.5f * (qx + rx), py_ = corner ? qy : 0.5f * (qy + ry);
        const float M = 100.0f;
        const bool lm = is_line_px((int)px_, (int)py_, p.line_stop);
        oos_q = alive && corner && (qx < -M || qx > float(WIDTH) + M || qy < -M || qy > float(HEIGHT) + M);
        off_q = alive && corner && !is_on_road(qx, qy, p.rw);
        line_q = alive && ((corner && hits_yellow_line(qx, qy, p.rw)) || lm);
    }
    const bool any_oos = (ballot(oos_q) & gmask) != 0ull;
    const bool any_off = (ballot(off_q) & gmask) != 0ull;
    const bool any_line = (ballot(line_q) & gmask) != 0ull;
    if (act) {
        if (sub < 4) {
            reinterpret_cast<float*>(&el.cx[i])[sub] = ccx[sub];
            reinterpret_cast<float*>(&el.cy[i])[sub] = ccy[sub];
        }
        if (sub == 0) {
            uint8_t done = 0, status = ST_ALIVE;
            if (!alive) { done = 1; status = ST_DEAD; }
            else if (succ) { done = 1; status = ST_SUCCESS; }
            else if (any_oos || any_off) { done = 1; status = ST_CRASH_WALL; }
            else if (any_line) { done = 1; status = ST_CRASH_LINE; }
            el.x[i] = k.x; el.y[i] = k.y; el.v[i] = k.v; el.h[i] = k.h; el.c[i] = cH; el.s[i] = sH;
            el.acc[i] = k.acc; el.steer[i] = k.steer; el.pidx[i] = pidx;
            if (alive) { el.prev_dist[i] = cur; el.pa0[i] = an; el.pa1[i] = sn; }
            el.t10x[i] = p10.x; el.t10y[i] = p10.y;
            el.done[i] = done; el.status[i] = status; el.rew[i] = rew;
            el.col[i] = 0ull; el.colnpc[i] = 0;
        }
    }
}

// The per-env body of the step before the LiDAR (k_cars, or the first part of
// k_step): el and nl are this wave's LDS.  Only what the LiDAR needs runs
// here -- kinematics, status, car-car resolution, respawn, the obstacle table
// and candidate masks; the rest (bonuses, team mix, flags, the state
// write-back and the observation head) is cars_post, which k_step runs after
// the LiDAR so that its latency-bound chain overlaps other waves' LiDAR
// instead of delaying this wave's.  FUSED: the LiDAR runs in the same wave
// (k_step) and reads the obstacle table and candidate masks from LDS, so they
// are not published to HBM.
// ESPLIT (k_step's early split, one env per two-wave workgroup): the LiDAR wave
// computes the poses after the kinematics itself and marches the road while this
// wave runs the car part; this wave leaves the beam offsets (el.rel) to it, records
// the respawned egos (el.envw[6]) at the end and passes workgroup barrier B.
// EARLY: phase 1's first path windows come by LDS DMA from group-layout route /
// index registers loaded in the state round (k_step without traffic).
// DIMS: the kernel can run a handle whose cars have other sizes than 54 x 24 px
// (k_cars, k_step<NM = 0>); p.dims then says whether this one does, and the car
// corners, the SAT pre-test and the LiDAR boxes take each car's length / width.
// TSC (the traffic early split's car waves, one ego per env): the workgroup's LiDAR wave
// loads the ego into this env's LDS and runs its phase 1 (ts_ego_phase) while this wave
// runs the NPC phase; the two meet at workgroup barrier H, then this wave goes on from the
// SAT.  The NPC phase's spawn test reads the ego's start-of-step position, which this wave
// keeps in envw[0..1] (the LiDAR wave overwrites el.x / el.y with the moved pose).
template <bool TRAFFIC, bool FUSED, class NL, int PK = 1, bool EARLY = false, bool ESPLIT = false, bool DIMS = false,
          bool TSC = false, int NC = 0>
__device__ __forceinline__ CarsCtx cars_pre(const SimParams& p, const StepInputs& in, const Outputs& out, const int e,
                                            const CarsLDS& el, NL* nl, int npc_cls = kDealClasses - 1) {
    static_assert(!ESPLIT || FUSED, "early split: k_step");
    static_assert(PK == 1 || (FUSED && !TRAFFIC), "several envs per wave: k_step without traffic");
    static_assert(!DIMS || (PK == 1 && !EARLY && !ESPLIT), "per-car sizes: the runtime-layout kernels");
    static_assert(!TRAFFIC || NL::kDims == DIMS, "NPC sizes in LDS exactly when the kernel handles them");
    // (a DIMS kernel keeps every car's size: all 54 x 24 unless p.dims; p.dims alone turns
    // off the SAT's circumcircle pre-test, which assumes that size)
    constexpr bool dims = DIMS;
    const bool all_pairs = DIMS && p.dims;
    // One wave per env: the order-dependent per-env logic (NPCs, kinematics,
    // status, collisions, respawn, observation head); the LiDAR block of the
    // observation is filled by the LiDAR body right after.  Per-agent phases run on
    // groups of 8 lanes per agent (8 agents per pass) so the window search,
    // the corner tests and the neighbour ranking are lane-parallel; global
    // memory is touched in two dependent rounds (state, then route table) and
    // written once at the end.
    const int tid = threadIdx.x & (WAVE - 1);
    const int NE = NC ? NC : p.N;  // agents per env (NC: the kernel's compile-time count)
    // PK > 1 (k_step, few agents per env): the wave steps envs e .. e + npk - 1;
    // agent slot i is agent i % NE of env e + i / NE, global agent e * NE + i
    // (consecutive envs are consecutive in the SoA).  N: the wave's agent slots.
    const int npk = PK == 1 ? 1 : (p.E - e < PK ? p.E - e : PK);
    const int N = PK == 1 ? NE : npk * NE;

    // ---- phase 0: ego state -> LDS (lane = agent).  An env whose previous
    // step ended starts from its spawns (vector auto-reset; reset +
    // add_car_with_route, :66-131).
    // Round A: every load the car part needs before its path window -- the env
    // flags, the actions, every state field, the LiDAR beam offsets and (first
    // pass of phase 1) each lane group's route and path index -- is issued back to
    // back and unconditionally (no load waits behind a branch on another load's
    // value); only an env being reset waits a second round for its spawn poses.
    // Then the path windows of phase 1's first pass are issued straight from the
    // group-layout route / index registers (round B), while the state goes
    // through LDS.  (Before: the flags, the actions, the state and the path window
    // were four dependent rounds.)
    const int ee = PK == 1 ? e : e + (tid < N ? tid : 0) / NE;  // the lane's env (lane = agent slot)
    const bool lane_on = tid < N;  // N <= 64: one agent slot per lane
    const int il = lane_on ? tid : 0;
    const int gl = e * NE + il;
    const uint32_t ug = (uint32_t)gl;
    const uint8_t pending_b = ldu(gmem(p.pending_reset), (uint32_t)ee);
    const int step_prev = ldu(gmem(p.step_count), (uint32_t)ee);
    const int npcs_prev = TRAFFIC ? gmem(p.npc.count)[e] : 0;
    const float a0 = ldu(gmem(in.actions), 2 * ug), a1 = ldu(gmem(in.actions), 2 * ug + 1);
    const int route_l = ldu(egoi(p, EF_ROUTE), ug);
    const float x0 = ldu(egof(p, EF_X), ug), y0 = ldu(egof(p, EF_Y), ug), v0 = ldu(egof(p, EF_V), ug);
    const float h0 = ldu(egof(p, EF_H), ug), acc0 = ldu(egof(p, EF_ACC), ug), steer0 = ldu(egof(p, EF_STEER), ug);
    const float pd0 = ldu(egof(p, EF_PREV_DIST), ug), pa00 = ldu(egof(p, EF_PA0), ug), pa10 = ldu(egof(p, EF_PA1), ug);
    const float sx0 = ldu(egof(p, EF_SX), ug), sy0 = ldu(egof(p, EF_SY), ug), sv0 = ldu(egof(p, EF_SV), ug);
    const float sh0 = ldu(egof(p, EF_SH), ug);
    const int pidx_l = ldu(egoi(p, EF_PIDX), ug), intent_l = ldu(egoi(p, EF_INTENT), ug);
    const uint8_t alive_l = ldu(gmem(p.ego.alive), ug);
    float len_l = CAR_LENGTH, wid_l = CAR_WIDTH;
    if constexpr (DIMS) {
        len_l = ldu(gmem(p.ego_dim), 2 * ug);
        wid_l = ldu(gmem(p.ego_dim), 2 * ug + 1);
    }
    // phase 1's first pass in group layout (lane (grp, sub): agent grp), without
    // traffic (there the NPC phase runs in between, and the window registers would
    // stay live through it): the agent's route, path index and env reset flag
    // EARLY (k_step's compile-time layouts without traffic: N <= 8 agent slots, the
    // window LDS in el.win)
    static_assert(!EARLY || (FUSED && !TRAFFIC), "LDS path windows: k_step without traffic");
    constexpr bool early = EARLY;
    const int ga = (tid >> 3) < N ? (tid >> 3) : 0;
    const int eea = PK == 1 ? e : e + ga / NE;
    int groute = 0, gpidx = 0;
    bool gpend = false;
    // (loads in one basic block, in-bounds by clamped indices rather than behind
    // branches: the scheduler keeps them together ahead of every use)
    // and its kinematic state and actions: phase 1's kinematics then read no LDS, so
    // no LDS read waits for round B's DMA before the window is needed (without alias
    // information an LDS read waits for every LDS DMA in flight)
    uint8_t gpend_b = 0, galive_b = 0;
    Kin gk{};
    float ga0 = 0.0f, ga1 = 0.0f;
    if constexpr (early) {
        const uint32_t ugg = (uint32_t)(e * NE + ga);
        groute = ldu(egoi(p, EF_ROUTE), ugg);
        gpidx = ldu(egoi(p, EF_PIDX), ugg);
        gpend_b = ldu(gmem(p.pending_reset), (uint32_t)eea);
        gk = Kin{ldu(egof(p, EF_X), ugg), ldu(egof(p, EF_Y), ugg), ldu(egof(p, EF_V), ugg), ldu(egof(p, EF_H), ugg),
                 ldu(egof(p, EF_ACC), ugg), ldu(egof(p, EF_STEER), ugg)};
        galive_b = ldu(gmem(p.ego.alive), ugg);
        ga0 = ldu(gmem(in.actions), 2 * ugg);
        ga1 = ldu(gmem(in.actions), 2 * ugg + 1);
    }
    float rl0 = 0.0f, rl1 = 0.0f;
    if (FUSED && !ESPLIT) {
        const int rmax = p.R - 1;
        rl0 = ldu(gmem(p.rel_angles), (uint32_t)(tid < rmax ? tid : rmax));
        rl1 = ldu(gmem(p.rel_angles), (uint32_t)(tid + WAVE < rmax ? tid + WAVE : rmax));
    }
    NpcRegs nreg{};
    // in flight with the ego loads; only the slots the env's deal class says are filled (the
    // class is its NPC count after the previous step; the last class and no deal: every slot)
    if constexpr (TRAFFIC) nreg = npc_load<DIMS>(p, e, tid, npc_cls < kDealClasses - 1 ? npc_cls : p.K);
    // every load above is issued before any of their values is used (a use scheduled
    // between them would put a wait for the first loads in front of the rest)
    __builtin_amdgcn_sched_barrier(0);
    static_assert(!TSC || (TRAFFIC && ESPLIT && PK == 1 && !DIMS), "TSC: the traffic early split's car waves");
    const bool pending = pending_b != 0;
    gpend = gpend_b != 0;
    const bool do_reset = in.auto_reset && pending;
    const int prev_step = do_reset ? 0 : step_prev;
    const int prev_npcs = TRAFFIC ? (do_reset ? 0 : npcs_prev) : 0;
    if (TSC && tid == 0) {  // the start-of-step position (the spawn after an auto-reset) for the NPC spawn test
        float sx_ = x0, sy_ = y0;
        if (do_reset) {
            const int rid = reset_route(p, in.rng_counter, ee, 0, route_l);
            sx_ = gmem(p.rt.spawn)[3 * rid];
            sy_ = gmem(p.rt.spawn)[3 * rid + 1];
        }
        el.envw[0] = __float_as_int(sx_);
        el.envw[1] = __float_as_int(sy_);
    }
    if (!TSC && lane_on) {
        el.a0[il] = a0;
        el.a1[il] = a1;
        el.route[il] = route_l;
        el.x[il] = x0; el.y[il] = y0; el.v[il] = v0; el.h[il] = h0;
        el.acc[il] = acc0; el.steer[il] = steer0; el.prev_dist[il] = pd0;
        el.pa0[il] = pa00; el.pa1[il] = pa10;
        el.sx[il] = sx0; el.sy[il] = sy0; el.sv[il] = sv0; el.sh[il] = sh0;
        el.pidx[il] = pidx_l; el.intent[il] = intent_l; el.alive[il] = alive_l;
    }
    if (DIMS && lane_on) {  // an env being reset gets new Cars of the default size (Car.h:19-20)
        el.len[il] = do_reset ? CAR_LENGTH : len_l;
        el.wid[il] = do_reset ? CAR_WIDTH : wid_l;
    }
    if constexpr (FUSED && !ESPLIT) {
        if (p.R <= 2 * WAVE) {
            if (tid < p.R) el.rel[tid] = rl0;
            if (tid + WAVE < p.R) el.rel[tid + WAVE] = rl1;
        } else {
            for (int b = tid; b < p.R; b += WAVE) el.rel[b] = gmem(p.rel_angles)[b];
        }
    }
    if (!TSC && lane_on && do_reset) {  // the lane's env was auto-reset: its agents start from their spawns
        const int rid = reset_route(p, in.rng_counter, ee, PK == 1 ? il : il - (ee - e) * NE, route_l);
        const float rx = gmem(p.rt.spawn)[3 * rid], ry = gmem(p.rt.spawn)[3 * rid + 1], rh = gmem(p.rt.spawn)[3 * rid + 2];
        el.route[il] = rid;
        el.x[il] = rx; el.y[il] = ry; el.v[il] = 0.0f; el.h[il] = rh;
        el.acc[il] = 0.0f; el.steer[il] = 0.0f; el.prev_dist[il] = 0.0f; el.pa0[il] = 0.0f; el.pa1[il] = 0.0f;
        el.sx[il] = rx; el.sy[il] = ry; el.sv[il] = 0.0f; el.sh[il] = rh;
        el.pidx[il] = 0; el.intent[il] = gmem(p.rt.intent)[rid]; el.alive[il] = 1;
    }
    // round B: the first pass's path windows, loaded straight into LDS (gfx950
    // global_load_lds_dwordx4: no VGPRs held while they are in flight) from the
    // group-layout route / index registers.  Agent grp's window is the 64 points
    // from s_e = start_i rounded down to even (16-B aligned: 32 chunks of 2 points,
    // [start_i, start_i + 50) and the look-ahead target start_i + <= 59 inside it);
    // lane (grp, sub) loads chunks 4 sub .. 4 sub + 3 (instruction m: chunk 4 sub +
    // m at win + m KB + grp * 128 + sub * 16) and reads back exactly those, so each
    // lane's 8 points arrive as 4 aligned 16-B LDS reads.  A fifth instruction brings
    // the route row's last segment (points plen, plen + 1: lane sub 0) and path[10, 11] (sub 1).
    // Chunks past the path's end are clamped to its last one: those points lie
    // beyond every window's range and are never used.
    int eroute = 0, epidx = 0;
    if (early) {
        const bool greset = in.auto_reset && gpend;
        eroute = greset ? reset_route(p, in.rng_counter, eea, PK == 1 ? ga : ga - (eea - e) * NE, groute) : groute;
        epidx = greset ? 0 : gpidx;
        if (greset) {  // agent ga starts from its spawn (as the lane layout above)
            gk = Kin{gmem(p.rt.spawn)[3 * eroute], gmem(p.rt.spawn)[3 * eroute + 1], 0.0f,
                     gmem(p.rt.spawn)[3 * eroute + 2], 0.0f, 0.0f};
            galive_b = 1;
        }
        const int start_i = epidx < 0 ? 0 : epidx;
        const int sub = tid & 7;
        const uint32_t rbase = (uint32_t)eroute * (uint32_t)(2 * 4 * p.rt.row);  // bytes
        typedef const __attribute__((address_space(1))) char gchar;
        gchar* path_b = (gchar*)gmem(p.rt.path);
        __attribute__((address_space(3))) char* win = (__attribute__((address_space(3))) char*)el.win;
#pragma unroll
        for (int m = 0; m < 4; ++m) {
            int c = (start_i >> 1) + sub * 4 + m;
            c = c < (p.rt.plen >> 1) ? c : (p.rt.plen >> 1) - 1;
            __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(path_b + rbase + c * 16),
                                             (__attribute__((address_space(3))) void*)(win + m * 1024), 16, 0, 0);
        }
        const int cx = sub == 0 ? p.rt.plen >> 1 : 5;  // points plen, plen + 1 (last segment) / 10, 11
        __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(path_b + rbase + cx * 16),
                                         (__attribute__((address_space(3))) void*)(win + 4 * 1024), 16, 0, 0);
    }
    const int step_no = prev_step + 1;  // res.step = ++step_count (:137)
    // gmem(p.step_count)[e] = step_no is stored with the other env flags (a store this
    // early would be drained by the vmcnt waits of every later load)
    // (no fence: an acquire fence would also wait for round B's LDS DMA, which
    // phase 1 first needs after the kinematics; one wave's LDS operations complete
    // in order, so ordering the code is enough)
    wave_lds_order();

    STAMP(0);
    int ncnt = 0;
    if constexpr (TSC) {
        wave_lds_sync();
        ncnt = npc_phase(p, in, e, prev_npcs, *nl, tid, reinterpret_cast<const float*>(el.envw),
                         reinterpret_cast<const float*>(el.envw + 1), nreg);
        __syncthreads();  // barrier H: the LiDAR wave has run this env's ego through phase 1
    } else if constexpr (TRAFFIC) {
        ncnt = npc_phase(p, in, e, prev_npcs, *nl, tid, el.x, el.y, nreg);
    }

    if (TRAFFIC && FUSED) {
        // the envs with many NPCs set the kernel's end: the rest of their step goes first
        // (3 or more NPCs: level 2, 6 or more: 3; config 4 +1.4 % over a fixed level)
        if (ncnt >= 6) __builtin_amdgcn_s_setprio(3);
        else if (ncnt >= 3) __builtin_amdgcn_s_setprio(2);
        else __builtin_amdgcn_s_setprio(1);
    } else if (TRAFFIC) {
        __builtin_amdgcn_s_setprio(0);
    }
    STAMP(1);

    // ---- phase 1: kinematics (:151-163), path index, base reward (:15-46),
    // status (:165-290).  Lane (grp, sub): agent i0 + grp, sub-task sub.
    const int grp = tid >> 3, sub = tid & 7;
    const unsigned long long gmask = 0xFFull << (grp * 8);
    for (int i0 = 0; i0 < (TSC ? 0 : N); i0 += 8) {  // (TSC: the LiDAR wave ran it)
        const int i = i0 + grp;
        const bool act = i < N;
        const int ii = act ? i : 0;  // idle groups mirror agent 0 so every lane reaches the ballots
        ego_phase1<early, dims>(p, in, el, i, act, ii, grp, sub, gmask, eroute, epidx, gk, galive_b, ga0, ga1);
    }
    // The LDS DMA of round B has landed (the loop waited for it before reading the
    // window), but the compiler cannot see that on every path into here, and with an
    // LDS DMA possibly pending it puts an s_waitcnt vmcnt(0) in front of every later
    // LDS access -- which then also waits for every global store issued before it
    // (cars_post's outputs and state write-back in front of the LiDAR's first LDS
    // access).  An explicit wait here (nothing else is in flight) retires the DMA for
    // the compiler too.
    if constexpr (early) __builtin_amdgcn_s_waitcnt(kWaitVmcnt0);
    wave_lds_sync();

    STAMP(2);
    // one ego per env and no NPCs: no car can touch another, and no LiDAR beam can
    // meet another car (configs 1 and 2) -- the SAT pairs, obstacle table and
    // candidate masks below are skipped (the masks stay empty)
    const bool lone = !TRAFFIC && NE == 1;
    // ---- car-car SAT (:292-318): ego pairs (i<j) and ego x NPC, one pair per lane
    for (int pbase = 0; pbase < (lone ? 0 : N * N); pbase += WAVE) {
        const int pi = pbase + tid;
        // (a, b) = (pi / N, pi % N); lane = 8a + b without the integer division when N <= 8
        const int a = N <= 8 ? (tid >> 3) : pi / N, b = N <= 8 ? (tid & 7) : pi % N;
        if (N <= 8 ? (a < N && b < N) : pi < N * N) {
            // two cars whose centres are more than the sum of their circumradii apart
            // (2 x 29.55 px; 60 px with margin for the rounding of the corners) cannot
            // overlap: the SAT runs only for lanes (and waves) with a close pair
            const float cdx = el.x[a] - el.x[b], cdy = el.y[a] - el.y[b];
            const bool close = !(cdx * cdx + cdy * cdy > 3600.0f) || all_pairs;  // (other sizes: every pair)
            if (a < b && (PK == 1 || a / NE == b / NE) && el.alive[a] && el.alive[b] && close &&
                sat_collide(reinterpret_cast<const float*>(&el.cx[a]), reinterpret_cast<const float*>(&el.cy[a]),
                            el.c[a], el.s[a], reinterpret_cast<const float*>(&el.cx[b]),
                            reinterpret_cast<const float*>(&el.cy[b]), el.c[b], el.s[b]))
                atomicOr(&el.col[a], 1ull << b);
        }
    }
    if constexpr (TRAFFIC) {
        for (int pbase = 0; pbase < N * ncnt; pbase += WAVE) {
            const int pi = pbase + tid;
            if (pi < N * ncnt) {
                const int a = pi / ncnt, b = pi % ncnt;
                const float cdx = el.x[a] - nl->x[b], cdy = el.y[a] - nl->y[b];
                const bool close = !(cdx * cdx + cdy * cdy > 3600.0f) || all_pairs;  // as for the ego pairs
                if (el.alive[a] && close && sat_collide(reinterpret_cast<const float*>(&el.cx[a]),
                                               reinterpret_cast<const float*>(&el.cy[a]), el.c[a], el.s[a],
                                               nl->cx[b], nl->cy[b], nl->c[b], nl->s[b]))
                    el.colnpc[a] = 1;
            }
        }
    }
    wave_lds_sync();

    STAMP(3);
    // ---- greedy resolution in (i, j) order (:292-318): lane = agent (N <= 64);
    // the order-dependent scan runs on wave-uniform masks
    {
        const int i = tid;
        const bool in_env = i < N;
        const uint8_t alive_i = in_env ? el.alive[i] : 0;
        const uint8_t done_i = in_env ? el.done[i] : 0;
        const unsigned long long col_i = in_env ? el.col[i] : 0ull;
        const bool colnpc_i = TRAFFIC && in_env && el.colnpc[i];
        unsigned long long donem = ballot(in_env && (done_i || !alive_i));
        const unsigned long long npcm = ballot(colnpc_i);
        unsigned long long crash = 0ull;
        // (most steps have no car-car contact at all: the scan is skipped)
        if (ballot(col_i != 0ull) != 0ull || npcm != 0ull) {
            for (int a = 0; a < N; ++a) {
                if ((donem >> a) & 1ull) continue;
                const unsigned long long ca = readlane64(col_i, a);
                const unsigned long long higher = (a == 63) ? 0ull : (~0ull << (a + 1));
                const unsigned long long hits = ca & ~donem & higher;
                if (hits) { donem |= hits | (1ull << a); crash |= hits | (1ull << a); }
                if (TRAFFIC && ((npcm >> a) & 1ull)) { donem |= 1ull << a; crash |= 1ull << a; }
            }
        }
        if (in_env && ((crash >> i) & 1ull)) { el.done[i] = 1; el.status[i] = ST_CRASH_CAR; }
    }
    wave_lds_sync();
    // respawn crashed egos (Car::respawn, Car.cpp:76-84; :339-351), lane = agent;
    // the final state is written back by cars_post
    for (int i = tid; i < N; i += WAVE) {
        const uint8_t st = el.status[i];
        if (p.respawn && el.alive[i] && el.done[i] && (st == ST_CRASH_CAR || st == ST_CRASH_WALL || st == ST_CRASH_LINE)) {
            const float sh = el.sh[i];
            float s, c;
            sincosf(sh, &s, &c);
            el.x[i] = el.sx[i]; el.y[i] = el.sy[i]; el.v[i] = el.sv[i]; el.h[i] = sh; el.c[i] = c; el.s[i] = s;
            el.pidx[i] = 0; el.prev_dist[i] = 0.0f; el.pa0[i] = 0.0f; el.pa1[i] = 0.0f;
            el.acc[i] = 0.0f; el.steer[i] = 0.0f;
            el.tgx[i] = el.t10x[i]; el.tgy[i] = el.t10y[i];  // path[min(0 + 10, 159)]
        }
    }
    if constexpr (ESPLIT) {  // the respawned egos (agent slots), for the LiDAR after barrier B
        const uint8_t st = el.status[tid < N ? tid : 0];
        const bool rs = tid < N && p.respawn && el.alive[tid < N ? tid : 0] && el.done[tid < N ? tid : 0] &&
                        (st == ST_CRASH_CAR || st == ST_CRASH_WALL || st == ST_CRASH_LINE);
        const unsigned long long m = ballot(rs);
        if (tid == 0) el.envw[6] = (int)(unsigned)m;
    }
    wave_lds_sync();

    STAMP(4);
    // ---- LiDAR obstacle table (:374-388): every ego (alive or not), then NPCs,
    // published to HBM for k_lidar together with each agent's candidate mask
    const int nob = lone ? 0 : N + ncnt;  // lone egos: no obstacle anyone could see
    const int OB = p.ob_stride;
    for (int o = tid; o < nob; o += WAVE) {
        float x, y, h, c, s, bl = CAR_LENGTH, bw = CAR_WIDTH;
        if (!TRAFFIC || o < N) {  // (no NPC branch without traffic: nl is null there)
            x = el.x[o]; y = el.y[o]; h = el.h[o]; c = el.c[o]; s = el.s[o];
            if (dims) { bl = el.len[o]; bw = el.wid[o]; }
        } else {
            const int k = o - N;
            x = nl->x[k]; y = nl->y[k]; h = nl->h[k]; c = nl->c[k]; s = nl->s[k];
            if constexpr (TRAFFIC && DIMS) { bl = nl->len[k]; bw = nl->wid[k]; }
        }
        const PxBox bx = aabb_px_d(x, y, c, s, bl, bw);
        const int4 b4 = make_int4(bx.x0, bx.x1, bx.y0, bx.y1);
        el.box[o] = b4;
        el.px[o] = x; el.py[o] = y; el.ph[o] = h;
        if (!FUSED) p.ob_box[e * OB + o] = b4;
    }
    for (int i = tid; i < N; i += WAVE) { el.cand[2 * i] = 0ull; el.cand[2 * i + 1] = 0ull; }
    wave_lds_sync();
    // per-agent candidate boxes: not self, not state-identical to self within
    // 1e-3 (Lidar.cpp:55-62), and within max_dist + 2 px of the agent (no probe
    // beyond max_dist exists, truncation moves a probe < 1 px)
    for (int pbase = 0; pbase < N * nob; pbase += WAVE) {
        const int pi = pbase + tid;
        const bool small = N <= 8 && nob <= 8;  // lane = 8a + o, no integer division
        // (nob > 0 inside the loop; the guard only keeps a compile-time N = 1 from a division by zero)
        const int a = small ? (tid >> 3) : pi / (nob > 0 ? nob : 1), o = small ? (tid & 7) : pi - a * nob;
        if (small ? (a < N && o < nob) : pi < N * nob) {
            const float cx = el.x[a], cy = el.y[a];
            if (o != a && (PK == 1 || a / NE == o / NE) && el.alive[a] &&
                !(fabs_f(el.px[o] - cx) < 1e-3f && fabs_f(el.py[o] - cy) < 1e-3f && fabs_f(el.ph[o] - el.h[a]) < 1e-3f)) {
                const int4 bx = el.box[o];
                const float ddx = fmaxf(fmaxf((float)bx.x - cx, cx - (float)bx.y), 0.0f);
                const float ddy = fmaxf(fmaxf((float)bx.z - cy, cy - (float)bx.w), 0.0f);
                const float reach = p.lidar_max + 2.0f;
                if (ddx * ddx + ddy * ddy <= reach * reach) atomicOr(&el.cand[2 * a + (o >> 6)], 1ull << (o & 63));
            }
        }
    }
    wave_lds_sync();
    if (!FUSED) {
        for (int i = tid; i < N; i += WAVE) {
            const int g = e * NE + i;
            gmem(p.ob_cand)[2 * g] = el.cand[2 * i];
            gmem(p.ob_cand)[2 * g + 1] = el.cand[2 * i + 1];
        }
    }

    STAMP(5);
    if constexpr (ESPLIT) {
        __syncthreads();  // barrier B: obstacle table, candidate masks, respawns
    }
    return CarsCtx{step_no, do_reset, ncnt, false};
}

// The traffic early split's LiDAR wave before its road march (the car waves' cars_pre<TSC>
// meanwhile run the NPC phase): the egos of the workgroup's PK envs, one each, from HBM
// into their envs' car LDS exactly as cars_pre's round A and auto-reset write them (lane j
// = env es[j]), then phase 1 for all of them in one pass (lane group j = env j's ego in its
// own LDS: the group's CarsLDS pointers differ per lane).  Returns the slots' alive mask.
template <int PK, int KF>
__device__ __forceinline__ unsigned long long ts_ego_phase(const SimParams& p, const StepInputs& in,
                                                           unsigned char* step_lds, const int reg, const int* es,
                                                           const int lane) {
    const bool on = lane < PK;
    int ee = es[0];
#pragma unroll
    for (int j = 1; j < PK; ++j) ee = lane == j ? es[j] : ee;
    const uint32_t ug = (uint32_t)ee;  // (one ego per env: the agent index is the env index)
    const uint8_t pending_b = ldu(gmem(p.pending_reset), ug);
    const float a0 = ldu(gmem(in.actions), 2 * ug), a1 = ldu(gmem(in.actions), 2 * ug + 1);
    const int route_l = ldu(egoi(p, EF_ROUTE), ug);
    const float x0 = ldu(egof(p, EF_X), ug), y0 = ldu(egof(p, EF_Y), ug), v0 = ldu(egof(p, EF_V), ug);
    const float h0 = ldu(egof(p, EF_H), ug), acc0 = ldu(egof(p, EF_ACC), ug), steer0 = ldu(egof(p, EF_STEER), ug);
    const float pd0 = ldu(egof(p, EF_PREV_DIST), ug), pa00 = ldu(egof(p, EF_PA0), ug), pa10 = ldu(egof(p, EF_PA1), ug);
    const float sx0 = ldu(egof(p, EF_SX), ug), sy0 = ldu(egof(p, EF_SY), ug), sv0 = ldu(egof(p, EF_SV), ug);
    const float sh0 = ldu(egof(p, EF_SH), ug);
    const int pidx_l = ldu(egoi(p, EF_PIDX), ug), intent_l = ldu(egoi(p, EF_INTENT), ug);
    const uint8_t alive_l = ldu(gmem(p.ego.alive), ug);
    __builtin_amdgcn_sched_barrier(0);
    const CarsLDS el = carve_cars_lds(step_lds + (on ? lane : 0) * reg, 1, KF);
    const bool do_reset = in.auto_reset && pending_b != 0;
    if (on) {
        el.a0[0] = a0; el.a1[0] = a1;
        el.route[0] = route_l;
        el.x[0] = x0; el.y[0] = y0; el.v[0] = v0; el.h[0] = h0;
        el.acc[0] = acc0; el.steer[0] = steer0; el.prev_dist[0] = pd0;
        el.pa0[0] = pa00; el.pa1[0] = pa10;
        el.sx[0] = sx0; el.sy[0] = sy0; el.sv[0] = sv0; el.sh[0] = sh0;
        el.pidx[0] = pidx_l; el.intent[0] = intent_l; el.alive[0] = alive_l;
    }
    if (on && do_reset) {  // the env was auto-reset: its ego starts from its spawn (as cars_pre)
        const int rid = reset_route(p, in.rng_counter, ee, 0, route_l);
        const float rx = gmem(p.rt.spawn)[3 * rid], ry = gmem(p.rt.spawn)[3 * rid + 1], rh = gmem(p.rt.spawn)[3 * rid + 2];
        el.route[0] = rid;
        el.x[0] = rx; el.y[0] = ry; el.v[0] = 0.0f; el.h[0] = rh;
        el.acc[0] = 0.0f; el.steer[0] = 0.0f; el.prev_dist[0] = 0.0f; el.pa0[0] = 0.0f; el.pa1[0] = 0.0f;
        el.sx[0] = rx; el.sy[0] = ry; el.sv[0] = 0.0f; el.sh[0] = rh;
        el.pidx[0] = 0; el.intent[0] = gmem(p.rt.intent)[rid]; el.alive[0] = 1;
    }
    wave_lds_sync();
    const unsigned long long am = ballot(on && el.alive[0] != 0);
    // phase 1, lane group g = env g's ego (N = 1: agent 0 of its own LDS)
    const int grp = lane >> 3, sub = lane & 7;
    const unsigned long long gmask = 0xFFull << (grp * 8);
    const bool act = grp < PK;
    const CarsLDS eg = carve_cars_lds(step_lds + (act ? grp : 0) * reg, 1, KF);
    ego_phase1<false, false>(p, in, eg, 0, act, 0, grp, sub, gmask, 0, 0, Kin{}, 0, 0.0f, 0.0f);
    wave_lds_sync();
    return am;
}

// The rest of the car part (after the LiDAR in k_step, right after cars_pre in
// k_cars): bonuses, team mix and env flags (:320-370), the reward / done /
// status outputs and the state write-back, the observation head (:418-520).
// Reads only the car LDS (the LiDAR never writes it).
template <bool TRAFFIC, bool FUSED, class NL, int PK = 1, bool DIMS = false, int NC = 0>
__device__ __forceinline__ void cars_post(const SimParams& p, const Outputs& out, const int e, const CarsLDS& el,
                                          const NL* nl, CarsCtx& cx) {
    const int tid = threadIdx.x & (WAVE - 1);
    const int NE = NC ? NC : p.N;  // agents per env (PK > 1: see cars_pre; NC: compile-time)
    const int npk = PK == 1 ? 1 : (p.E - e < PK ? p.E - e : PK);
    const int N = PK == 1 ? NE : npk * NE;
    const int step_no = cx.step_no, ncnt = cx.ncnt;
    const bool do_reset = cx.do_reset;
    const int grp = tid >> 3, sub = tid & 7;
    const unsigned long long gmask = 0xFFull << (grp * 8);
    // ---- bonuses, team mix, flags (:320-370), lane = agent
    {
        const int i = tid;
        const bool in_env = i < N;
        const uint8_t alive_i = in_env ? el.alive[i] : 0;
        const uint8_t done_i = in_env ? el.done[i] : 0, st_i = in_env ? el.status[i] : 0;
        float rew_i = in_env ? el.rew[i] : 0.0f;
        if (done_i) {
            if (st_i == ST_CRASH_CAR) rew_i += p.k_cv;
            else if (st_i == ST_CRASH_WALL || st_i == ST_CRASH_LINE) rew_i += p.k_co;
            else if (st_i == ST_SUCCESS) rew_i += p.k_succ;
        }
        if (p.use_team && N > 0) {  // sequential sum in agent order, as the reference
            float avg = 0.0f;
            if (PK == 1) {
                if (N <= 8) {  // (unrolled: constant lanes, no scalar loop)
#pragma unroll
                    for (int a = 0; a < 8; ++a) {
                        const float r = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(rew_i), a));
                        avg = a < N ? avg + r : avg;
                    }
                } else {
                    for (int a = 0; a < N; ++a) avg += __int_as_float(__builtin_amdgcn_readlane(__float_as_int(rew_i), a));
                }
                avg /= float(N);
            } else {
                for (int ps = 0; ps < npk; ++ps) {  // each env's own mean
                    float sm = 0.0f;
                    for (int a = 0; a < NE; ++a)
                        sm += __int_as_float(__builtin_amdgcn_readlane(__float_as_int(rew_i), ps * NE + a));
                    sm /= float(NE);
                    avg = (i < N && i / NE == ps) ? sm : avg;
                }
            }
            rew_i = (1.0f - p.alpha) * rew_i + p.alpha * avg;
        }
        const unsigned long long alive_m = ballot(in_env && alive_i);
        const unsigned long long succ_m = ballot(in_env && alive_i && done_i && st_i == ST_SUCCESS);
        const unsigned long long done_m = ballot(in_env && done_i);
        // the env flags: lane ps < npk holds env e + ps (PK == 1: every lane env e)
        unsigned long long emask = ~0ull;
        int step_e = step_no;
        if (PK > 1) {
            const unsigned long long one = NE >= 64 ? ~0ull : ((1ull << NE) - 1ull);
            emask = tid < npk ? one << (tid * NE) : 0ull;
            for (int ps = 0; ps < npk; ++ps) {
                const int v = __builtin_amdgcn_readlane(step_no, ps * NE);
                step_e = tid == ps ? v : step_e;
            }
        }
        const int alive_cnt = __builtin_popcountll(alive_m & emask), succ_cnt = __builtin_popcountll(succ_m & emask);
        const bool terminated = p.respawn ? (succ_cnt > 0 && succ_cnt == alive_cnt) : ((done_m & emask) != 0ull);
        const bool truncated = p.max_steps > 0 && step_e >= p.max_steps;
        if (PK == 1) cx.ended = terminated || truncated;
        if (in_env) {
            const int g = e * NE + i;
            out.rew[g] = rew_i;
            out.done[g] = done_i;
            out.status[g] = st_i;
        }
        if (PK > 1 ? tid < npk : tid == 0) {
            const int ev = e + (PK > 1 ? tid : 0);
            gmem(p.step_count)[ev] = step_e;
            out.term[ev] = terminated;
            out.trunc[ev] = truncated;
            out.alive_cnt[ev] = alive_cnt;
            out.step[ev] = step_e;
            gmem(p.pending_reset)[ev] = (terminated || truncated) ? 1 : 0;
        }
    }
    // ---- the final ego state back to HBM (lane = agent)
    ego_writeback(p, e, NE, N, el, do_reset, tid, DIMS);
    if (out.state) {
        // the state gather format: the post-step state the root rebuilds the head from
        // (launch_decode_state), instead of the head itself
        const size_t n = (size_t)out.state_n;
        __attribute__((address_space(1))) uint8_t* sb = gmem(out.state);
        for (int i = tid; i < N; i += WAVE) {
            const size_t a = (size_t)e * NE + i;
            reinterpret_cast<__attribute__((address_space(1))) float*>(sb)[a] = el.x[i];
            reinterpret_cast<__attribute__((address_space(1))) float*>(sb + 4 * n)[a] = el.y[i];
            reinterpret_cast<__attribute__((address_space(1))) float*>(sb + 8 * n)[a] = el.v[i];
            reinterpret_cast<__attribute__((address_space(1))) float*>(sb + 12 * n)[a] = el.h[i];
            reinterpret_cast<__attribute__((address_space(1))) int16_t*>(sb + 16 * n)[a] = (int16_t)el.route[i];
            reinterpret_cast<__attribute__((address_space(1))) int16_t*>(sb + 18 * n)[a] = (int16_t)el.pidx[i];
            sb[20 * n + a] = (uint8_t)el.intent[i];
            sb[21 * n + a] = el.alive[i];
        }
        return;
    }
    // ---- observation head (:418-520)
    QSTAMP(5);
    const int C = PK > 1 ? NE : N + (TRAFFIC ? ncnt : 0);  // neighbour candidates per agent (+ itself)
    // (the fused kernels' compile-time layout without traffic holds N <= 8 agents: C <= 8,
    // and the per-lane path below -- with its std::sort pass -- is not compiled into them)
    constexpr bool kFew = !TRAFFIC && FUSED && !DIMS;
    if (kFew || C <= 8) {
        // lane (grp, sub): agent i0 + grp, neighbour candidate sub; rank = position
        // in the stable distance order (== libstdc++ insertion sort, <= 16 elements)
        for (int i0 = 0; i0 < N; i0 += 8) {
            const int i = i0 + grp;
            const bool act = i < N;
            const int ii = act ? i : 0;
            const bool alv = act && el.alive[ii] != 0;
            const float x = el.x[ii], y = el.y[ii], v = el.v[ii], h = el.h[ii];
            const int j = sub;
            const int js = PK == 1 ? j : (ii / NE) * NE + j;  // candidate j's agent slot
            bool valid = false;
            float ox = 0.0f, oy = 0.0f, ov = 0.0f, oh = 0.0f;
            int oi = 0;
            if (alv && j < C && js != ii) {
                if (js < N) {
                    valid = el.alive[js] != 0;
                    ox = el.x[js]; oy = el.y[js]; ov = el.v[js]; oh = el.h[js]; oi = el.intent[js];
                } else {
                    const int kk = j - N;
                    valid = nl->alive[kk] != 0;
                    ox = nl->x[kk]; oy = nl->y[kk]; ov = nl->v[kk]; oh = nl->h[kk]; oi = nl->intent[kk];
                }
            }
            const float ddx = ox - x, ddy = oy - y;
            // an invalid candidate's distance is NaN: it compares false both ways, so it
            // is neither before nor tied with anyone
            const float d = valid ? __builtin_sqrtf(ddx * ddx + ddy * ddy) : __builtin_nanf("");
            // rank among the group's 7 other candidates, each brought in by DPP moves
            // (quad permutations, then the same after the half-row mirror: lanes sub ^ k
            // and 7 - (sub ^ k), k = 0..3), no LDS permutes
            int rank = 0;
            auto before = [&](float dk, int kk) { rank += (dk < d || (dk == d && kk < j)) ? 1 : 0; };
            const float dm = dpp_f(d, 0x141);  // row_half_mirror: candidate 7 - sub
            before(dpp_f(d, 0xB1), sub ^ 1);   // quad_perm [1,0,3,2]
            before(dpp_f(d, 0x4E), sub ^ 2);   // quad_perm [2,3,0,1]
            before(dpp_f(d, 0x1B), sub ^ 3);   // quad_perm [3,2,1,0]
            before(dm, 7 - sub);
            before(dpp_f(dm, 0xB1), 7 - (sub ^ 1));
            before(dpp_f(dm, 0x4E), 7 - (sub ^ 2));
            before(dpp_f(dm, 0x1B), 7 - (sub ^ 3));
            const int nb = __builtin_popcountll(ballot(valid) & gmask);
            // one straight-line block for every lane: the agent's own features (the
            // lane of its own index: never a candidate), its look-ahead terms, or a
            // neighbour's features -- the atan2f chain runs beside the divisions
            const bool self = js == ii;
            const float dxd = el.tgx[ii] - x, dyd = el.tgy[ii] - y;  // path[min(idx + 10, 159)] (:444-452)
            const float f4 = __builtin_sqrtf(dxd * dxd + dyd * dyd) / float(WIDTH);
            // one wrap per lane: the own lane's bearing of the look-ahead point, a
            // neighbour lane's relative heading
            const float wr = wrap_angle(self ? atan2f_wave(-dyd, dxd) - h : oh - h) / PI_F;
            const float f5 = wr;
            const float f0 = (self ? x : ox - x) / float(WIDTH);
            const float f1 = (self ? y : oy - y) / float(HEIGHT);
            const float f2 = (self ? v : ov - v) / PHYSICS_MAX_SPEED;
            const float f3 = self ? h / PI_F : wr;
            if (act) {
                float* row = out.obs + (size_t)(e * NE + i) * out.obs_ld;
                if (!alv) {
                    for (int cc = sub; cc < OBS_HEAD; cc += 8) row[cc] = 0.0f;
                } else {
                    if (self) {
                        row[0] = f0; row[1] = f1; row[2] = f2; row[3] = f3; row[4] = f4; row[5] = f5;
                    }
                    if (valid && rank < NEIGHBOR_COUNT) {
                        float* o = row + 6 + 5 * rank;
                        o[0] = f0; o[1] = f1; o[2] = f2; o[3] = f3; o[4] = float(oi);
                    }
                    if (sub < NEIGHBOR_COUNT && sub >= nb) {
                        float* o = row + 6 + 5 * sub;
                        o[0] = o[1] = o[2] = o[3] = o[4] = 0.0f;
                    }
                }
                for (int cc = OBS_HEAD + p.lidar_slots + sub; cc < out.obs_ld; cc += 8) row[cc] = 0.0f;
            }
        }
    } else if constexpr (!kFew) {
        bool exact = false;  // (N <= 64: one pass, lane i = agent i)
        float dl = 0.0f;
        for (int i = tid; i < N; i += WAVE) {
            const int g = e * NE + i;
            float* row = out.obs + (size_t)g * out.obs_ld;
            if (!el.alive[i]) {
                for (int c = 0; c < OBS_HEAD; ++c) row[c] = 0.0f;
                for (int c = OBS_HEAD + p.lidar_slots; c < out.obs_ld; ++c) row[c] = 0.0f;
                continue;
            }
            exact = write_obs_head_tg<TRAFFIC>(p, i, el, nl, ncnt, el.tgx[i], el.tgy[i], row, out.obs_ld == p.D, &dl);
        }
        if constexpr (PK == 1) {
            const unsigned long long m = ballot(exact);
            // (more than 64 candidates only with the runtime layout's egos and traffic: with the
            // compile-time traffic layout the env has one ego, and without traffic <= 63 others)
            if (__builtin_expect(m != 0ull, 0))
                obs_exact_pass<TRAFFIC, TRAFFIC && DIMS>(p, m, dl, el, nl, ncnt, out.obs + (size_t)e * NE * out.obs_ld,
                                                         out.obs_ld);
        }
    }
    STAMP(6);
}

template <bool TRAFFIC>
__global__ __launch_bounds__(WAVE) void k_cars(SimParams p, StepInputs in, Outputs out, int e_begin) {
    extern __shared__ __align__(16) unsigned char cars_lds[];
    const int e = e_begin + xcd_env((int)blockIdx.x, (int)gridDim.x);
#if defined(MEV_STAMPS_R)
    STAMP_RAW(0);
#endif
    const CarsLDS el = carve_cars_lds(cars_lds, p.N, cars_k(p), true);
    __shared__ typename std::conditional<TRAFFIC, NpcLDS, char>::type nl_storage;
    NpcLDS* nl = nullptr;
    if constexpr (TRAFFIC) nl = &nl_storage;
    CarsCtx cx = cars_pre<TRAFFIC, false, NpcLDS, 1, false, false, true>(p, in, out, e, el, nl);
    wave_lds_sync();
    cars_post<TRAFFIC, false, NpcLDS, 1, true>(p, out, e, el, nl, cx);
}

// ------------------------------------------------------------- LiDAR ---
// Lidar::update (cpp/Lidar.cpp:16-90) for every (env, agent, beam), reading
// the poses k_cars left in HBM (after respawn) and the obstacle boxes /
// candidate masks it published.
//
// The reference marches k = 0..S-1 (dist_k = k*step) and stops at the first k
// whose truncated pixel is off-screen (no hit), off-road (k>0, hit) or inside
// another car's AABB (k>0, hit).  We find the same k with far fewer probes:
//  1. road/screen: exact probe at k, then skip ahead by the number of steps
//     provably safe from the real-valued point (truncation moves a pixel by
//     < 1 px, margin 1.5 px): every skipped probe is on-screen and strictly
//     inside a road strip or the corner square, so it could not have stopped
//     the march;
//  2. cars: for each candidate box, the probes whose real point lies in the
//     box's real slab (box_lo/box_hi) form a superset range of k; those (and
//     only below the k of step 1) are probed exactly, in march order.
// Bit-identical to the sequential march (tests/test_parity_gpu.py,
// tests/test_gpu_vs_oracle.py).
// The float rounding of the probe position, of the reciprocal and of the
// accumulated distances is absorbed by the slab margins and by one extra probe
// index at each end of the range, so a real hit is never dropped.

// Straight-line LiDAR arithmetic: the value is computed on every lane (an empty
// volatile asm statement the compiler cannot sink into a branch), so a select
// replaces the divergent branch -- exec-mask bookkeeping and a pipeline break --
// the compiler would otherwise wrap around a short computation.  No instruction
// is emitted for it.
template <class T>
__device__ __forceinline__ T lidar_keep(T v) {
    asm volatile("" : "+v"(v));
    return v;
}
// beam steps over a provably safe stretch (0 when it is shorter than one step)
__device__ __forceinline__ int safe_steps(float safe, float stp, float inv_stp) {
    const int j = lidar_keep((int)(safe * inv_stp));
    return (safe >= stp) ? j : 0;
}

// Distance along a beam from its real point (fx, fy) over which every probe is
// provably on screen and on the road (the truncated pixel is within 1 px per
// axis, < 1.42 px, of the real point).  Each bound below alone guarantees its
// stretch, so the road bound is their maximum; all are directional:
//  - strips: distance to the strip edge (|x - 375| = rw - 1.5) the ray heads for;
//  - centre square: inside the square shrunk by 1.55 px, within the current
//    quadrant (only its own grass disc can be met there), outside that disc
//    grown by 2 px (extra margin for the tangent-case rounding of the root):
//    distance to the first of the grown disc, the shrunk square's edge and the
//    quadrant's edge;
//  - screen: distance to the half-pixel-inset screen edge.
__device__ inline float road_safe(float fx, float fy, float dx, float dy, float idx, float idy, float iadx,
                                  float iady, float rwm, float ccen, float crf) {
    const float big = 1.0e6f;
    const float rx = fx - 375.0f, ry = fy - 375.0f;
    const float ax = fabs_f(rx), ay = fabs_f(ry);
    const float sx = ax < rwm ? rwm * iadx - rx * idx : 0.0f;
    const float sy = ay < rwm ? rwm * iady - ry * idy : 0.0f;
    const float sqm = ccen - 1.55f, rg = crf + 2.0f;
    // the quadrant the ray is in, or heads into from an axis (rx == 0: the sign of dx)
    const float qx = rx != 0.0f ? rx : dx, qy = ry != 0.0f ? ry : dy;
    const float ocx = rx - (qx >= 0.0f ? ccen : -ccen), ocy = ry - (qy >= 0.0f ? ccen : -ccen);
    const float bq = ocx * dx + ocy * dy;
    const float cq = ocx * ocx + ocy * ocy - rg * rg;
    const float disc = bq * bq - cq;
    const float troot = lidar_keep(-bq - __builtin_amdgcn_sqrtf(disc));
    const float tdisc = cq <= 0.0f ? 0.0f : ((disc < 0.0f || bq >= 0.0f) ? big : troot);
    const float tsq = fminf(sqm * iadx - rx * idx, sqm * iady - ry * idy);
    const float tq = fminf(rx * dx < 0.0f ? -rx * idx : big, ry * dy < 0.0f ? -ry * idy : big);
    const float sc = fmaxf(ax, ay) < sqm ? fminf(tdisc, fminf(tsq, tq)) : 0.0f;
    const float road = fmaxf(fmaxf(sx, sy), sc);
    const float tx = (dx > 0.0f ? 748.5f - fx : fx - 0.5f) * iadx;
    const float ty = (dy > 0.0f ? 748.5f - fy : fy - 0.5f) * iady;
    return fminf(road, fminf(tx, ty));
}

// road_safe from a point every lane of the wave shares (phase 1: the car centre
// of the pass's agent): the strip and centre-square terms are wave-uniform
// branches, so a car outside the centre square does not evaluate the disc root.
__device__ inline float road_safe_uniform(float fx, float fy, float dx, float dy, float idx, float idy, float iadx,
                                          float iady, float rwm, float ccen, float crf) {
    const float big = 1.0e6f;
    const float rx = fx - 375.0f, ry = fy - 375.0f;
    const float ax = fabs_f(rx), ay = fabs_f(ry);
    const float sqm = ccen - 1.55f, rg = crf + 2.0f;
    float road = 0.0f;
    if (__builtin_amdgcn_readfirstlane((int)(ax < rwm))) road = fmaxf(road, rwm * iadx - rx * idx);
    if (__builtin_amdgcn_readfirstlane((int)(ay < rwm))) road = fmaxf(road, rwm * iady - ry * idy);
    if (__builtin_amdgcn_readfirstlane((int)(fmaxf(ax, ay) < sqm))) {
        const float qx = rx != 0.0f ? rx : dx, qy = ry != 0.0f ? ry : dy;
        const float ocx = rx - (qx >= 0.0f ? ccen : -ccen), ocy = ry - (qy >= 0.0f ? ccen : -ccen);
        const float bq = ocx * dx + ocy * dy;
        const float cq = ocx * ocx + ocy * ocy - rg * rg;
        const float disc = bq * bq - cq;
        const float troot = lidar_keep(-bq - __builtin_amdgcn_sqrtf(disc));
        const float tdisc = cq <= 0.0f ? 0.0f : ((disc < 0.0f || bq >= 0.0f) ? big : troot);
        const float tsq = fminf(sqm * iadx - rx * idx, sqm * iady - ry * idy);
        const float tq = fminf(rx * dx < 0.0f ? -rx * idx : big, ry * dy < 0.0f ? -ry * idy : big);
        road = fmaxf(road, fminf(tdisc, fminf(tsq, tq)));
    }
    const float tx = (dx > 0.0f ? 748.5f - fx : fx - 0.5f) * iadx;
    const float ty = (dy > 0.0f ? 748.5f - fy : fy - 0.5f) * iady;
    return fminf(road, fminf(tx, ty));
}

// atan2 to ~1e-5 rad and wrap to [-pi, pi]: culling only (beam ranges carry one
// beam of margin); every hit is still decided by exact probes.
__device__ inline float atan2_fast(float y, float x) {
    const float ax = fabs_f(x), ay = fabs_f(y);
    const float mx = fmaxf(ax, ay), mn = fminf(ax, ay);
    const float t = mn * __builtin_amdgcn_rcpf(fmaxf(mx, 1e-30f));
    const float s2 = t * t;
    float r = ((-0.0464964749f * s2 + 0.15931422f) * s2 - 0.327622764f) * s2 * t + t;
    r = ay > ax ? 1.57079637f - r : r;
    r = x < 0.0f ? 3.14159274f - r : r;
    return y < 0.0f ? -r : r;
}

__device__ inline float wrap_pi_fast(float a) { return a - 6.28318531f * rintf(a * 0.159154943f); }

// Real-coordinate slab of the pixels [lo, hi] of an integer box: (int)f lies
// in [lo, hi] only if f lies in [lo, hi + 1) (f >= 0: truncation is floor) or
// in (lo - 1, hi + 1) (f < 0 when lo <= 0); 0.01 px absorbs the float rounding
// of the probe position (< 1e-4 px) and of the reciprocal.
__device__ inline float box_lo(int lo) { return (float)(lo > 0 ? lo : lo - 1) - 0.01f; }
__device__ inline float box_hi(int hi) { return (float)hi + 1.01f; }

// Clip [lo, hi] (distances along the ray) to where coordinate c0 + dc*t lies in [a, b].
__device__ inline void slab_clip(float c0, float dc, float idc, float a, float b, float& lo, float& hi) {
    if (fabs_f(dc) < 1e-6f) {  // constant to < 2.5e-4 px over the ray
        if (c0 < a || c0 > b) { lo = 1.0f; hi = 0.0f; }
        return;
    }
    const float t1 = (a - c0) * idc, t2 = (b - c0) * idc;
    lo = fmaxf(lo, fminf(t1, t2));
    hi = fminf(hi, fmaxf(t1, t2));
}



// Per-wave LDS of k_lidar: ag float4[G] (x, y, heading, agent id) of the
// group's alive agents, dir float2[G*R] beam directions, res int[G*R] stop of
// each beam (k << 1 | hit), and the car-phase segments: seg_jo int[C]
// (agent << 8 | box), seg_rg int4[C] (three beam ranges lo | count << 16, total),
// seg_bx int4[C] (the box); C = G * cmax, cmax = the most
// candidate boxes one agent can have (every other ego, plus the NPC slots).
// The road march's queue of unfinished beams, ushort[G*R], is only live
// before the car phase and shares the segment area.

// Probes tested per step of the road march (phase 1's first probes after a beam's
// safe stretch from the car centre, and each pooled iteration).
#ifndef MEV_LIDAR_NPR
#define MEV_LIDAR_NPR 2
#endif
constexpr int LIDAR_NPR = MEV_LIDAR_NPR;
// The march's tail (the queue empty, the few longest beams still running, lanes
// mostly idle): once at most kMarchHelp beams run, each gets a group of 2-8 lanes
// that test kNptHelp consecutive probes each per step (config 3 39.4 -> 35.6 us,
// config 2 19.4 -> 15.6 us; in the traffic kernel +0.6 %).  Measured around it: a
// plain tail with 6 probes per lane and step (38.0 / 18.1 us), groups from 8 or 32
// beams, 2 or 4 probes per helper lane.  k_lidar marches plainly.
constexpr int kMarchHelp = 16;
constexpr int kNptHelp = 3;
static_assert(kMarchHelp <= 32, "helper groups have at least 2 lanes");

struct LidarLayout {
    int ag, dir, res, seg_jo, seg_rg, seg_bx, queue, scr, bytes;
};

__host__ __device__ inline int lidar_cand_max(const SimParams& p) { return p.N - 1 + (p.traffic ? p.K : 0); }

// with_bx: a per-segment copy of the obstacle box (k_lidar, whose boxes are in
// HBM); k_step reads them from its own LDS obstacle table instead.
// beams: capacity of the beam arrays (>= G * R).
__host__ __device__ constexpr LidarLayout lidar_layout_beams(int G, int beams, int cmax, bool with_bx) {
    LidarLayout L{};
    const int C = G * cmax;
    int off = 0;
    L.ag = off; off += G * 16;
    L.dir = off; off += beams * 8;
    L.res = off; off += beams * 4;
    off = (off + 15) & ~15;
    L.seg_rg = off; off += C * 16;
    L.seg_bx = off; off += with_bx ? C * 16 : 0;
    L.seg_jo = off; off += C * 4;
    L.queue = L.seg_rg;
    if (off < L.queue + beams * 2) off = L.queue + beams * 2;
    off = (off + 15) & ~15;
    L.scr = off; off += WAVE * 4;  // the car phase's segment lookup (3c)
    L.bytes = (off + 15) & ~15;
    return L;
}
__host__ __device__ inline LidarLayout lidar_layout(int G, int R, int cmax, bool with_bx = true) {
    return lidar_layout_beams(G, G * R, cmax, with_bx);
}

int lidar_group(int R) {
    // ~256 beams per wave pool: G = 4 agents at R = 64 (measured best of 1..16, tools/kernel_time.py)
    int g = 256 / (R > 0 ? R : 1);
    return g < 1 ? 1 : (g > 64 ? 64 : g);
}

// Where the LiDAR body reads each agent's pose and the obstacle table from:
// HBM as k_cars published it (k_lidar), or the LDS of the same wave's
// cars_body (k_step).
struct LidarSrcHbm {
    static constexpr bool kBoxLds = false;  // boxes come from HBM: cache one per segment in LDS
    const SimParams& p;
    __device__ float rel(int b) const { return gmem(p.rel_angles)[b]; }
    __device__ bool alive(int g) const { return gmem(p.ego.alive)[g] != 0; }
    __device__ float4 pose(int g) const { return make_float4(egof(p, EF_X)[g], egof(p, EF_Y)[g], egof(p, EF_H)[g], __int_as_float(g)); }
    __device__ void cand(int g, unsigned long long& c0, unsigned long long& c1) const {
        c0 = gmem(p.ob_cand)[2 * g];
        c1 = gmem(p.ob_cand)[2 * g + 1];
    }
    __device__ int4 box(int g, int o) const { return p.ob_box[(size_t)(g / p.N) * p.ob_stride + o]; }
};
struct LidarSrcLds {
    static constexpr bool kBoxLds = true;  // the obstacle table is in this wave's LDS
    const CarsLDS& el;
    int g0;  // global index of the env's agent 0
    __device__ float rel(int b) const { return el.rel[b]; }
    __device__ bool alive(int g) const { return el.alive[g - g0] != 0; }
    __device__ float4 pose(int g) const {
        const int i = g - g0;
        return make_float4(el.x[i], el.y[i], el.h[i], __int_as_float(g));
    }
    __device__ void cand(int g, unsigned long long& c0, unsigned long long& c1) const {
        c0 = el.cand[2 * (g - g0)];
        c1 = el.cand[2 * (g - g0) + 1];
    }
    __device__ int4 box(int, int o) const { return el.box[o]; }
};
// The LiDAR wave of the traffic early split: ENVS envs of one ego each, env j's
// car LDS (carved at base + j * reg bytes, the obstacle table of that env) and
// one beam-offset array; an agent's env is found from its global index (N = 1:
// the env index), so the phase-3 pairs of different envs share the 64 lanes.
template <int ENVS>
struct LidarSrcLdsEnvs {
    static constexpr bool kBoxLds = true;  // the obstacle tables are in this workgroup's LDS
    const CarsLDS& el0;  // env 0's arrays
    int reg;             // bytes between two envs' car LDS
    const float* relp;
    int env[ENVS];       // the workgroup's envs (wave-uniform)
    __device__ int off(int g) const {
        int j = 0;
#pragma unroll
        for (int u = 1; u < ENVS; ++u) j = g == env[u] ? u : j;
        return j * reg;
    }
    template <class T>
    __device__ const T* at(const T* p0, int g) const {
        return reinterpret_cast<const T*>(reinterpret_cast<const unsigned char*>(p0) + off(g));
    }
    __device__ float rel(int b) const { return relp[b]; }
    __device__ bool alive(int g) const { return at(el0.alive, g)[0] != 0; }
    __device__ float4 pose(int g) const {
        return make_float4(at(el0.x, g)[0], at(el0.y, g)[0], at(el0.h, g)[0], __int_as_float(g));
    }
    __device__ void cand(int g, unsigned long long& c0, unsigned long long& c1) const {
        const unsigned long long* c = at(el0.cand, g);
        c0 = c[0];
        c1 = c[1];
    }
    __device__ int4 box(int g, int o) const { return at(el0.box, g)[o]; }
};

// Lidar::update (Lidar.cpp:16-90) + Lidar::normalized for the agents
// [a0, a0 + na) (na <= G) of one wave; base/lay: the wave's LDS.  Phase 1
// computes the beam directions in lockstep; phase 2 marches the road with
// the group's beams fed to the 64 lanes from a queue, so a lane that
// finishes a short beam takes the next one instead of idling until the
// longest beam of its agent is done (lockstep cost = max over the agent's
// beams, pooled cost ~ their mean); phase 3 resolves the cars as packed
// (agent, box, beam) pairs and writes the observation's LiDAR block.
//
// PART (k_step's early split, the LiDAR wave of a two-wave workgroup): 1 = phases 1-2
// (the road march) only, from the poses the car wave staged in ag[] after the
// kinematics; 2 = phases 1-2 again for the compacted agents in `redo` (egos the car
// part respawned since; the caller has put their new poses in ag[]), then phase 3
// and the block writes.  0 = everything.
#ifndef MEV_DENSE_ILP
#define MEV_DENSE_ILP 2
#endif
// P1 = 1: R is a multiple of 64 (the dense phase-1 walk below is not compiled in); P1 = 2: R is
// not (the dense walk for every pool, the agent-pair loop not compiled in); P1 >= 64: R = P1, a
// compile-time beam count (64: config 3, 96: the reference's default LiDAR, 128: config 5).
template <bool TAB, int ILP, class Src, int NPT = LIDAR_NPR, bool HELP = false, int PART = 0, int P1 = 0>
__device__ __forceinline__ void lidar_body(const SimParams& p, const Outputs& out, const Src& src, const int G,
                                           const int a0, const int na, const int lane, unsigned char* base,
                                           const LidarLayout& lay, const unsigned long long redo = 0ull,
                                           const unsigned long long alive_in = 0ull) {
    const int R = P1 >= WAVE ? P1 : p.R;  // (P1 >= 64: exactly that many beams, a compile-time count)
    const int LS = P1 >= WAVE ? P1 : p.lidar_slots;  // (and every beam in the observation: fixed_r)
    float4* ag = reinterpret_cast<float4*>(base + lay.ag);
    float2* dir = reinterpret_cast<float2*>(base + lay.dir);
    int* res = reinterpret_cast<int*>(base + lay.res);
#if defined(MEV_STAMPS_R)  // slots 3/4: entry of the env's first/second pool; 5/6: their car-phase end
    const int se_ = a0 / p.N, sp_ = ((a0 % p.N) / G) & 1;
    if (lane == 0) p.debug[se_ * 8 + 3 + sp_] = __builtin_amdgcn_s_memrealtime();
#endif

    // ---- phase 1: alive agents of the group (compacted), beam directions
    // (PART 1/2: the alive agents as the caller computed them -- in the early split
    // the LiDAR wave starts before the car wave has staged the state)
    bool alv = false;
    if (PART != 0) alv = (alive_in >> lane) & 1ull;
    else if (lane < na) alv = src.alive(a0 + lane);
    const unsigned long long am = PART != 0 ? alive_in : ballot(alv);
    const int nal = __popcll(am);
    if (PART == 0 && alv) {  // (PART 1/2: staged by the car wave / the caller)
        const int g = a0 + lane;
        ag[lane_rank(am)] = src.pose(g);
    }
    if (PART != 2 && __popcll(am) != na) {  // dead agents: LiDAR block of the observation is zero (:425-427)
        for (int j = 0; j < na; ++j) {
            if ((am >> j) & 1ull) continue;
            if (out.lidar_u8) {  // compact gather format: the dead-agent code
                uint8_t* crow = out.lidar_u8 + (size_t)(a0 + j) * LS;
                for (int b = lane; b < LS; b += WAVE) crow[b] = (uint8_t)kLidarCodeDead;
                continue;
            }
            float* row = out.obs + (size_t)(a0 + j) * out.obs_ld + OBS_HEAD;
            for (int b = lane; b < LS; b += WAVE) row[b] = 0.0f;
        }
    }
    wave_lds_sync();
    const float stp = p.lidar_step;
    const int S = p.lidar_steps;
    const float rwf = (float)p.irw;
    const float inv_stp = __builtin_amdgcn_rcpf(stp);
    const float crf = CORNER_RADIUS, ccen = rwf + crf;
    const float cr2p1 = crf * crf + 1.0f;
    const float rwm = rwf - 1.5f;
    // the reference's stop test of march probe k at (cx_, cy_) + d_k (dx_, dy_):
    // returns the beam's result (k << 1 | hit; S << 1 past the last probe) or -1
    // to go on, and the probe's real point
    auto probe = [&](float cx_, float cy_, float dx_, float dy_, int k_, float& fx, float& fy) -> int {
        const bool past = k_ >= S;
        const int kc = past ? S - 1 : k_;
        const float d = TAB ? gmem(p.dist_tab)[kc] : (float)kc * stp;
        fx = cx_ + dx_ * d;
        fy = cy_ + dy_ * d;
        const int px = (int)fx, py = (int)fy;
        // exact reference predicates at the truncated pixel: screen, then
        // (k > 0) road == RoadGeometry::is_on_road at integer pixels:
        //   on_road <=> dist^2 to the grass-disc centre >= cr^2 + 1
        //               and (in a strip: min(ax, ay) <= rw  or  corner square: max <= rw + cr)
        const unsigned pmax = (unsigned)px > (unsigned)py ? (unsigned)px : (unsigned)py;
        const bool off_screen = pmax >= (unsigned)WIDTH;
        const float iax = fabs_f((float)(px - 375)), iay = fabs_f((float)(py - 375));
        const float qdx = iax - ccen, qdy = iay - ccen;
        const float onv = fmaxf(fminf(fminf(iax, iay) - rwf, fmaxf(iax, iay) - ccen), cr2p1 - (qdx * qdx + qdy * qdy));
        const bool stop = off_screen | ((k_ > 0) & (onv > 0.0f));
        const int code = lidar_keep(stop ? ((k_ << 1) | (off_screen ? 0 : 1)) : -1);
        return past ? (S << 1) : code;
    };
    // probes k_ .. k_ + NPR - 1 in march order: the first stop wins; (fx, fy) is
    // the last probe's point
    auto probes_n = [&](auto np, float cx_, float cy_, float dx_, float dy_, int k_, float& fx, float& fy) -> int {
        int r = -1;
#pragma unroll
        for (int t = 0; t < decltype(np)::value; ++t) {
            const int c = probe(cx_, cy_, dx_, dy_, k_ + t, fx, fy);
            r = r >= 0 ? r : c;
        }
        return r;
    };
    auto probes = [&](float cx_, float cy_, float dx_, float dy_, int k_, float& fx, float& fy) -> int {
        return probes_n(std::integral_constant<int, LIDAR_NPR>{}, cx_, cy_, dx_, dy_, k_, fx, fy);
    };

    // directions; then the first probes of each beam: probe 0 is only
    // screen-tested (no road test at dist 0); if the car centre is on screen,
    // every probe within the safe distance from it is skipped, and the next
    // LIDAR_NPR probes are tested right here — most beams stop among them (the
    // edge of the road lies within a few steps of the provably safe stretch).
    // Beams still running go to the queue of the pooled march.
    unsigned short* queue = reinterpret_cast<unsigned short*>(base + lay.queue);
    int qn = 0;
    // beam offsets rel[b] of the first two chunks of 64 beams, loaded once:
    // a global load inside the loop would expose its latency every iteration
    const float rel_c0 = lane < R ? src.rel(lane) : 0.0f;
    const float rel_c1 = lane + WAVE < R ? src.rel(lane + WAVE) : 0.0f;
    // one beam: direction (Lidar.cpp:24-26) and the first probes; returns the
    // beam's result (>= 0) or -(next probe to test) - 1
    // (uni, wave-uniform: every lane's beam starts from the same car centre -- the
    // wave-uniform safe bound; else a chunk holding two agents' beams)
    auto setup = [&](const float4& a, float rel_b, auto small, float2& d, bool uni) -> int {
        float sn, cs;
#if defined(MEV_EXP_FASTSIN)  // timing-only (wrong results): phase 1's beam directions by the hardware sin/cos
        sn = __sinf(a.z + rel_b);
        cs = __cosf(a.z + rel_b);
        (void)small;
#else
        if constexpr (decltype(small)::value) sincosf_below120(a.z + rel_b, &sn, &cs);
        else sincosf(a.z + rel_b, &sn, &cs);
#endif
        const float dx = cs, dy = -sn;
        d = make_float2(dx, dy);
        const int px = (int)a.x, py = (int)a.y;
        const unsigned pmax = (unsigned)px > (unsigned)py ? (unsigned)px : (unsigned)py;
        const float idx = __builtin_amdgcn_rcpf(dx), idy = __builtin_amdgcn_rcpf(dy);
        float safe;
        if (uni)
            safe = road_safe_uniform(a.x, a.y, dx, dy, idx, idy, fabs_f(idx), fabs_f(idy), rwm, ccen, crf);
        else
            safe = road_safe(a.x, a.y, dx, dy, idx, idy, fabs_f(idx), fabs_f(idy), rwm, ccen, crf);
        // probes 1 .. j lie within j*step <= safe of the centre (car centre on screen)
        const int k1 = pmax < (unsigned)WIDTH ? 1 + safe_steps(safe, stp, inv_stp) : 0;
        float fx, fy;
        const int r = probes_n(std::integral_constant<int, LIDAR_NPR>{}, a.x, a.y, dx, dy, k1, fx, fy);
        return r >= 0 ? r : -(k1 + LIDAR_NPR) - 1;
    };
    // one pass of the early split's re-march: compacted agent j (PART 2)
    auto pass1_one = [&](auto small, const int j) {
        const float4 a = ag[j];
        for (int b0 = 0; b0 < R; b0 += WAVE) {
            const int b = b0 + lane;
            const bool vb = b < R;
            const float rel_b = b0 == 0 ? rel_c0 : (b0 == WAVE ? rel_c1 : (vb ? src.rel(b) : 0.0f));
            float2 d;
            const int r = setup(a, rel_b, small, d, true);
            if (vb) {
                dir[j * R + b] = d;
                res[j * R + b] = r >= 0 ? r : -r - 1;
            }
            const bool pend = vb && r < 0;
            const unsigned long long m = ballot(pend);
            if (pend) queue[qn + lane_rank(m)] = (unsigned short)(j * R + b);
            qn += __popcll(m);
        }
    };
    // ILP = 2: two agents per pass, two independent dependency chains (sincosf's
    // double polynomial, the safe distance, the probes) the compiler interleaves
    // (k_step, 128 VGPRs); ILP = 1 in k_lidar, whose 64-VGPR budget would spill.
    // R not a multiple of 64 (several agents): the dense layout instead -- the pool's
    // nal*R beams as consecutive 64-lane chunks, an agent's beams running on into the
    // next chunk, ILP chunks per pass; R = 96 takes 6 chunks per 4 agents, not 8
    // half-empty ones.  (One loop for both measured 2 % slower at config 3: the chunk
    // walk's bookkeeping and the offsets' LDS reads in front of every pass.)
    const bool dense = P1 >= WAVE ? (P1 & (WAVE - 1)) != 0 : (P1 == 2 || (P1 == 0 && (R & (WAVE - 1)) != 0 && nal > 1));
    auto phase1 = [&](auto small) {
        if constexpr (PART == 2) {  // the respawned agents only
            for (unsigned long long tm = redo; tm; tm &= tm - 1ull) pass1_one(small, __builtin_ctzll(tm));
        } else if (dense) {
            const float invRp = 1.0f / (float)R;
            const int nq = nal * R;
            constexpr int DI = ILP > 1 ? MEV_DENSE_ILP : 1;
            for (int c0 = 0; c0 < nq; c0 += DI * WAVE) {
                if (PART == 0 && 4 * c0 >= nq) __builtin_amdgcn_s_setprio(kPrioP1B);
                int q[DI];
                float4 a[DI];
                float rb[DI];
#pragma unroll
                for (int u = 0; u < DI; ++u) {
                    q[u] = c0 + u * WAVE + lane;
                    const int qc = q[u] < nq ? q[u] : nq - 1;
                    const int j = (int)(((float)qc + 0.5f) * invRp);  // exact (see load_beam)
                    a[u] = ag[j];
                    rb[u] = src.rel(qc - j * R);
                }
                float2 d[DI];
                int r[DI];
#pragma unroll
                for (int u = 0; u < DI; ++u) r[u] = setup(a[u], rb[u], small, d[u], false);
#pragma unroll
                for (int u = 0; u < DI; ++u) {
                    const bool vq = q[u] < nq;
                    if (vq) {
                        dir[q[u]] = d[u];
                        res[q[u]] = r[u] >= 0 ? r[u] : -r[u] - 1;  // result, or the next probe to test
                    }
                    const bool pend = vq && r[u] < 0;
                    const unsigned long long m = ballot(pend);
                    if (pend) queue[qn + lane_rank(m)] = (unsigned short)q[u];
                    qn += __popcll(m);
                }
            }
        } else {
        for (int j = 0; j < nal; j += ILP) {
            if (PART == 0 && 4 * j >= nal) __builtin_amdgcn_s_setprio(kPrioP1B);
            float4 a[ILP];
#pragma unroll
            for (int u = 0; u < ILP; ++u) a[u] = ag[j + u < nal ? j + u : j];
            for (int b0 = 0; b0 < R; b0 += WAVE) {
                const int b = b0 + lane;
                const bool vb = b < R;
                const float rel_b = b0 == 0 ? rel_c0 : (b0 == WAVE ? rel_c1 : (vb ? src.rel(b) : 0.0f));
                float2 d[ILP];
                int r[ILP];
#pragma unroll
                for (int u = 0; u < ILP; ++u) r[u] = setup(a[u], rel_b, small, d[u], true);
#pragma unroll
                for (int u = 0; u < ILP; ++u) {
                    const bool in = j + u < nal;  // wave-uniform
                    if (vb && in) {
                        dir[(j + u) * R + b] = d[u];
                        res[(j + u) * R + b] = r[u] >= 0 ? r[u] : -r[u] - 1;  // result, or the next probe to test
                    }
                    const bool pend = vb && in && r[u] < 0;
                    const unsigned long long m = ballot(pend);
                    if (pend) queue[qn + lane_rank(m)] = (unsigned short)((j + u) * R + b);
                    qn += __popcll(m);
                }
            }
        }
        }
    };
    // |heading| < 100 for every agent (always, unless set_state() planted a
    // wild heading): |h + rel| < 120, the range of the branch-free sincosf
    const bool hsmall = ballot(lane < nal && !(fabs_f(ag[lane < nal ? lane : 0].z) < 100.0f)) == 0ull;
    if (ILP > 1 && hsmall) phase1(std::true_type{});  // k_lidar: one instantiation (64 VGPRs)
    else phase1(std::false_type{});
    wave_lds_sync();
#if defined(MEV_EXP_STOP) && MEV_EXP_STOP == 2  // timing-only: stop after phase 1
    if (Src::kBoxLds) return;
#endif
#if defined(MEV_STAMPS_R)  // one pool per env: slot 4 = end of phase 1
    if (lane == 0 && na == p.N) p.debug[se_ * 8 + 4] = __builtin_amdgcn_s_memrealtime();
#endif

    if (PART == 0) __builtin_amdgcn_s_setprio(kPrioP2);
#if defined(MEV_EXP_TSNOMARCH)  // timing-only (wrong results): the early splits' first part without its march
    if constexpr (PART == 1) return;
#endif
    // ---- phase 2: pooled road + screen march of the queued beams
    // (Lidar.cpp:31-48, first stop wins): LIDAR_NPR exact probes, then a jump
    // over the provably safe stretch after the last one
    // (one beam per lane: measured, a second interleaved beam per lane doubles
    // the per-iteration cost while the long beams still set the trip count)
    const float invR = 1.0f / (float)R;
    int next = qn < WAVE ? qn : WAVE;
    int slot = lane < qn ? (int)queue[lane] : -1;
    float cx = 0.0f, cy = 0.0f, dx = 0.0f, dy = 0.0f, idx = 0.0f, idy = 0.0f, iadx = 0.0f, iady = 0.0f;
    int k = 0;
    auto load_beam = [&](int qq) {
        // agent of beam slot qq = j*R + b: exact float quotient (qq < 2^20, R <= 1024)
        const int j = (int)(((float)qq + 0.5f) * invR);
        const float4 a = ag[j];
        const float2 d = dir[qq];
        cx = a.x; cy = a.y; dx = d.x; dy = d.y;
        idx = __builtin_amdgcn_rcpf(dx);
        idy = __builtin_amdgcn_rcpf(dy);
        iadx = fabs_f(idx);
        iady = fabs_f(idy);
        k = res[qq];
    };
    if (slot >= 0) load_beam(slot);
    int* hscr = reinterpret_cast<int*>(base + lay.scr);  // phase 3's scratch, free until then
    bool help = false;
    while (ballot(slot >= 0) != 0ull) {
        // the tail down to <= 16 beams: continue with 4 lanes per beam (below)
        if (HELP && next >= qn && __popcll(ballot(slot >= 0)) <= kMarchHelp) {
            help = true;
            break;
        }
        // branch-free body: every lane evaluates its probes; idle lanes only skip the store
        const bool act = slot >= 0;
        float fx, fy;
        int r, npr = LIDAR_NPR;
        if (NPT != LIDAR_NPR && next >= qn) {  // wave-uniform: the queue is empty
            r = probes_n(std::integral_constant<int, NPT>{}, cx, cy, dx, dy, k, fx, fy);
            npr = NPT;
        } else {
            r = probes(cx, cy, dx, dy, k, fx, fy);
        }
        const float safe = road_safe(fx, fy, dx, dy, idx, idy, iadx, iady, rwm, ccen, crf);
        // probes kl+1 .. kl+j lie within j*step <= safe of the last probe kl = k + npr - 1
        const int kn = k + npr + safe_steps(safe, stp, inv_stp);
        const bool fin = act & ((r >= 0) | (kn >= S));
        if (fin) res[slot] = r >= 0 ? r : (S << 1);
        k = kn;
        const unsigned long long fm = ballot(fin);
        if (fm != 0ull) {
            if (fin) {
                const int nq = next + lane_rank(fm);
                slot = nq < qn ? (int)queue[nq] : -1;
                if (slot >= 0) load_beam(slot);
            }
            next += __popcll(fm);
        }
    }
    if (HELP && help) {
        // The last running beams (<= kMarchHelp), GS lanes each (GS = 64 / the
        // beams rounded up to a power of two, 2..8): lane j of a beam's group tests
        // probes k + j*NPH .. k + (j+1)*NPH - 1, the earliest stop of the group wins
        // (results are ordered by k: DPP min), and the group jumps from its last lane's
        // last probe (DPP broadcast) -- the same probes and jumps, in march order.
        constexpr int NPH = kNptHelp;
        const unsigned long long am = ballot(slot >= 0);
        const int nb = __popcll(am);
        if (slot >= 0) {
            const int rk = lane_rank(am);
            hscr[2 * rk] = slot;
            hscr[2 * rk + 1] = k;
        }
        wave_lds_sync();
        auto group_march = [&](auto gs_c) {
            constexpr int GS = decltype(gs_c)::value;
            const int gi = lane / GS, j = lane & (GS - 1);
            slot = gi < nb ? hscr[2 * gi] : -1;
            const int k_h = gi < nb ? hscr[2 * gi + 1] : 0;
            if (slot >= 0) load_beam(slot);
            k = k_h;
            while (ballot(slot >= 0) != 0ull) {
                float fx, fy;
                const int k0 = k + j * NPH;
                int r = probes_n(std::integral_constant<int, NPH>{}, cx, cy, dx, dy, k0, fx, fy);
                r = r >= 0 ? r : 0x7fffffff;
                const float safe = road_safe(fx, fy, dx, dy, idx, idy, iadx, iady, rwm, ccen, crf);
                int kn = k0 + NPH + safe_steps(safe, stp, inv_stp);
                r = min(r, __builtin_amdgcn_mov_dpp(r, 0xB1, 0xf, 0xf, false));  // quad_perm [1,0,3,2]
                if constexpr (GS == 2) {
                    kn = __builtin_amdgcn_mov_dpp(kn, 0xF5, 0xf, 0xf, false);  // quad_perm [1,1,3,3]
                } else {
                    r = min(r, __builtin_amdgcn_mov_dpp(r, 0x4E, 0xf, 0xf, false));  // quad_perm [2,3,0,1]
                    kn = __builtin_amdgcn_mov_dpp(kn, 0xFF, 0xf, 0xf, false);        // quad_perm [3,3,3,3]
                    if constexpr (GS == 8) {
                        // the other quad's minimum and lane 7's jump by the half-row mirror
                        r = min(r, __builtin_amdgcn_mov_dpp(r, 0x141, 0xf, 0xf, false));
                        const int km = __builtin_amdgcn_mov_dpp(kn, 0x141, 0xf, 0xf, false);
                        kn = j < 4 ? km : kn;
                    }
                }
                const bool fin = slot >= 0 && (r != 0x7fffffff || kn >= S);
                if (fin && j == 0) res[slot] = r != 0x7fffffff ? r : (S << 1);
                slot = fin ? -1 : slot;
                k = kn;
            }
        };
        if (nb <= 8) group_march(std::integral_constant<int, 8>{});
        else if (nb <= 16) group_march(std::integral_constant<int, 4>{});
        else group_march(std::integral_constant<int, 2>{});
    }
    wave_lds_sync();
    if constexpr (PART == 1) return;  // the early split's road march: phase 3 after the car part
#if defined(MEV_EXP_STOP) && MEV_EXP_STOP == 3  // timing-only: stop after phase 2
    if (Src::kBoxLds) return;
#endif
#if defined(MEV_STAMPS_R)  // one pool per env: slot 6 = end of phase 2
    if (lane == 0 && na == p.N) p.debug[se_ * 8 + 6] = __builtin_amdgcn_s_memrealtime();
#endif

    __builtin_amdgcn_s_setprio(kPrioP3);
    // ---- phase 3: cars (Lidar.cpp:50-80) as a list of (agent, box, beam) pairs.
    // A box can only stop the beams whose ray enters its slab box, i.e. the
    // beams inside the angular span of its real slab box seen from the agent:
    // 3a lists (agent, candidate box) segments, 3b turns each into beam ranges,
    // 3c packs the pairs of all the group's agents into the 64 lanes (scan + segment lookup)
    // and resolves each by exact probes inside its slab range, keeping the
    // earliest stop per beam with an LDS atomicMin on (k << 1 | hit); 3d writes
    // the LiDAR block.
    int* seg_jo = reinterpret_cast<int*>(base + lay.seg_jo);
    int4* seg_rg = reinterpret_cast<int4*>(base + lay.seg_rg);
    int4* seg_bx = reinterpret_cast<int4*>(base + lay.seg_bx);
    int* scr = reinterpret_cast<int*>(base + lay.scr);
    int M = 0;
    // 3a: lane j < nal fetches agent j's candidate masks once; the loop then
    // reads them with readlane instead of two dependent LDS round trips per agent
    unsigned long long cl0 = 0ull, cl1 = 0ull;
    if (lane < nal) src.cand(__float_as_int(ag[lane].w), cl0, cl1);
    for (int j = 0; j < nal; ++j) {
        const unsigned long long c0 = readlane64(cl0, j), c1 = readlane64(cl1, j);
        const int n0 = __popcll(c0);
        if ((c0 >> lane) & 1ull) seg_jo[M + lane_rank(c0)] = (j << 8) | lane;
        if ((c1 >> lane) & 1ull) seg_jo[M + n0 + lane_rank(c1)] = (j << 8) | (lane + WAVE);
        M += n0 + __popcll(c1);
    }
    wave_lds_sync();
    // 3b: beam ranges.  Beam b points along h + rel[b], rel[b] = rel[0] + b*dphi;
    // the range covers the angular span of the box's real slab (box_lo/box_hi):
    // a ray outside it never meets the slab, so none of its probes can land in
    // the box.
    const float rel0 = src.rel(0);
    const bool all_beams = R == 1 || !p.beam_cull;  // (no linear model of the offsets: SimParams::beam_cull)
    const float dphi = R > 1 ? (src.rel(R - 1) - rel0) / (float)(R - 1) : 1.0f;
    const float idphi = 1.0f / dphi;
    const float period = 6.28318531f * idphi;  // beam indices per revolution
    for (int m = lane; m < M; m += WAVE) {
        const int jo = seg_jo[m];
        const float4 a = ag[jo >> 8];
        const int4 bx = src.box(__float_as_int(a.w), jo & 255);
        if (!Src::kBoxLds) seg_bx[m] = bx;
        const float ex0 = box_lo(bx.x), ex1 = box_hi(bx.y);
        const float ey0 = box_lo(bx.z), ey1 = box_hi(bx.w);
        int4 rg;
        if (all_beams || (a.x >= ex0 && a.x <= ex1 && a.y >= ey0 && a.y <= ey1)) {  // (on its edge too)
            rg = make_int4(0 | (R << 16), 0, 0, R);  // inside the widened box: every beam
        } else {
            // the box's silhouette seen from the agent (outside it): the two corners
            // that bound its angular span -- the near side's ends when the agent faces
            // a side, else the corners across the diagonal the agent does not lie on
            const bool lx = a.x < ex0, hx = a.x > ex1, ly = a.y < ey0, hy = a.y > ey1;
            const bool mx = !lx && !hx, my = !ly && !hy;
            const float Xa = my ? (lx ? ex0 : ex1) : (mx ? ex0 : ((lx == ly) ? ex1 : ex0));
            const float Ya = my ? ey0 : (mx ? (ly ? ey0 : ey1) : ey0);
            const float Xb = my ? Xa : (mx ? ex1 : ((lx == ly) ? ex0 : ex1));
            const float Yb = my ? ey1 : (mx ? Ya : ey1);
            // (relative to the direction of the box centre, as with four corners: both
            // lie within +-pi/2 of it even when the agent nearly touches the box)
            const float phc = atan2_fast(-(0.5f * (ey0 + ey1) - a.y), 0.5f * (ex0 + ex1) - a.x);
            const float da = wrap_pi_fast(atan2_fast(-(Ya - a.y), Xa - a.x) - phc);
            const float db = wrap_pi_fast(atan2_fast(-(Yb - a.y), Xb - a.x) - phc);
            const float dmin = fminf(0.0f, fminf(da, db)), dmax = fmaxf(0.0f, fmaxf(da, db));
            float w = phc + dmin - a.z - rel0;
            w -= 6.28318531f * floorf(w * 0.159154943f);  // [0, 2*pi)
            // beams b with rel0 + b*dphi in the span, widened by 2e-4 rad (20x the
            // error of atan2_fast and of the linear model of the host's angles)
            const float marg = 2.0e-4f;
            const float ulo = (w - marg) * idphi, uhi = (w + (dmax - dmin) + marg) * idphi;
            int lo[3], cn[3];
#pragma unroll
            for (int sft = 0; sft < 3; ++sft) {
                const float sh = (float)(sft - 1) * period;
                int l0 = (int)ceilf(ulo + sh), l1 = (int)floorf(uhi + sh);
                l0 = l0 < 0 ? 0 : l0;
                l1 = l1 > R - 1 ? R - 1 : l1;
                lo[sft] = l0;
                cn[sft] = l1 >= l0 ? l1 - l0 + 1 : 0;
            }
            rg = make_int4(lo[0] | (cn[0] << 16), lo[1] | (cn[1] << 16), lo[2] | (cn[2] << 16), cn[0] + cn[1] + cn[2]);
        }
        seg_rg[m] = rg;
    }
    wave_lds_sync();
    // 3c: the pairs of all the group's agents packed into the 64 lanes
    for (int cb = 0; cb < M; cb += WAVE) {
        const int nseg = M - cb < WAVE ? M - cb : WAVE;
        const int cnt = lane < nseg ? seg_rg[cb + lane].w : 0;
        const int incl = wave_scan_add(cnt);  // DPP, no LDS round trips
        const int excl = incl - cnt;
        const int T = __builtin_amdgcn_readlane(incl, WAVE - 1);
        int carry = 0;  // (start << 8 | segment) of the segment running into this chunk
        for (int q0 = 0; q0 < T; q0 += WAVE) {
            const int q = q0 + lane;
            // segment of pair q: the last m with excl[m] <= q.  Each segment that
            // starts in this chunk writes (start << 8 | m) + 1 to the LDS slot of
            // its start; a max-scan spreads it over the segment's lanes (starts
            // increase with m, so the max is the latest); one LDS round trip
            // instead of a chain of lane shuffles.
            const bool starts = cnt > 0 && excl >= q0 && excl < q0 + WAVE;
            scr[lane] = 0;
            wave_lds_sync();  // lanes' writes to the same slot: the zeroing must not sink past the scatter
            if (starts) scr[excl - q0] = ((excl << 8) | lane) + 1;
            wave_lds_sync();
            const int got = wave_scan_max(scr[lane]);
            wave_lds_sync();  // the next chunk rewrites scr
            const int cur = got > 0 ? got - 1 : carry;
            carry = __builtin_amdgcn_readlane(cur, WAVE - 1);
            const int sm = cur & 255;
            const int r = q - (cur >> 8);
            if (q < T) {
                const int m = cb + sm;
                const int j = seg_jo[m] >> 8;
                const float4 a = ag[j];
                const int4 rg = seg_rg[m];
                const int4 bx = Src::kBoxLds ? src.box(__float_as_int(a.w), seg_jo[m] & 255) : seg_bx[m];
                const int cA = rg.x >> 16, cB = rg.y >> 16;
                const int b = r < cA ? (rg.x & 0xffff) + r
                                     : (r < cA + cB ? (rg.y & 0xffff) + r - cA : (rg.z & 0xffff) + r - cA - cB);
                const int slot = j * R + b;
                const int kr = res[slot] >> 1;
                const float2 dd = dir[slot];
                // probes that can land in the box: the ray's interval inside the
                // box's real slab (see box_lo), as a superset range of k ...
                float lo = 0.0f, hi = 1.0e6f;
                slab_clip(a.x, dd.x, __builtin_amdgcn_rcpf(dd.x), box_lo(bx.x), box_hi(bx.y), lo, hi);
                slab_clip(a.y, dd.y, __builtin_amdgcn_rcpf(dd.y), box_lo(bx.z), box_hi(bx.w), lo, hi);
                // d_k = k*step exactly without the table: the slab's 0.01 px absorbs the
                // rounding of k = lo/step; the table's accumulated distances get one probe
                int ka, kb;
                if (TAB) {
                    ka = (int)(fmaxf(lo, 0.0f) * inv_stp) - 1;
                    kb = (int)(fminf(hi, 1.0e6f) * inv_stp) + 1;
                } else {
                    ka = (int)ceilf(fmaxf(lo, 0.0f) * inv_stp);
                    kb = (int)(fminf(hi, 1.0e6f) * inv_stp);
                }
                ka = ka < 1 ? 1 : ka;  // no car test at dist == 0
                kb = kb < kr - 1 ? kb : kr - 1;
                if (lo > hi) kb = 0;
                // ... resolved by exact probes in march order
                for (int kk = ka; kk <= kb; ++kk) {
                    // a runtime table test here, not march_dist<TAB>: measured 4 us per
                    // step faster in k_step, and without it k_lidar's 64-VGPR
                    // allocation spills ~180 registers
                    const float d = p.dist_tab ? gmem(p.dist_tab)[kk] : (float)kk * p.lidar_step;
                    const int px = (int)(a.x + dd.x * d), py = (int)(a.y + dd.y * d);
                    if (px >= bx.x && px <= bx.y && py >= bx.z && py <= bx.w) {
                        atomicMin(&res[slot], (kk << 1) | 1);
                        break;
                    }
                }
            }
        }
    }
    wave_lds_sync();
#if defined(MEV_STAMPS_R)
    if (lane == 0) p.debug[se_ * 8 + 5 + sp_] = __builtin_amdgcn_s_memrealtime();
#endif
#if defined(MEV_EXP_STOP) && MEV_EXP_STOP == 4  // timing-only: stop after phase 3 (no LiDAR block writes)
    if (Src::kBoxLds) return;
#endif
    // 3d: Lidar::normalized (:92-98), the LiDAR block of each alive agent's row
    if (out.lidar_u8) {  // compact gather format: one code per beam (0 no hit, k + 1 hit at probe k)
        for (int j = 0; j < nal; ++j) {
            const int g = __float_as_int(ag[j].w);
            uint8_t* crow = out.lidar_u8 + (size_t)g * LS;
            for (int b = lane; b < LS; b += WAVE) {
                const int r = res[j * R + b];
                crow[b] = (uint8_t)((r & 1) ? (r >> 1) + 1 : 0);
            }
        }
        return;
    }
    if (LS <= WAVE) {
        // lane = beam: the agents' global indices come from one LDS read (readlane per
        // row) and 8 rows' results are read before any is stored (one LDS wait per 8 rows)
        const int gl = lane < nal ? __float_as_int(ag[lane].w) : 0;
        const bool beam = lane < LS;
        // (the LiDAR constants read once and pinned in VGPRs by one asm: the compiler cannot
        // rematerialize an asm result, so it stops re-issuing their scalar loads for every
        // row -- three dependent scalar-cache round trips per row)
        float l_max = p.lidar_max, l_step = p.lidar_step, l_inv = p.lidar_inv;
        asm volatile("" : "+v"(l_max), "+v"(l_step), "+v"(l_inv));
        auto row_value = [&](int r) {
            const float dk = TAB ? gmem(p.dist_tab)[r >> 1] : (float)(r >> 1) * l_step;
            return ((r & 1) ? dk : l_max) * l_inv;
        };
        for (int j0 = 0; j0 < nal; j0 += 8) {
            int rr[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) rr[u] = (j0 + u < nal && beam) ? res[(j0 + u) * R + lane] : 0;
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                if (j0 + u < nal && beam) {
                    const int g = __builtin_amdgcn_readlane(gl, j0 + u);
                    out.obs[(size_t)g * out.obs_ld + OBS_HEAD + lane] = row_value(rr[u]);
                }
            }
        }
    } else {
        for (int j = 0; j < nal; ++j) {
            const int g = __float_as_int(ag[j].w);
            float* row = out.obs + (size_t)g * out.obs_ld + OBS_HEAD;
            for (int b = lane; b < LS; b += WAVE)
                row[b] = ((res[j * R + b] & 1) ? march_dist<TAB>(p, res[j * R + b] >> 1) : p.lidar_max) * p.lidar_inv;
        }
    }
}

template <bool TAB>
__global__ __launch_bounds__(256, 8) void k_lidar(SimParams p, Outputs out, int G, int a_begin, int a_end) {
    // Each wave owns a group of G agents (G*R <= max(256, R) beams).
    extern __shared__ __align__(16) unsigned char lds_raw[];
    const int lane = threadIdx.x & (WAVE - 1);
    const int wv = threadIdx.x / WAVE;
    const int blk = xcd_env((int)blockIdx.x, (int)gridDim.x);  // neighbouring groups on one XCD
    const int a0 = __builtin_amdgcn_readfirstlane(a_begin + (blk * (int)(blockDim.x / WAVE) + wv) * G);
    if (a0 >= a_end) return;  // wave-uniform exit: the kernel has no block-level barrier
    const int na = a_end - a0 < G ? a_end - a0 : G;
    __builtin_amdgcn_s_setprio(kPrioLidar);
    const LidarLayout lay = lidar_layout(G, p.R, lidar_cand_max(p));
    lidar_body<TAB, 1>(p, out, LidarSrcHbm{p}, G, a0, na, lane, lds_raw + (size_t)wv * (size_t)lay.bytes, lay);
}


// Agents per LiDAR pool in k_step: the env's N agents in the fewest pools of at
// most 512 beams, balanced (all N in one pool at config 3; 8 x 96 beams as 4 + 4
// agents, 384 beams each, not 5 + 3: each pool's march ends on its longest beams,
// and 4 agents of 96 beams fill six whole 64-lane chunks in phase 1).
__host__ __device__ constexpr int step_pool_n(int N, int R) {
    int g = 512 / (R > 0 ? R : 1);
    g = g < 1 ? 1 : g;
    if (g >= N) return N;
    const int pools = (N + g - 1) / g;
    return (N + pools - 1) / pools;
}
__host__ __device__ inline int step_pool(const SimParams& p) { return step_pool_n(p.N, p.R); }

// LDS of one k_step wave: cars LDS, the staged heads [N][31], the beam offsets
// [R], the env flags [8], then the LiDAR pool of step_pool(p) agents.
struct StepLayout {
    int head, rel, envw, lidar, bytes;
};
__host__ __device__ inline StepLayout step_layout(const SimParams& p) {
    StepLayout L;
    int off = (int)lds_al(cars_lds_bytes(p.N, cars_k(p), true));  // (k_step<NM = 0> keeps the car sizes)
    L.head = off;  // (no staged heads: the car part writes its rows' heads itself)
    L.rel = off; off += (int)lds_al((size_t)p.R * 4);
    L.envw = off; off += 32;
    L.lidar = off; off += lidar_layout(step_pool(p), p.R, lidar_cand_max(p), false).bytes;
    L.bytes = off;
    return L;
}

// Compile-time LDS geometry (NM > 0): every array sized for its capacity --
// N <= NM agents, R <= kFixedRays beams per agent, one LiDAR pool of <= 512
// beams, no NPCs -- so each LDS address is a constant offset from the wave's
// base instead of a runtime pointer held in an SGPR.  The ~40 runtime LDS
// pointers of the NM = 0 layout made k_step spill 131 SGPRs into VGPR lanes
// (a v_readlane per reload).
constexpr int kFixedRays = 128;
constexpr int kPoolBeams = 512;
template <int NM, int KM = 0>
struct FixedLayout {
    static_assert(NM >= 1 && NM <= 64, "agents per env");
    static constexpr int beams = NM * kFixedRays < kPoolBeams ? NM * kFixedRays : kPoolBeams;
    static constexpr int cars = (int)lds_al(cars_lds_bytes(NM, KM));
    static constexpr int rel = cars;
    static constexpr int envw = rel + kFixedRays * 4;
    static constexpr int lidar = envw + 32;
    static constexpr LidarLayout lay = lidar_layout_beams(NM, beams, NM - 1 + KM, false);
    static constexpr int bytes = lidar + lay.bytes;
};
template <int NM, int KM>
__host__ __device__ inline StepLayout step_layout_t(const SimParams& p) {
    if constexpr (NM == 0) return step_layout(p);
    else return StepLayout{FixedLayout<NM, KM>::rel, FixedLayout<NM, KM>::rel, FixedLayout<NM, KM>::envw,
                           FixedLayout<NM, KM>::lidar, FixedLayout<NM, KM>::bytes};
}
// the handle's shape fits the compile-time layout of NM agents and (traffic) KM
// NPC slots within a wave's 10 KB LDS share, the NPC arrays included
template <int NM, int KM>
__host__ __device__ inline bool fixed_fits(const SimParams& p) {
    // R <= 128 puts every pool (step_pool agents) within the layout's beams
    const bool npcs = KM == 0 ? !p.traffic : (p.traffic && p.K <= KM);
    const size_t npc_lds = KM == 0 ? 0 : sizeof(NpcLDST<(KM ? KM : 1)>);
    // (a handle with cars of other sizes runs the runtime layout, NM = 0)
    return p.N <= NM && p.R <= kFixedRays && npcs && !p.dims &&
           (size_t)FixedLayout<NM, KM>::bytes + npc_lds <= 10 * 1024;
}

// agents per phase-1 pass in k_step (independent dependency chains interleaved;
// 3 or 4 raise register pressure and lose); 1 in the early split's LiDAR wave
// (8 waves per SIMD)
#ifndef MEV_PHASE1_ILP
#define MEV_PHASE1_ILP 2
#endif
#ifndef MEV_ESPLIT_ILP
#define MEV_ESPLIT_ILP 1
#endif
constexpr int kPhase1Ilp = MEV_PHASE1_ILP;
constexpr int kEsplitIlp = MEV_ESPLIT_ILP;

// The whole step in one wave per env: cars_body, then the LiDAR of the env's
// N agents in pools, from the same wave's LDS.  No HBM hand-off, no second
// launch, and no global store before a later global load (its vmcnt wait would
// drain them); a wave
// whose env finishes its car logic early starts its LiDAR while other waves
// on the SIMD are still in theirs.  The car part runs at a higher issue
// priority: it is the latency-bound critical path of each wave.
// The parameters come through a device-resident copy (pp, refreshed by the
// host only when they change) rather than by value: LLVM loads every kernel
// argument in the entry block, so by value the ~130 dwords of SimParams stay
// live through the whole kernel and the SGPR allocator spills them into VGPR
// lanes (a v_readlane per reload); through the pointer each field is an s_load
// next to its use.
//
// SPLIT (small batches, <= 2048 workgroups: <= 4 waves per SIMD): two waves per
// workgroup share its LDS; wave 0 runs cars_pre, then both pass a barrier and
// wave 1 runs the LiDAR while wave 0 runs cars_post -- the two latency chains
// after the car part overlap instead of following each other.
//
// The NPC-aware deal of the next step (traffic, §3.1c): this env joins its list's
// class for step t + 1 (an env that ended restarts without NPCs after its
// auto-reset).  It runs where the car part ends (measured against the end of
// k_step: no difference, r3_ab_deferwb.txt).
template <bool TRAFFIC>
__device__ __forceinline__ void deal_append(const SimParams& p, const StepInputs& in, const CarsCtx& cx, const int e) {
    if constexpr (TRAFFIC) {
        if (!(in.deal & 2)) return;
        const int lane0 = threadIdx.x & (WAVE - 1);
        const int x = (int)blockIdx.x & (kDealLists - 1);
        const int nxt = in.deal_ring == 2 ? 0 : in.deal_ring + 1;
        if (lane0 == 0) {
            const int c = (in.auto_reset && cx.ended) ? 0 : (cx.ncnt < kDealClasses - 1 ? cx.ncnt : kDealClasses - 1);
            const int slot = atomicAdd(p.deal_cnt + (size_t)nxt * kDealRingInts + (x * kDealClasses + c) * kDealPad, 1);
            // (ring nxt of the orders too: workgroups of this step that start later still
            // read ring deal_ring, so the orders are never overwritten while in use)
            const size_t ring_off = (size_t)nxt * kDealLists * kDealClasses * (size_t)p.E;
            gmem(p.deal_order)[ring_off + ((size_t)x * kDealClasses + c) * p.E + slot] = e;
        }
        if (blockIdx.x == 0 && lane0 < kDealLists * kDealClasses) {  // clear ring t + 2
            const int clr = nxt == 2 ? 0 : nxt + 1;
            gmem(p.deal_cnt)[(size_t)clr * kDealRingInts + lane0 * kDealPad] = 0;
        }
    }
}

// ESPLIT (early split, large batches, one env per two-wave workgroup, 8 waves per
// SIMD at <= 64 VGPRs): the LiDAR wave computes the agents' poses after Car::update
// itself and marches the road (LiDAR phases 1-2) while the car wave runs the car
// part; after barrier B (obstacle table, candidate masks, respawns) it re-marches
// the respawned egos' beams and resolves the cars (phase 3) while the car wave runs
// cars_post.  The car waves' latency-bound chains and the LiDAR waves'
// VALU-bound phases then share each SIMD instead of following each other.
// Issue levels: the LiDAR wave's kinematics and road march 3 (its critical path),
// the car wave 2 (slack until barrier B), the LiDAR wave after B (re-march, car
// pairs, block writes) 1.  Waves per SIMD: 4 (split), 8 (early split, one env per
// workgroup).
constexpr int kSplitWpe = 4;
constexpr int kEsplitWpe = 8;
// the traffic early split: kTsplitEnvs envs (car waves) + one LiDAR wave per workgroup,
// kTsplitWpe waves per SIMD (config 4: 4096 envs -> 6144 waves on 1024 SIMDs).  Two envs,
// not four: the LiDAR wave's march of its egos' beams, which the light envs' car waves wait
// for at barrier H, halves -- config 4 148.4 -> 150.8 M, 1024 / 2048 / 3072 envs 2-4 %
// faster (profiles/r6_ab_ts2_*.txt; variant builds ts2* via MEV_TSPLIT_ENVS)
#ifndef MEV_TSPLIT_ENVS
#define MEV_TSPLIT_ENVS 2
#endif
constexpr int kTsplitEnvs = MEV_TSPLIT_ENVS;
// the traffic early split's LiDAR wave issues at level 1 (its ego phase 1 and road march
// have slack beside a heavy env's NPC phase, which sets the kernel's end): config 4
// 143.4 -> 151.2 M against level 3 (profiles/r5_ab_tsprio*_cfg4.txt, four rounds; 2: 149 M,
// 0: 150 M)
#ifndef MEV_TSPLIT_LPRIO
#define MEV_TSPLIT_LPRIO 1
#endif
constexpr int kPrioTsplitLidar = MEV_TSPLIT_LPRIO;
constexpr int kTsplitRays = kFixedRays;  // LiDAR pool beams per env
// (6: 2048 three-wave workgroups at 4096 envs, all resident at once.  With four envs per
// workgroup a 5-wave budget (93 VGPRs) did not fit 4096 envs in one residency round --
// five waves do not spread evenly over a CU's four SIMDs: 38.3 us against 28.7 us at 3072
// envs; at 80 VGPRs they did, profiles/r5_ts_wpe_cfg4.txt)
constexpr int kTsplitWpe = 6;
constexpr int kPrioEsplitRoad = 3;
constexpr int kPrioEsplitCars = 2;
#ifndef MEV_TSPLIT_CPRIO
#define MEV_TSPLIT_CPRIO kPrioEsplitCars
#endif
constexpr int kPrioTsplitCars = MEV_TSPLIT_CPRIO;  // the traffic early split's car waves
constexpr int kPrioEsplitCarPhase = 1;
// P1 (lidar_body's): 1 a LiDAR of a multiple of 64 beams, 2 of another beam count, >= 64 exactly P1
// beams (64: config 3, 96: the reference's default LiDAR, 128: config 5)
template <bool TRAFFIC, bool TAB, int NM, int KM = MAXK, int PK = 1, bool SPLIT = false, bool ESPLIT = false, int P1 = 0,
          int NC = 0>
__global__ __launch_bounds__((TRAFFIC && ESPLIT) ? (PK + 1) * WAVE : (SPLIT ? 2 * WAVE : WAVE),
                             (TRAFFIC && ESPLIT) ? kTsplitWpe
                                                 : ((ESPLIT && PK == 1) ? kEsplitWpe : (SPLIT ? kSplitWpe : 4))) void k_step(
    const SimParams* __restrict__ pp, StepInputs in, Outputs out) {
#include "mev_step_body.inc"
}

// ------------------------------------------------- persistent step server ---
// k_serve: the fused step of a small host-mode handle as a persistent kernel.  A
// host step then costs a mailbox round trip over PCIe instead of a kernel launch
// plus a stream synchronisation (the single env of the reference's env.py: 22 us
// per step launched).  Wave 0 of each workgroup polls the command
// line of the ServeBox (system-scope loads of host-coherent memory) until a new
// command, a stop, or sa.idle_ticks of the 100 MHz clock without one; it hands the
// command to the other wave through LDS.  A step runs k_step's body (mev_step_body.inc) -- the same code
// as k_step, the same grid -- reading the actions from and writing the outputs to
// the handle's pinned block; then every wave releases its writes at system scope
// and workgroup b publishes done[b] = the command's number.  Every exit (stop, or
// idle) publishes exited[b] = the instance's epoch first, so the host knows to
// launch a new instance; that instance starts from done[b] and never serves a
// command twice.  Every wave reaches the exit: the poll loop is bounded by the
// clock, a step by its own work.
template <bool TRAFFIC, bool TAB, int NM, int KM, bool SPLIT, int SP1 = 0, int SNC = 0>
__global__ __launch_bounds__(SPLIT ? 2 * WAVE : WAVE, SPLIT ? kSplitWpe : 4) void k_serve(
    const SimParams* __restrict__ pp, ServeArgs sa, Outputs out) {
    __shared__ uint32_t cmdw[kServeLine];
    constexpr int PK = 1;
    constexpr bool ESPLIT = false;
    constexpr int P1 = SP1, NC = SNC;  // (the beams and agents per env at compile time, as in k_step)
    const int lane = threadIdx.x & (WAVE - 1);
    const bool w0 = threadIdx.x < WAVE;
    ServeBox* box = sa.box;
    uint32_t last_seq = 0xffffffffu;  // never a posted number: the first poll reads the line at once
    uint32_t served = __builtin_amdgcn_readfirstlane(
        __hip_atomic_load(&box->done[blockIdx.x], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM));
    for (;;) {
        if (w0) {
            const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
            uint32_t seq = last_seq, quit = 0u;
            for (;;) {
                seq = __builtin_amdgcn_readfirstlane(
                    __hip_atomic_load(&box->seq, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM));
                if (seq != last_seq) break;
                if (__builtin_amdgcn_s_memrealtime() - t0 > sa.idle_ticks) {
                    quit = 1u;
                    break;
                }
                __builtin_amdgcn_s_sleep(4);
            }
            // the command line, written before seq: seq cmd sid dt spawn_prob auto_reset spawn rng_lo rng_hi
            uint32_t word = 0u;
            if (lane < kServeLine) word = __hip_atomic_load(&box->seq + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            if (lane == 0) word = seq;
            if (lane == 1 && quit) word = kServeStop;
            if (lane < kServeLine) cmdw[lane] = word;
        }
        __syncthreads();
        const uint32_t seq = cmdw[0], cmd = cmdw[1], sid = cmdw[2];
        if (cmd != kServeStep) break;  // a stop, or idle
        last_seq = seq;
        if (sid == served) {  // a re-post of a step this workgroup has answered
            __syncthreads();  // (wave 0 rewrites cmdw only after every wave has read it)
            continue;
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");  // the actions the host wrote before seq
        StepInputs in{};
        in.actions = sa.actions;
        in.spawn_route = cmdw[6] ? sa.spawn_route : nullptr;
        in.dt = __uint_as_float(cmdw[3]);
        in.spawn_prob = __uint_as_float(cmdw[4]);
        in.auto_reset = (int32_t)cmdw[5];
        in.rng_counter = (uint64_t)cmdw[7] | ((uint64_t)cmdw[8] << 32);
        [&]() {  // one step: k_step's body (its returns end the lambda)
#include "mev_step_body.inc"
        }();
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");  // this wave's outputs and state written
        __syncthreads();  // (also: nobody reads cmdw or the step's LDS any more)
        if (threadIdx.x == 0) __hip_atomic_store(&box->done[blockIdx.x], sid, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        served = sid;
    }
    if (threadIdx.x == 0) __hip_atomic_store(&box->exited[blockIdx.x], sa.epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}


// ------------------------------------------------- reset / re-observe ---
// IntersectionEnv::reset + add_car_with_route (cpp/IntersectionEnv.cpp:66-131)
// and the reset observation (LiDAR block = max_dist / max_dist).
template <bool TRAFFIC>
__global__ __launch_bounds__(WAVE) void k_reset(SimParams p, const uint8_t* mask, Outputs out, int do_reset,
                                                uint64_t rng_counter) {
    const int e = blockIdx.x;
    const int lane = threadIdx.x;
    const int N = p.N;
    if (mask && !mask[e]) return;
    __shared__ EgoLDS el;
    __shared__ typename std::conditional<TRAFFIC, NpcLDS, char>::type nl_storage;
    NpcLDS* nl = nullptr;
    if constexpr (TRAFFIC) nl = &nl_storage;
    for (int i = lane; i < N; i += WAVE) {
        const int g = e * N + i;
        if (do_reset) {
            const int rid = reset_route(p, rng_counter, e, i, egoi(p, EF_ROUTE)[g]);
            egoi(p, EF_ROUTE)[g] = rid;
            egof(p, EF_X)[g] = gmem(p.rt.spawn)[3 * rid];
            egof(p, EF_Y)[g] = gmem(p.rt.spawn)[3 * rid + 1];
            egof(p, EF_V)[g] = 0.0f;
            egof(p, EF_H)[g] = gmem(p.rt.spawn)[3 * rid + 2];
            egof(p, EF_SX)[g] = egof(p, EF_X)[g]; egof(p, EF_SY)[g] = egof(p, EF_Y)[g]; egof(p, EF_SV)[g] = 0.0f; egof(p, EF_SH)[g] = egof(p, EF_H)[g];
            egof(p, EF_ACC)[g] = 0.0f; egof(p, EF_STEER)[g] = 0.0f; egof(p, EF_PREV_DIST)[g] = 0.0f;
            egof(p, EF_PA0)[g] = 0.0f; egof(p, EF_PA1)[g] = 0.0f; egoi(p, EF_PIDX)[g] = 0;
            egoi(p, EF_INTENT)[g] = gmem(p.rt.intent)[rid]; gmem(p.ego.alive)[g] = 1;
            gmem(p.ego_dim)[2 * g] = CAR_LENGTH;  // reset + add_car_with_route: new Cars of the
            gmem(p.ego_dim)[2 * g + 1] = CAR_WIDTH;  // default size (Car.h:19-20)
        }
        el.x[i] = egof(p, EF_X)[g]; el.y[i] = egof(p, EF_Y)[g]; el.v[i] = egof(p, EF_V)[g]; el.h[i] = egof(p, EF_H)[g];
        el.alive[i] = gmem(p.ego.alive)[g]; el.intent[i] = egoi(p, EF_INTENT)[g]; el.pidx[i] = egoi(p, EF_PIDX)[g];
    }
    int ncnt = 0;
    if (do_reset) {
        if (lane == 0) {
            gmem(p.step_count)[e] = 0;
            gmem(p.pending_reset)[e] = 0;
            if (TRAFFIC) gmem(p.npc.count)[e] = 0;
        }
    } else if constexpr (TRAFFIC) {
        ncnt = gmem(p.npc.count)[e];
        if (lane < ncnt) {
            const int g = e * p.K + lane;
            nl->x[lane] = npcf(p, NF_X)[g]; nl->y[lane] = npcf(p, NF_Y)[g]; nl->v[lane] = npcf(p, NF_V)[g]; nl->h[lane] = npcf(p, NF_H)[g];
            nl->intent[lane] = npci(p, NF_INTENT)[g]; nl->alive[lane] = gmem(p.npc.alive)[g];
        }
    }
    wave_lds_sync();
    bool exact = false;  // (N <= 64: one pass, lane i = agent i)
    float dl = 0.0f;
    for (int i = lane; i < N; i += WAVE) {
        const int g = e * N + i;
        float* row = out.obs + (size_t)g * p.D;
        if (!el.alive[i]) {
            for (int c = 0; c < p.D; ++c) row[c] = 0.0f;
            continue;
        }
        const float* path = p.rt.path + (size_t)egoi(p, EF_ROUTE)[g] * (2 * p.rt.row);
        exact = write_obs_head<TRAFFIC>(p, i, el, nl, ncnt, path, el.pidx[i], row, &dl);
        for (int b = 0; b < p.lidar_slots; ++b) row[OBS_HEAD + b] = p.lidar_max * p.lidar_inv;
    }
    const unsigned long long m = ballot(exact);
    if (__builtin_expect(m != 0ull, 0))
        obs_exact_pass<TRAFFIC, TRAFFIC>(p, m, dl, el, nl, ncnt, out.obs + (size_t)e * N * p.D, (size_t)p.D);
}

static hipError_t launch_part(const SimParams& p, const StepInputs& in, const Outputs& out, int e0, int e1,
                              hipStream_t s, const hipEvent_t* ev) {
    // k_cars then k_lidar over the envs [e0, e1)
    if (e1 <= e0) return hipSuccess;
    if (ev) (void)hipEventRecord(ev[0], s);
    const unsigned cars_lds = (unsigned)cars_lds_bytes(p.N, cars_k(p), true);
    if (p.traffic) hipLaunchKernelGGL(k_cars<true>, dim3(e1 - e0), dim3(WAVE), cars_lds, s, p, in, out, e0);
    else hipLaunchKernelGGL(k_cars<false>, dim3(e1 - e0), dim3(WAVE), cars_lds, s, p, in, out, e0);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    if (ev) (void)hipEventRecord(ev[1], s);
    const int a_begin = e0 * p.N, a_end = e1 * p.N, na = a_end - a_begin;
    int G = lidar_group(p.R);
    // small batches: trade pool size for waves (~4 per SIMD on 256 CUs) so latency is hidden
    while (G > 1 && na / G < 4096) G = (G + 1) / 2;
    static const int g_env = [] { const char* v = getenv("MEV_LIDAR_G"); return v ? atoi(v) : 0; }();
    if (g_env > 0 && g_env <= 64 && (size_t)g_env * p.R <= 1024) G = g_env;  // experiments (tools/kernel_time.py)
    // LDS: shrink the group, then the waves per block, to stay within 40 KB (64 KB hard) per block
    int wpb = 4;
    while (G > 1 && wpb * lidar_layout(G, p.R, lidar_cand_max(p)).bytes > 40 * 1024) G = (G + 1) / 2;
    const int wave_lds = lidar_layout(G, p.R, lidar_cand_max(p)).bytes;
    while (wpb > 1 && wpb * wave_lds > 64 * 1024) wpb /= 2;
    const int groups = (na + G - 1) / G;
    const unsigned blocks = (unsigned)((groups + wpb - 1) / wpb);
    if (p.dist_tab)
        hipLaunchKernelGGL(k_lidar<true>, dim3(blocks), dim3(wpb * WAVE), wpb * wave_lds, s, p, out, G, a_begin, a_end);
    else
        hipLaunchKernelGGL(k_lidar<false>, dim3(blocks), dim3(wpb * WAVE), wpb * wave_lds, s, p, out, G, a_begin, a_end);
    e = hipGetLastError();
    if (ev && e == hipSuccess) (void)hipEventRecord(ev[2], s);
    return e;
}

// NPC slots of the fused kernel's LDS arrays (NpcLDST<KM>): the smallest
// compiled capacity that holds the handle's max_npcs
static int fused_npc_cap(const SimParams& p) { return p.K <= 32 ? 32 : 64; }

// LDS of one k_step wave: the dynamic part (cars + one LiDAR pool of
// step_pool(p) agents) plus, with traffic, the static NPC arrays
static size_t fused_lds_bytes(const SimParams& p) {
    size_t b = (size_t)step_layout(p).bytes;
    // (the runtime-layout traffic kernels hold the NPC sizes too: NpcLDST<KM, true>)
    if (p.traffic) b += fused_npc_cap(p) == 32 ? sizeof(NpcLDST<32, true>) : sizeof(NpcLDST<64, true>);
    return b;
}

// k_step applies when its LDS fits one workgroup (64 KB); it is the automatic
// choice when it also fits a wave's share at 4 waves per SIMD (128 VGPRs): a CU
// holds 16 waves, so a wave may take 160 KB / 16 = 10 KB.
static bool fused_fits(const SimParams& p) {
    return fused_lds_bytes(p) <= 64 * 1024;
}

int step_kernel_for(const SimParams& p) {
    const bool fusable = fused_fits(p);
    if (p.step_kernel == 1) return 1;
    if (p.step_kernel == 2) return fusable ? 2 : 0;
    // auto: fused when a wave's LDS leaves 4 waves per SIMD and either the batch fills
    // the chip with one wave per env (>= 4 per CU), or an env's beams fit one k_lidar
    // group anyway (N * R <= 256: the second launch buys nothing, 1 env x 1 agent 70 ->
    // 82 k steps/s fused), or the env fits the compile-time 8-slot layout: its k_step
    // (two waves per env below 2048 workgroups, counts at compile time) beats the
    // LiDAR's finer per-group waves at every batch size since round 6 (8 agents x 64
    // beams: 64 envs 21.2 -> 16.7 us, 768 envs 27.2 -> 18.3 us; profiles/r6_stepk_small.txt).
    // Larger envs at small batches keep the two-kernel path.
    const bool small_env = p.N * p.R <= 256 || (!p.traffic && fixed_fits<8, 0>(p));
    return (fusable && fused_lds_bytes(p) <= 10 * 1024 && (p.E >= 1024 || small_env)) ? 2 : 1;
}

// envs per k_step wave (1, 2 or 4) for a handle without traffic whose N agents
// fit the 8-slot layout: several small envs share a wave's lanes, so one latency
// chain serves them all.  p.step_pack (mev_set_step_pack) chooses; 0 = automatic.
// Automatic: the most envs per wave that keeps >= 2048 waves (2 per SIMD) --
// config 2 (4096 x 1 agent): 2 envs per wave, 177 -> 202 M agent-steps/s; 4
// envs per wave (1024 waves, one per SIMD) 194 M (profiles/r2_pack_sweep.txt).
int step_pack(const SimParams& p) {
    if (p.traffic || !fixed_fits<8, 0>(p)) return 1;
    if (step_esplit(p)) return esplit_pack(p);
    int pk = p.step_pack;
    if (pk != 1 && pk != 2 && pk != 4 && pk != 8) {
        pk = 4;
        while (pk > 1 && p.E / pk < 2048) pk /= 2;
    }
    while (pk > 1 && pk * p.N > 8) pk /= 2;
    return pk;
}

// two waves per fused workgroup (k_step SPLIT) when that keeps <= 4 waves per SIMD
// (<= 2048 workgroups; 256 CUs x 4 SIMDs)
constexpr int kSplitMaxWg = 2048;
// Envs per workgroup of the early split (k_step ESPLIT; 0: it does not apply).  An
// explicit mev_set_step_pack is kept (reduced to <= 8 agent slots) when the slots'
// beams fit one 512-beam LiDAR pool.  Automatic: 4 envs while their beams stay
// <= 256 and >= 1024 workgroups remain, else 2 envs within one pool and >= 1024
// workgroups, else 0 (the automatic choice then keeps one wave per env / the plain
// split; mev_set_step_split(3) forces one env per workgroup at 8 waves per SIMD).
// Measured against the plain split's best, one MI355X (profiles/r3_esplit_shapes.txt):
// 4096 x 1 x 64 beams (config 2) 13.3 -> 11.6 us per step at 4 envs, 4096 x 4 x 64
// 24.1 -> 22.0 at 2, 2048 x 1 x 64 12.4 -> 10.0 at 2, 4096 x 1 x 128 15.5 -> 14.4 at 2.
int esplit_pack(const SimParams& p) {
    // traffic: kTsplitEnvs one-ego envs per workgroup (every workgroup full, and the
    // NPC-aware deal's lists of E / 8 envs split into whole workgroups).  Automatic at
    // every such E: with two envs per workgroup it beats one wave per env from 16 to
    // 16384 envs -- 16-512 envs 25-35 %, 8192 envs 145 -> 165 M, 16384 160 -> 190 M
    // agent-steps/s (profiles/r6_ts2_auto_*.txt).  (Round 5's four envs per workgroup
    // lost at 8192 envs, 55.9 -> 59.0 us, profiles/r5_ab_ts6_cfg4.txt.)
    if (p.traffic)
        return fixed_fits<1, 32>(p) && p.R <= kTsplitRays && p.E % (8 * kTsplitEnvs) == 0 &&
                       (p.step_split == 3 || p.step_split == 0)
                   ? kTsplitEnvs
                   : 0;
    if (!fixed_fits<8, 0>(p) || p.N > 8) return 0;
    const int nr = p.N * p.R;
    int pk = p.step_pack;
    if (pk == 1 || pk == 2 || pk == 4 || pk == 8) {
        while (pk > 1 && pk * p.N > 8) pk /= 2;
        return pk * nr <= kPoolBeams ? pk : 0;
    }
    if (4 * p.N <= 8 && 4 * nr <= kPoolBeams / 2 && p.E / 4 >= 1024) return 4;
    if (2 * p.N <= 8 && 2 * nr <= kPoolBeams && p.E / 2 >= 1024) return 2;
    return p.step_split == 3 && nr <= kPoolBeams ? 1 : 0;
}
// the early split: automatic (mode 0) where esplit_pack finds >= 2 envs per
// workgroup, or forced (mode 3)
bool step_esplit(const SimParams& p) {
    if (p.step_split == 1 || p.step_split == 2) return false;
    const int pk = esplit_pack(p);
    return p.step_split == 3 ? pk > 0 : pk >= 2;
}
bool step_split(const SimParams& p) {
    if (p.traffic || !fixed_fits<8, 0>(p) || p.step_split == 1 || step_esplit(p)) return false;
    if (p.step_split == 2) return true;
    const int pk = step_pack(p);
    return (p.E + pk - 1) / pk <= kSplitMaxWg;
}

// the beam count a k_step instantiation fixes at compile time (its P1): 64, 96 or 128
// beams, every one in the observation; else 0
static int fixed_r(const SimParams& p) {
    return (p.R == 64 || p.R == 96 || p.R == 128) && p.lidar_slots == p.R ? p.R : 0;
}

template <bool TAB>
static void launch_fused(const SimParams& p, const SimParams* dp, const StepInputs& in, const Outputs& out,
                         hipStream_t s) {
    if (p.traffic) {
        if (fixed_fits<1, 32>(p)) {  // compile-time LDS layout (config 4: one ego, <= 32 NPC slots)
            const unsigned lds = (unsigned)FixedLayout<1, 32>::bytes;  // + the static NpcLDST
            if (step_esplit(p)) {  // the traffic early split: kTsplitEnvs car waves + a LiDAR wave
                constexpr int P = kTsplitEnvs;
                const unsigned tl = (unsigned)(P * FixedLayout<1, 32>::lidar + lidar_layout_beams(P, P * kTsplitRays, 32, false).bytes);
                if (fixed_r(p) == 64)  // (config 4: the beam count at compile time)
                    hipLaunchKernelGGL((k_step<true, TAB, 1, 32, P, true, true, 64>), dim3(p.E / P), dim3((P + 1) * WAVE), tl,
                                       s, dp, in, out);
                else
                    hipLaunchKernelGGL((k_step<true, TAB, 1, 32, P, true, true>), dim3(p.E / P), dim3((P + 1) * WAVE), tl, s,
                                       dp, in, out);
                return;
            }
            hipLaunchKernelGGL((k_step<true, TAB, 1, 32>), dim3(p.E), dim3(WAVE), lds, s, dp, in, out);
            return;
        }
        const unsigned lds = (unsigned)step_layout(p).bytes;  // + the static NpcLDST
        if (fused_npc_cap(p) == 32) hipLaunchKernelGGL((k_step<true, TAB, 0, 32>), dim3(p.E), dim3(WAVE), lds, s, dp, in, out);
        else hipLaunchKernelGGL((k_step<true, TAB, 0, 64>), dim3(p.E), dim3(WAVE), lds, s, dp, in, out);
    } else if (fixed_fits<8, 0>(p)) {  // compile-time LDS layout
        const unsigned lds = (unsigned)FixedLayout<8>::bytes;
        const int pk = step_pack(p);
        const int wg = (p.E + pk - 1) / pk;
        const int fr = fixed_r(p);
        if (step_esplit(p)) {  // early split: a car wave and a LiDAR wave per workgroup
            if (pk == 8) hipLaunchKernelGGL((k_step<false, TAB, 8, MAXK, 8, true, true>), dim3(wg), dim3(2 * WAVE), lds, s, dp, in, out);
            else if (pk == 4 && p.N == 1 && fr == 64)  // (config 2: agents per env and beams at compile time)
                hipLaunchKernelGGL((k_step<false, TAB, 8, MAXK, 4, true, true, 64, 1>), dim3(wg), dim3(2 * WAVE), lds, s, dp, in, out);
            else if (pk == 4 && p.N == 1)
                hipLaunchKernelGGL((k_step<false, TAB, 8, MAXK, 4, true, true, 0, 1>), dim3(wg), dim3(2 * WAVE), lds, s, dp, in, out);
            else if (pk == 4) hipLaunchKernelGGL((k_step<false, TAB, 8, MAXK, 4, true, true>), dim3(wg), dim3(2 * WAVE), lds, s, dp, in, out);
            else if (pk == 2 && p.N == 1 && fr == 96)  // (the reference's defaults: one agent, 96 beams)
                hipLaunchKernelGGL((k_step<false, TAB, 8, MAXK, 2, true, true, 96, 1>), dim3(wg), dim3(2 * WAVE), lds, s, dp, in, out);
            else if (pk == 2 && p.N == 1)
                hipLaunchKernelGGL((k_step<false, TAB, 8, MAXK, 2, true, true, 0, 1>), dim3(wg), dim3(2 * WAVE), lds, s, dp, in, out);
            else if (pk == 2) hipLaunchKernelGGL((k_step<false, TAB, 8, MAXK, 2, true, true>), dim3(wg), dim3(2 * WAVE), lds, s, dp, in, out);
            else hipLaunchKernelGGL((k_step<false, TAB, 8, MAXK, 1, true, true>), dim3(wg), dim3(2 * WAVE), lds, s, dp, in, out);
            return;
        }
        if (step_split(p)) {  // two waves per workgroup (<= 4 waves per SIMD)
            if (pk == 8) hipLaunchKernelGGL((k_step<false, TAB, 8, MAXK, 8, true>), dim3(wg), dim3(2 * WAVE), lds, s, dp, in, out);
            else if (pk == 4) hipLaunchKernelGGL((k_step<false, TAB, 8, MAXK, 4, true>), dim3(wg), dim3(2 * WAVE), lds, s, dp, in, out);
            else if (pk == 2) hipLaunchKernelGGL((k_step<false, TAB, 8, MAXK, 2, true>), dim3(wg), dim3(2 * WAVE), lds, s, dp, in, out);
            else if (p.N == 8 && fr == 64)  // (configs 3 / 5 and 96 beams' shapes in smaller batches)
                hipLaunchKernelGGL((k_step<false, TAB, 8, MAXK, 1, true, false, 64, 8>), dim3(wg), dim3(2 * WAVE), lds, s, dp, in, out);
            else if (p.N == 8 && fr == 96)
                hipLaunchKernelGGL((k_step<false, TAB, 8, MAXK, 1, true, false, 96, 8>), dim3(wg), dim3(2 * WAVE), lds, s, dp, in, out);
            else if (p.N == 8 && fr == 128)
                hipLaunchKernelGGL((k_step<false, TAB, 8, MAXK, 1, true, false, 128, 8>), dim3(wg), dim3(2 * WAVE), lds, s, dp, in, out);
            else if (p.N == 1)  // (config 1: one agent per env at compile time)
                hipLaunchKernelGGL((k_step<false, TAB, 8, MAXK, 1, true, false, 0, 1>), dim3(wg), dim3(2 * WAVE), lds, s, dp, in, out);
            else hipLaunchKernelGGL((k_step<false, TAB, 8, MAXK, 1, true>), dim3(wg), dim3(2 * WAVE), lds, s, dp, in, out);
            return;
        }
        if (pk == 8) hipLaunchKernelGGL((k_step<false, TAB, 8, MAXK, 8>), dim3(wg), dim3(WAVE), lds, s, dp, in, out);
        else if (pk == 4) hipLaunchKernelGGL((k_step<false, TAB, 8, MAXK, 4>), dim3(wg), dim3(WAVE), lds, s, dp, in, out);
        else if (pk == 2) hipLaunchKernelGGL((k_step<false, TAB, 8, MAXK, 2>), dim3(wg), dim3(WAVE), lds, s, dp, in, out);
        else if (fr == 64 && p.N == 8)
            hipLaunchKernelGGL((k_step<false, TAB, 8, MAXK, 1, false, false, 64, 8>), dim3(wg), dim3(WAVE), lds, s, dp, in, out);
        else if (fr == 64)
            hipLaunchKernelGGL((k_step<false, TAB, 8, MAXK, 1, false, false, 64>), dim3(wg), dim3(WAVE), lds, s, dp, in, out);
        else if (fr == 96 && p.N == 8)
            hipLaunchKernelGGL((k_step<false, TAB, 8, MAXK, 1, false, false, 96, 8>), dim3(wg), dim3(WAVE), lds, s, dp, in, out);
        else if (fr == 96)
            hipLaunchKernelGGL((k_step<false, TAB, 8, MAXK, 1, false, false, 96>), dim3(wg), dim3(WAVE), lds, s, dp, in, out);
        else if (fr == 128 && p.N == 8)
            hipLaunchKernelGGL((k_step<false, TAB, 8, MAXK, 1, false, false, 128, 8>), dim3(wg), dim3(WAVE), lds, s, dp, in, out);
        else if (fr == 128)
            hipLaunchKernelGGL((k_step<false, TAB, 8, MAXK, 1, false, false, 128>), dim3(wg), dim3(WAVE), lds, s, dp, in, out);
        else if ((p.R & (WAVE - 1)) == 0)
            hipLaunchKernelGGL((k_step<false, TAB, 8, MAXK, 1, false, false, 1>), dim3(wg), dim3(WAVE), lds, s, dp, in, out);
        else hipLaunchKernelGGL((k_step<false, TAB, 8, MAXK, 1, false, false, 2>), dim3(wg), dim3(WAVE), lds, s, dp, in, out);
    } else {
        const unsigned lds = (unsigned)step_layout(p).bytes;
        hipLaunchKernelGGL((k_step<false, TAB, 0>), dim3(p.E), dim3(WAVE), lds, s, dp, in, out);
    }
}

hipError_t launch_step(const SimParams& p, const SimParams* dp, const StepInputs& in, const Outputs& out,
                       hipStream_t s, const hipEvent_t* ev) {
    const int kind = step_kernel_for(p);
    if (kind == 0) return hipErrorInvalidValue;
    if (kind == 2) {
        if (ev) (void)hipEventRecord(ev[0], s);
        if (p.dist_tab) launch_fused<true>(p, dp, in, out, s);
        else launch_fused<false>(p, dp, in, out, s);
        hipError_t e = hipGetLastError();
        if (ev && e == hipSuccess) { (void)hipEventRecord(ev[1], s); (void)hipEventRecord(ev[2], s); }
        return e;
    }
    return launch_part(p, in, out, 0, p.E, s, ev);
}

// k_serve runs the handle's fused step (one workgroup per env): the compile-time
// layouts of launch_fused for small batches -- the split kernel without traffic,
// one ego with <= 32 NPC slots -- and, for more NPC slots (env.py's 64), the
// dynamic traffic layout, which at one env may take more than a wave's 10 KB share
bool serve_fits(const SimParams& p) {
    if (step_kernel_for(p) == 0 || p.step_kernel == 1 || p.dims) return false;
    if (p.E > kServeMaxWG) return false;
    if (p.traffic) return fixed_fits<1, 32>(p) || (p.K > 32 && fused_fits(p));
    return fixed_fits<8, 0>(p) && step_pack(p) == 1 && !step_esplit(p) && p.step_split != 1;
}

hipError_t launch_serve(const SimParams& p, const SimParams* dp, const ServeArgs& sa, const Outputs& out,
                        hipStream_t s) {
    if (!serve_fits(p)) return hipErrorInvalidValue;
    if (p.traffic && fixed_fits<1, 32>(p)) {
        const unsigned lds = (unsigned)FixedLayout<1, 32>::bytes;
        if (p.dist_tab) hipLaunchKernelGGL((k_serve<true, true, 1, 32, false>), dim3(p.E), dim3(WAVE), lds, s, dp, sa, out);
        else hipLaunchKernelGGL((k_serve<true, false, 1, 32, false>), dim3(p.E), dim3(WAVE), lds, s, dp, sa, out);
    } else if (p.traffic) {
        const unsigned lds = (unsigned)step_layout(p).bytes;  // + the static NpcLDST<64>
        if (p.dist_tab) hipLaunchKernelGGL((k_serve<true, true, 0, 64, false>), dim3(p.E), dim3(WAVE), lds, s, dp, sa, out);
        else hipLaunchKernelGGL((k_serve<true, false, 0, 64, false>), dim3(p.E), dim3(WAVE), lds, s, dp, sa, out);
    } else {
        const unsigned lds = (unsigned)FixedLayout<8>::bytes;
        // (env.py's common shapes with their counts at compile time: one agent, 8 agents x 64 / 96 beams)
        const dim3 g(p.E), b(2 * WAVE);
        if (p.N == 1) {
            if (p.dist_tab) hipLaunchKernelGGL((k_serve<false, true, 8, MAXK, true, 0, 1>), g, b, lds, s, dp, sa, out);
            else hipLaunchKernelGGL((k_serve<false, false, 8, MAXK, true, 0, 1>), g, b, lds, s, dp, sa, out);
        } else if (p.N == 8 && fixed_r(p) == 64) {
            if (p.dist_tab) hipLaunchKernelGGL((k_serve<false, true, 8, MAXK, true, 64, 8>), g, b, lds, s, dp, sa, out);
            else hipLaunchKernelGGL((k_serve<false, false, 8, MAXK, true, 64, 8>), g, b, lds, s, dp, sa, out);
        } else if (p.N == 8 && fixed_r(p) == 96) {
            if (p.dist_tab) hipLaunchKernelGGL((k_serve<false, true, 8, MAXK, true, 96, 8>), g, b, lds, s, dp, sa, out);
            else hipLaunchKernelGGL((k_serve<false, false, 8, MAXK, true, 96, 8>), g, b, lds, s, dp, sa, out);
        } else {
            if (p.dist_tab) hipLaunchKernelGGL((k_serve<false, true, 8, MAXK, true>), g, b, lds, s, dp, sa, out);
            else hipLaunchKernelGGL((k_serve<false, false, 8, MAXK, true>), g, b, lds, s, dp, sa, out);
        }
    }
    return hipGetLastError();
}

hipError_t launch_reset(const SimParams& p, const uint8_t* env_mask, const Outputs& out, hipStream_t s,
                        uint64_t rng_counter) {
    if (p.traffic) hipLaunchKernelGGL(k_reset<true>, dim3(p.E), dim3(WAVE), 0, s, p, env_mask, out, 1, rng_counter);
    else hipLaunchKernelGGL(k_reset<false>, dim3(p.E), dim3(WAVE), 0, s, p, env_mask, out, 1, rng_counter);
    return hipGetLastError();
}

hipError_t launch_observe_reset_lidar(const SimParams& p, const Outputs& out, hipStream_t s) {
    if (p.traffic) hipLaunchKernelGGL(k_reset<true>, dim3(p.E), dim3(WAVE), 0, s, p, nullptr, out, 0, 0ull);
    else hipLaunchKernelGGL(k_reset<false>, dim3(p.E), dim3(WAVE), 0, s, p, nullptr, out, 0, 0ull);
    return hipGetLastError();
}

// ------------------------------------------- compact gather format unpack ---
// obs rows [n][D] from the compact format's heads [n][31] and LiDAR codes
// [n][slots] through the decode table (mev_lidar_decode_table): the same floats the
// plain step writes; padding columns are zero.  Thread = (row, column).
__global__ void k_unpack_lidar_u8(const float* head, const uint8_t* codes, const float* table, float* obs, int n,
                                  int D, int slots) {
    const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= (size_t)n * D) return;
    const size_t row = t / D;
    const int c = (int)(t - row * D);
    float v = 0.0f;
    if (c < OBS_HEAD) v = head[row * OBS_HEAD + c];
    else if (c < OBS_HEAD + slots) v = table[codes[row * slots + (c - OBS_HEAD)]];
    obs[t] = v;
}

hipError_t launch_unpack_lidar_u8(const float* head, const uint8_t* codes, const float* table, float* obs, int n,
                                  int D, int slots, hipStream_t s) {
    const size_t total = (size_t)n * D;
    if (total == 0) return hipSuccess;
    hipLaunchKernelGGL(k_unpack_lidar_u8, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, head, codes, table,
                       obs, n, D, slots);
    return hipGetLastError();
}

// The state gather format's decode (root): one wave per env rebuilds its agents'
// rows from the shipped post-step state -- get_observations (IntersectionEnv.cpp:
// 418-520) is a pure function of it -- with the step's own write_obs_head_tg,
// and the LiDAR block from the codes through the decode table.  No traffic (the
// format is refused for traffic handles: NPC states would outweigh the rows).
__global__ __launch_bounds__(WAVE) void k_decode_state(SimParams p, const uint8_t* state0, const uint8_t* codes0,
                                                       size_t stride, int C, const float* table, float* obs) {
    struct StateLDS {
        float x[MAXN], y[MAXN], v[MAXN], h[MAXN];
        int32_t intent[MAXN];
        uint8_t alive[MAXN];
    };
    __shared__ StateLDS el;
    const int lane = threadIdx.x;
    const int g = blockIdx.x, r = g / C, c = g - r * C;
    const int N = p.N, D = p.D, L = p.lidar_slots;
    const size_t n = (size_t)C * N;
    const uint8_t* sb = state0 + (size_t)r * stride;
    const uint8_t* cb = codes0 + (size_t)r * stride;
    int route = 0, pidx = 0;
    if (lane < N) {
        const size_t a = (size_t)c * N + lane;
        el.x[lane] = reinterpret_cast<const float*>(sb)[a];
        el.y[lane] = reinterpret_cast<const float*>(sb + 4 * n)[a];
        el.v[lane] = reinterpret_cast<const float*>(sb + 8 * n)[a];
        el.h[lane] = reinterpret_cast<const float*>(sb + 12 * n)[a];
        route = reinterpret_cast<const int16_t*>(sb + 16 * n)[a];
        pidx = reinterpret_cast<const int16_t*>(sb + 18 * n)[a];
        el.intent[lane] = sb[20 * n + a];
        el.alive[lane] = sb[21 * n + a];
    }
    __syncthreads();
    bool exact = false;  // (N <= 64: one pass, lane i = agent i)
    float dl = 0.0f;
    for (int i = lane; i < N; i += WAVE) {
        float* row = obs + ((size_t)g * N + i) * D;
        if (!el.alive[i]) {
            for (int q = 0; q < OBS_HEAD; ++q) row[q] = 0.0f;
            continue;
        }
        // a route id this table does not have (a peer's mev_add_route; mev_comm_init checks
        // the tables, so only a corrupt message gets here): counted (overflow[2]) and the
        // look-ahead terms NaN, never a clamped route's point
        const bool bad = route < 0 || route >= p.rt.nroutes;
        if (bad) atomicAdd(p.overflow + 2, 1ull);
        const int rt = bad ? 0 : route;
        const int ti = pidx + 10 < p.rt.plen - 1 ? (pidx + 10 < 0 ? 0 : pidx + 10) : p.rt.plen - 1;
        const float* path = p.rt.path + (size_t)rt * (2 * p.rt.row);
        const float nan = __builtin_nanf("");
        exact = write_obs_head_tg<false>(p, i, el, (const NpcLDST<MAXK>*)nullptr, 0, bad ? nan : path[2 * ti],
                                         bad ? nan : path[2 * ti + 1], row, false, &dl);
    }
    const unsigned long long m = ballot(exact);
    if (__builtin_expect(m != 0ull, 0))
        obs_exact_pass<false, false>(p, m, dl, el, (const NpcLDST<MAXK>*)nullptr, 0, obs + (size_t)g * N * D, (size_t)D);
    // LiDAR block and padding, every lane: (agent, column) pairs
    const int tail = D - OBS_HEAD;
    for (int t = lane; t < N * tail; t += WAVE) {
        const int i = t / tail, b = t - i * tail;
        const size_t a = (size_t)c * N + i;
        // (a dead agent's codes decode to 0 anyway; an unused slot's zeroed message has alive 0)
        obs[((size_t)g * N + i) * D + OBS_HEAD + b] = (b < L && el.alive[i]) ? table[cb[a * L + b]] : 0.0f;
    }
}

hipError_t launch_decode_state(const SimParams& p, const uint8_t* state0, const uint8_t* codes0, size_t stride, int C,
                               int n_env, const float* table, float* obs, hipStream_t s) {
    if (n_env <= 0) return hipSuccess;
    if (p.traffic || p.N > MAXN) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_decode_state, dim3((unsigned)n_env), dim3(WAVE), 0, s, p, state0, codes0, stride, C, table,
                       obs);
    return hipGetLastError();
}

// ----------------------------------------------------- masked restore ---
// mev_restore with an env mask: block (e, field) copies env e's slice of one
// snapshot field back into the live state when mask[e] is set.
__global__ __launch_bounds__(WAVE) void k_restore(RestoreTab tab, const uint8_t* src, const uint8_t* mask) {
    const int e = blockIdx.x, f = blockIdx.y;
    if (f >= tab.n || !mask[e]) return;
    const int bpe = tab.bpe[f];
    const uint8_t* s = src + tab.src_off[f] + (size_t)e * bpe;
    uint8_t* d = tab.dst[f] + (size_t)e * bpe;
    if ((bpe & 3) == 0) {
        for (int w = threadIdx.x; w < (bpe >> 2); w += WAVE)
            reinterpret_cast<uint32_t*>(d)[w] = reinterpret_cast<const uint32_t*>(s)[w];
    } else {
        for (int b = threadIdx.x; b < bpe; b += WAVE) d[b] = s[b];
    }
}

hipError_t launch_restore(const RestoreTab& tab, const uint8_t* src, const uint8_t* env_mask, int E, hipStream_t s) {
    hipLaunchKernelGGL(k_restore, dim3(E, tab.n), dim3(WAVE), 0, s, tab, src, env_mask);
    return hipGetLastError();
}

}  // namespace mev
