/*
 * marlenv.h — C ABI of libmarlenv_hip.so, the MI355X (gfx950) batched
 * intersection environment.
 *
 * This is the drop-in boundary that replaces the reference's pybind11 module
 * `MARLEnv` (reference cpp/bindings.cpp:11-95) as reached through
 * cpp_backend.py (reference cpp_backend.py:30-66) and env.py (reference
 * env.py:80-221).  One handle holds E independent environment instances
 * ("envs") of the reference's IntersectionEnv (reference
 * cpp/IntersectionEnv.h:23-105), each with N ego agents and (traffic mode) up
 * to max_npcs NPC cars, resident on ONE GPU in structure-of-arrays layout.
 *
 * Conventions
 *  - Every function returns 0 on success or a negative MEV_E* code; the
 *    message is available from mev_last_error() (thread-local).  No C++
 *    exception crosses this boundary.
 *  - Buffers are caller-owned.  Host pointers unless MEV_DEVICE_PTRS is set in
 *    the call's flags, in which case every pointer in that call is a device
 *    pointer on the handle's device and the call does not synchronise.
 *  - All work of a handle is ordered on one HIP stream (mev_set_stream).
 *  - Lane points are numbered 0..8L-1: "IN_k" -> k-1, "OUT_k" -> 4L+k-1
 *    (reference cpp/RouteGen.cpp:7-53).  A route is a (start point, end point)
 *    pair (reference IntersectionEnv::add_car_with_route,
 *    cpp/IntersectionEnv.cpp:78-131).
 *  - Status codes: 0 ALIVE, 1 DEAD, 2 SUCCESS, 3 CRASH_WALL, 4 CRASH_LINE,
 *    5 CRASH_CAR (the strings of reference cpp/Reward.h:16-29 / env.py:193).
 */
#ifndef MARLENV_H
#define MARLENV_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MEV_ABI_VERSION 3  /* 2: MEV_GATHER_STATE, MEV_PK_STATE (MEV_PK_FIELDS 7 -> 8), mev_unpack_gathered;
                              3: mev_set_car_dims / mev_get_car_dims, mev_set_beam_angles / mev_get_beam_angles,
                              mev_decode_errors, snapshot format 2 (car sizes, route table check) */

enum {
    MEV_OK = 0,
    MEV_E_INVALID = -1,  /* bad argument / configuration          */
    MEV_E_HIP = -2,      /* HIP runtime error                      */
    MEV_E_NOMEM = -3,    /* device or host allocation failed       */
    MEV_E_RANGE = -4     /* index out of range (std::out_of_range) */
};

enum { MEV_ALIVE = 0, MEV_DEAD = 1, MEV_SUCCESS = 2, MEV_CRASH_WALL = 3, MEV_CRASH_LINE = 4, MEV_CRASH_CAR = 5 };

/* flags for mev_step / mev_reset / mev_get_outputs */
#define MEV_DEVICE_PTRS 0x1u /* all pointers in this call are device pointers; no host sync */
#define MEV_AUTO_RESET 0x2u  /* an env whose previous step ended (terminated|truncated) is reset
                                before this step (gym-style vector auto-reset) */
/* MEV_GATHER_TO_ROOT (0x4) is declared with the multi-GPU entry points below */

typedef struct mev_handle mev_handle;

/* Configuration: fields mirror reference env.py:81-131 config keys and
 * IntersectionEnv::configure* (cpp/IntersectionEnv.cpp:50-64). */
typedef struct {
    int32_t num_envs;        /* E >= 1                                                     */
    int32_t num_agents;      /* N, 1..64 ego cars per env                                   */
    int32_t num_lanes;       /* lanes per direction (reference default 3)                  */
    int32_t lidar_rays;      /* R in [1, 1024] (reference hard-codes 96, IntersectionEnv.cpp:113) */
    float lidar_fov_deg;     /* 360                                                        */
    float lidar_max_dist;    /* 250 px                                                     */
    float lidar_step;        /* 4 px                                                       */
    int32_t obs_dim;         /* 0 => 31 + R; 127 reproduces the reference layout exactly   */
    int32_t traffic_flow;    /* NPC traffic mode (TrafficFlow.cpp)                          */
    float traffic_density;   /* arrival rate (1/s), clamped >= 0                            */
    int32_t use_team_reward;
    int32_t respawn_enabled;
    int32_t max_steps;       /* truncation; <= 0 disables                                   */
    float reward[8];         /* k_prog, v_min_ms, k_stuck, k_cv, k_co, k_succ, k_sm, alpha  */
    int32_t max_npcs;        /* NPC slots per env, 0..64 (overflowing spawns are dropped)    */
    uint64_t seed;           /* on-device Philox stream for NPC spawns                      */
    int32_t device;          /* HIP device ordinal                                          */
} mev_config;

/* Per-step arguments (reference IntersectionEnv::step, cpp/IntersectionEnv.cpp:133-392,
 * + get_observations :418-520). */
typedef struct {
    const float* actions;       /* [E][N][2] (throttle, steer); never clipped (Car.cpp:9-40) */
    float dt;                   /* seconds (reference default 1/60)                          */
    const int32_t* spawn_route; /* optional [E]: traffic-route index the NPC spawner uses this
                                   step (-1 = no spawn attempt); NULL = on-device Philox draw.
                                   Replays the reference's RNG decisions (TrafficFlow.cpp:275-329). */
    float* obs;                 /* optional [E][N][obs_dim]                                  */
    float* reward;              /* optional [E][N]                                           */
    uint8_t* done;              /* optional [E][N]                                           */
    uint8_t* status;            /* optional [E][N]                                           */
    uint8_t* terminated;        /* optional [E]                                              */
    uint8_t* truncated;         /* optional [E]                                              */
    int32_t* agents_alive;      /* optional [E]                                              */
    int32_t* step;              /* optional [E] step counter after this step                 */
    uint32_t flags;             /* MEV_DEVICE_PTRS | MEV_AUTO_RESET                           */
} mev_step_args;

/* Full simulator state, SoA.  Ego arrays are [E][N], NPC arrays [E][max_npcs].
 * Any NULL pointer is skipped.  Replaces EnvState/get_state/set_state
 * (reference cpp/EnvState.h:9-15, cpp/IntersectionEnv.cpp:394-416) and exposes
 * the Car fields the pybind layer hides (acc, steering_angle, spawn_state,
 * prev_dist_to_goal, prev_action; cpp/Car.h:16-46). */
typedef struct {
    float *x, *y, *v, *heading, *acc, *steering, *prev_dist, *prev_a0, *prev_a1;
    float *spawn_x, *spawn_y, *spawn_v, *spawn_heading;
    int32_t *path_index, *route, *intention;
    uint8_t* alive;
    float *npc_x, *npc_y, *npc_v, *npc_heading, *npc_acc, *npc_steering;
    int32_t *npc_path_index, *npc_route, *npc_intention;
    uint8_t* npc_alive;
    int32_t* npc_count;  /* [E] */
    int32_t* step_count; /* [E] */
} mev_state;

const char* mev_last_error(void);
int mev_abi_version(void);
int mev_device_count(int32_t* count);

int mev_config_default(mev_config* cfg);
int mev_create(const mev_config* cfg, mev_handle** out);
int mev_destroy(mev_handle* h);
int mev_get_config(const mev_handle* h, mev_config* cfg);
int mev_obs_dim(const mev_handle* h, int32_t* obs_dim);
/* A handle starts on its own non-blocking stream.  mev_set_stream orders all
 * later work on `stream` (a hipStream_t; NULL = the legacy default stream),
 * e.g. torch.cuda.current_stream().cuda_stream; mev_use_own_stream reverts. */
int mev_set_stream(mev_handle* h, void* stream);
int mev_use_own_stream(mev_handle* h);
int mev_sync(mev_handle* h);

/* Runtime reconfiguration, effective from the next step: reference
 * IntersectionEnv::configure / configure_traffic (cpp/IntersectionEnv.cpp:50-60)
 * and writes to its reward_config (env.py:57-77, cpp/Reward.h:5-14). */
int mev_configure(mev_handle* h, int32_t use_team, int32_t respawn, int32_t max_steps);
int mev_configure_traffic(mev_handle* h, int32_t enabled, float density);
int mev_set_reward(mev_handle* h, const float* reward8);

/* Host-side single-car helpers with the reference's exact arithmetic, for API
 * parity with the bound MARLEnv.Car methods (cpp/bindings.cpp:24-25); they do
 * not touch any device.  kin = {x, y, v, heading, acc, steering_angle}
 * (Car::update, cpp/Car.cpp:9-40); box = {x, y, heading, length, width}
 * (Car::check_collision, cpp/Car.cpp:86-141). */
int mev_car_update(float* kin, float throttle, float steer_input, float dt);
int mev_car_check_collision(const float* box_a, const float* box_b, int32_t* collide);

/* Lane points / routes (reference cpp/RouteGen.cpp). */
int mev_num_points(const mev_handle* h, int32_t* n);
int mev_point_xy(const mev_handle* h, int32_t point, float* xy);
int mev_route_id(const mev_handle* h, int32_t start_point, int32_t end_point, int32_t* route);
/* path [max(n, 160)][2], intent, spawn (x, y, heading) of a route of n points
 * (mev_route_len; a route of n < 160 points reads back padded with its last point) */
int mev_route_info(const mev_handle* h, int32_t route, float* path, int32_t* intent, float* spawn);
int mev_route_len(const mev_handle* h, int32_t route, int32_t* npoints);
int mev_path_len(void);
/* A route of the caller's own: path [npoints][2], 2 <= npoints <= 4096 (every
 * path the reference generates has 160, RouteGen.cpp:111-205), and intent (0
 * straight, 1 left, 2 right) appended to the handle's route table; *route
 * receives its id (>= P*P, the lane-layout routes).  Cars and NPCs then take it
 * like any route (mev_set_ego_routes, mev_set_state); a reset spawns at path[0]
 * heading to path[1].  Replaces assigning Car.path in the reference
 * (cpp/bindings.cpp:29, a read-write std::vector member): every reader clamps
 * to path.size() (Car.cpp:56, IntersectionEnv.cpp:177-179,446,
 * TrafficFlow.cpp:55,89,263), as the device does, also for a car whose
 * path_index lies past its path's end (set through mev_set_state: the index
 * search keeps it, the look-ahead clamps to path.back(), an NPC's ghost scan is
 * empty).  A path longer than the table's rows re-lays the table out at that
 * length rounded up to 16 points (one re-upload; every route keeps its ids).
 * mev_add_route(h, path, intent, route) = mev_add_route_n(h, path, 160, ...). */
int mev_add_route(mev_handle* h, const float* path, int32_t intent, int32_t* route);
int mev_add_route_n(mev_handle* h, const float* path, int32_t npoints, int32_t intent, int32_t* route);
/* Per-car size: reference Car::length / Car::width (cpp/Car.h:19-20), read-write through
 * cpp/bindings.cpp:24-25 and used by Car::corners (status tests and the SAT car-car
 * collision, Car.cpp:86-141) and by the LiDAR's box of each car (Lidar.cpp:65-75).
 * ego_dims [E][N][2] and npc_dims [E][max_npcs][2] hold (length, width) in px; NULL leaves
 * that array unchanged.  Every car starts at the reference's 54 x 24 px; a reset (and the
 * MEV_AUTO_RESET of mev_step) gives its egos that size again (new Cars, reference
 * IntersectionEnv::reset + add_car_with_route), a spawned NPC has it, a respawned ego keeps
 * its own (Car::respawn, Car.cpp:76-84); NPC sizes move with their NPCs.  Values must be
 * finite with |value| <= 1e4.  While any car differs from 54 x 24 the steps run the
 * runtime-layout kernels (k_cars + k_lidar or k_step without the compile-time layouts; no
 * step server) -- mev_car_dims_active says whether that is the case. */
int mev_set_car_dims(mev_handle* h, const float* ego_dims, const float* npc_dims);
int mev_get_car_dims(mev_handle* h, float* ego_dims, float* npc_dims);
int mev_car_dims_active(const mev_handle* h, int32_t* active);
/* LiDAR beam offsets (radians, [lidar_rays]): reference Lidar::rel_angles (cpp/Lidar.h:17,
 * read-write through cpp/bindings.cpp:92), by default the cfg's fov formula
 * (Lidar.cpp:4-14).  Lidar::update casts beam i along heading + rel_angles[i] for i < rays
 * (Lidar.cpp:24-25), so a reference Lidar whose rays was lowered casts the first rays
 * angles of its list: a handle of that many rays with those angles reproduces it.  Any
 * finite list with |angle| <= 1000 is taken; one the car-pair culling cannot model
 * linearly (uneven beyond 1e-5 rad, descending, constant, wider than a revolution) is
 * simulated without that culling (exact, slower). */
int mev_set_beam_angles(mev_handle* h, const float* rel);
int mev_get_beam_angles(mev_handle* h, float* rel);
/* Ego routes for every (env, agent): route ids [E][N] (reference env.py:104-106,148-151). */
int mev_set_ego_routes(mev_handle* h, const int32_t* routes);
/* NPC route list (reference configure_routes / init_traffic_routes, TrafficFlow.cpp:198-238). */
int mev_set_traffic_routes(mev_handle* h, const int32_t* routes, int32_t count);
int mev_default_traffic_routes(const mev_handle* h, int32_t* routes, int32_t* count);

/* Reset the envs selected by env_mask ([E], NULL = all): reference
 * IntersectionEnv::reset + add_car_with_route per agent (cpp/IntersectionEnv.cpp:66-131).
 * Writes the reset observation (LiDAR block = 1.0: no cast at reset). */
int mev_reset(mev_handle* h, const uint8_t* env_mask, float* obs, uint32_t flags);

/* One step of every env. */
int mev_step(mev_handle* h, const mev_step_args* args);

/* Outputs of the last step / reset, from the handle's own device buffers.
 * Lifetime: after a step that wrote caller-owned output buffers (device
 * pointers in mev_step_args), this call, mev_device_outputs and
 * mev_output_dlpack read those buffers -- keep them allocated and unmodified
 * until the next mev_step / mev_reset of the handle (or read the outputs from
 * them directly). */
int mev_get_outputs(mev_handle* h, float* obs, float* reward, uint8_t* done, uint8_t* status,
                    uint8_t* terminated, uint8_t* truncated, int32_t* agents_alive, int32_t* step,
                    uint32_t flags);

/* State snapshot / restore (host pointers).  mev_set_state recomputes the
 * observation with LiDAR = 1.0, as after a reset. */
int mev_get_state(mev_handle* h, const mev_state* out);
int mev_set_state(mev_handle* h, const mev_state* in);

/* Device pointers of the handle's internal output buffers (zero-copy consumers),
 * holding the last step's / reset's outputs: a step that wrote elsewhere (caller
 * buffers, the pinned block of a small host-mode step, a packed gather row) is
 * first copied into them on the handle's stream (caller buffers must still be
 * valid then: see mev_get_outputs).  Device-mode steps without output pointers
 * write them in place. */
int mev_device_outputs(mev_handle* h, float** obs, float** reward, uint8_t** done, uint8_t** status,
                       uint8_t** terminated, uint8_t** truncated);

/* Route randomisation at reset (the reference's test.py draws
 * a random route from the mapping on every reset, test.py:36-39,118-119): with
 * count > 0, every reset -- mev_reset and the MEV_AUTO_RESET of mev_step --
 * draws each agent's route uniformly from routes[0..count) (Philox keyed by the
 * handle seed, the reset counter, env and agent).  count = 0 restores fixed
 * routes (mev_set_ego_routes), the reference env.py behaviour. */
int mev_set_reset_routes(mev_handle* h, const int32_t* routes, int32_t count);

/* Device snapshots for batched rollbacks (EnvState +
 * get_state/set_state, reference cpp/EnvState.h:9-15, IntersectionEnv.cpp:394-416):
 * the whole state of every env plus the last step's outputs, in one
 * self-describing buffer of mev_snapshot_size bytes.  With MEV_DEVICE_PTRS the
 * buffer (and env_mask) live on the handle's device and the copies are
 * device-to-device.  mev_restore restores every env (env_mask NULL; also the
 * handle's Philox counter) or only the envs with env_mask[e] != 0; afterwards
 * mev_get_outputs returns the snapshot's outputs.  The car sizes (mev_set_car_dims)
 * are part of the state.  A snapshot restores only into a handle of the same shape
 * whose route table begins with the snapshot handle's routes (mev_add_route, same
 * paths in the same order); otherwise MEV_E_INVALID and the handle is unchanged. */
int mev_snapshot_size(mev_handle* h, uint64_t* bytes);
int mev_snapshot(mev_handle* h, void* dst, uint32_t flags);
int mev_restore(mev_handle* h, const void* src, const uint8_t* env_mask, uint32_t flags);

/* Diagnostics (cumulative): route ids in state-format gather messages this handle's route
 * table does not have (mev_unpack_gathered; their rows' look-ahead terms are NaN).
 * mev_comm_init already refuses ranks whose route tables differ. */
int mev_decode_errors(mev_handle* h, int64_t* count);
/* Diagnostics: spawns dropped because max_npcs was full (cumulative). */
int mev_npc_overflow(mev_handle* h, int64_t* count);
/* Diagnostics (cumulative): the spawn overflow above, and the NPC turns the
 * controller ran one after another because its parallel rounds disagreed
 * (mev_kernels.hip npc_phase: round B changed a throttle; results are the
 * sequential ones either way). */
int mev_npc_stats(mev_handle* h, int64_t* overflow, int64_t* sequential_turns);
/* Diagnostics: per-env phase timestamps [E][8] of the last step; all zero
 * unless the library was built with -DMEV_STAMPS (tools/phase_profile.py). */
int mev_debug_stamps(mev_handle* h, uint64_t* out);
/* Measurement: with timing enabled (every = n > 0), every n-th mev_step
 * records HIP events on the handle's stream before k_cars, between k_cars and
 * k_lidar, and after k_lidar (every = 0 disables).  mev_kernel_times returns
 * the summed device durations (ms) of the two kernels over the timed steps
 * and their count since the previous call (or since enabling), then clears
 * them; it waits for the recorded steps to finish.  With the fused step kernel
 * (mev_set_step_kernel) cars_ms holds k_step's duration and lidar_ms is 0. */
int mev_kernel_timing(mev_handle* h, int32_t every);
int mev_kernel_times(mev_handle* h, double* cars_ms, double* lidar_ms, int64_t* steps);
/* Scheduling (results are identical either way): which kernels run a step.
 * 1 = k_cars (one wave per env) then k_lidar (one wave per group of agents),
 * with the obstacle table handed over through HBM; 2 = the fused k_step, one
 * wave per env running both parts back to back from its LDS; 0 = automatic
 * (fused when its LDS -- car tables, NPC slots in traffic mode, one LiDAR pool
 * -- fits a wave's 10 KB share at 4 waves per SIMD, and E >= 1024 or an env's
 * beams fit one LiDAR group (N * R <= 256) or, without traffic, N <= 8 agents
 * and R <= 128 beams).  Asked for
 * explicitly, the fused kernel runs whenever that LDS fits one workgroup
 * (64 KB); otherwise the call fails with MEV_E_INVALID.  mev_get_step_kernel returns the kernel
 * the next step will use (1 or 2).  Replaces nothing in the reference (its
 * step is one sequential loop, cpp/IntersectionEnv.cpp:133-392). */
int mev_set_step_kernel(mev_handle* h, int32_t kernel);
int mev_get_step_kernel(const mev_handle* h, int32_t* kernel);
/* Scheduling (results are identical either way): envs per fused k_step wave.
 * With few agents per env (N <= 4, no traffic) 2, 4 or 8 envs share a wave's
 * 64 lanes (8 agent slots), so one wave's latency chain steps them all.
 * 0 = automatic; a request is reduced to fit N * envs <= 8.  mev_get_step_pack
 * returns what the next step uses (1 on the two-kernel path).  Replaces
 * nothing in the reference (one env per IntersectionEnv object). */
int mev_set_step_pack(mev_handle* h, int32_t envs_per_wave);
int mev_get_step_pack(const mev_handle* h, int32_t* envs_per_wave);
/* Scheduling (results are identical either way): two waves per fused k_step
 * workgroup -- the car part, then the LiDAR in one wave beside the rest of the
 * car part (rewards, flags, observation head) in the other.  0 = automatic (on
 * when the batch needs <= 2048 workgroups, i.e. <= 4 waves per SIMD, no traffic),
 * 1 = off, 2 = on (no traffic), 3 = early split (no traffic, one env per
 * workgroup, N * R <= 512: the LiDAR wave marches the road from the poses after
 * the kinematics while the car wave resolves collisions).  With traffic, one ego
 * per env, <= 32 NPC slots, R <= 128 and E a multiple of 16, the early split is
 * two envs per workgroup: one wave per env runs the NPC controller and the car
 * logic, one wave runs the two egos' kinematics, status and LiDAR beside them;
 * automatic (mode 0) and by 3.  mev_get_step_split
 * returns 1 (split) or 2 (early split) when the next step uses it.  Replaces
 * nothing in the reference. */
int mev_set_step_split(mev_handle* h, int32_t mode);
int mev_get_step_split(const mev_handle* h, int32_t* split);
/* Scheduling (results are identical either way): the NPC-aware env deal of the
 * fused traffic k_step -- workgroups take envs heaviest NPC count first, from
 * orders the previous step built.  on: 1 (default; MEV_NO_DEAL=1 in the
 * environment makes 0 the default), 0 = the XCD-aware identity order.  Replaces
 * nothing in the reference. */
int mev_set_env_deal(mev_handle* h, int32_t on);
/* Host-mode steps as a persistent step server (results are identical either
 * way).  A step with host buffers (no MEV_DEVICE_PTRS) of a small handle (<= 64
 * envs, outputs <= 256 KB, the fused kernel, no traffic above one ego / 32 NPC
 * slots) is answered by a kernel that stays resident between steps (k_serve):
 * the host posts the step in a mailbox of pinned memory and the kernel answers
 * once its outputs are there -- a PCIe round trip instead of a kernel launch and
 * a stream synchronisation.  The kernel leaves when no step is posted for its
 * idle limit and is launched again by the next one; every other call on the
 * handle stops it first.  Only on the handle's own stream (not after
 * mev_set_stream); the kernel itself runs on a non-blocking highest-priority
 * stream of its own; at most 2 servers are resident per process (other handles
 * step launched).  A server slot belongs to the handle that took it -- across its
 * server's idle exits and paused stretches -- until the handle is closed, turns
 * serving off, moves to another stream, or has made no host-mode step for 50 ms
 * when another handle asks for a slot; so a round-robin over more small handles
 * than slots serves the first two to step, whatever the timing of idle exits.
 * While it is resident, every device-wide wait of the process
 * (hipDeviceSynchronize, torch.cuda.synchronize(), frees that wait for the
 * device) waits for its idle exit, so the idle limit is adaptive: 8 x the
 * moving average of the host's time between an answer and the next post,
 * within [0.2, 2] ms; after 4 consecutive posts that found the server already
 * gone (a device-wide wait or a slow host between steps) the next 1024 host
 * steps are launched instead.  MEV_SERVE_IDLE_MS=n (1..1000) fixes the limit.
 * mode: 0 = off, 1 = automatic (default; MEV_NO_SERVE=1 in the environment
 * turns it off).  mev_serve_stats: steps served, server launches, whether one
 * is running.  Replaces nothing in the reference (its env.py steps one
 * IntersectionEnv per call on the CPU, cpp/bindings.cpp:53-55). */
int mev_set_serve(mev_handle* h, int32_t mode);
int mev_serve_stats(const mev_handle* h, uint64_t* steps, uint64_t* launches, int32_t* running);

/* ---- Multi-GPU: the per-step RCCL gather of the stacked outputs ----------
 * envs are sharded over the GPUs of a node, one process and
 * one handle per GPU, with no communication inside a step; the one collective
 * is a gather of every rank's step outputs to a root rank over xGMI.  The
 * reference has no counterpart (each IntersectionEnv is a single instance,
 * cpp/IntersectionEnv.h:23-105).
 *
 * Packed layout of one rank's outputs (slots = envs per rank, the largest
 * shard; a smaller shard leaves the tail of its slots unused), one contiguous
 * message per rank:
 *   obs f32 [slots][N][D] | reward f32 [slots][N] | done u8 [slots][N] |
 *   status u8 [slots][N] | terminated u8 [slots] | truncated u8 [slots]
 * each field 256-B aligned, the total padded to 256 B.  Host-only (no device). */
#define MEV_GATHER_TO_ROOT 0x4u /* mev_step: write the outputs packed and gather them to the root rank */
#define MEV_COMM_ID_BYTES 128   /* == NCCL_UNIQUE_ID_BYTES */
enum { MEV_PK_OBS = 0, MEV_PK_REWARD, MEV_PK_DONE, MEV_PK_STATUS, MEV_PK_TERMINATED, MEV_PK_TRUNCATED, MEV_PK_COUNT,
       MEV_PK_LIDAR = MEV_PK_COUNT /* compact formats only */, MEV_PK_STATE /* state format only */, MEV_PK_FIELDS };
int mev_packed_layout(int32_t slots, int32_t num_agents, int32_t obs_dim, uint64_t* offsets /*[MEV_PK_COUNT]*/,
                      uint64_t* bytes);
/* Gather formats (mev_set_gather_format, before mev_comm_init):
 *   MEV_GATHER_F32 (default): the layout above, obs rows as the plain step writes them;
 *   MEV_GATHER_LIDAR_U8: obs holds only each row's 31-float head, [slots][N][31], and a
 *     field MEV_PK_LIDAR, u8 [slots][N][lidar_slots], holds one code per beam: 0 no hit
 *     (max_dist), k + 1 a hit at march probe k, 255 a dead agent.  Lossless: the floats
 *     are table[code] (mev_lidar_decode_table, 256 entries), bit-identical to the plain
 *     step's; padding columns beyond 31 + lidar_slots are zero.  At R = 64, N = 8 a row
 *     shrinks from 380 B to 194 B (the message from 12.66 MB to 6.37 MB at 4096 envs).
 *   MEV_GATHER_STATE (no traffic): no observation field at all; the LiDAR codes as in
 *     MEV_GATHER_LIDAR_U8, and a field MEV_PK_STATE with each agent's post-step state
 *     as arrays of n = slots * N: x, y, v, heading f32 | route, path index i16 |
 *     intention, alive u8 (22 B per agent).  get_observations (cpp/IntersectionEnv.cpp:
 *     418-520) is a pure function of that state, so the root rebuilds the 31-float
 *     head with the step's own device code (mev_unpack_gathered), bit-identical to
 *     the plain step's rows.  At R = 64, N = 8 a row is 92 B instead of 380 B (the
 *     message 3.03 MB instead of 12.66 MB at 4096 envs); the ranks also skip the head.
 * mev_packed_layout2: offsets of all MEV_PK_FIELDS fields for any format (fields a
 * format does not use are empty).  Host-only. */
#define MEV_GATHER_F32 0
#define MEV_GATHER_LIDAR_U8 1
#define MEV_GATHER_STATE 2
int mev_packed_layout2(int32_t slots, int32_t num_agents, int32_t obs_dim, int32_t lidar_slots, int32_t format,
                       uint64_t* offsets /*[MEV_PK_FIELDS]*/, uint64_t* bytes);
int mev_set_gather_format(mev_handle* h, int32_t format);
int mev_lidar_decode_table(const mev_handle* h, float* table /*[256]*/);
/* ncclGetUniqueId: called by ONE process (any), then shared with every rank
 * out of band (e.g. a TCP store); id is MEV_COMM_ID_BYTES bytes. */
int mev_comm_unique_id(uint8_t* id);
/* Join the communicator of `world` ranks (ncclCommInitRank on the handle's
 * device; collective: every rank calls it) and allocate the double-buffered
 * packed buffers: two send buffers on a non-root rank, two [world][bytes]
 * gather buffers on the root.  slots = envs per rank of the largest shard
 * (0 = num_envs). */
int mev_comm_init(mev_handle* h, const uint8_t* id, int32_t world, int32_t rank, int32_t root, int32_t slots);
int mev_comm_destroy(mev_handle* h);
/* mev_step with MEV_GATHER_TO_ROOT (the args' obs/reward/done/status/
 * terminated/truncated pointers must be NULL): the step kernel writes this
 * rank's outputs straight into its packed slot (on the root: its row of the
 * gather buffer, no copy), then one grouped ncclSend (non-root) / ncclRecv
 * from every peer (root) runs on the handle's communication stream, ordered
 * after the step by an event, so it overlaps the next step.  Step t and t+2
 * share a buffer: step t+2 waits for gather t.  agents_alive / step still go
 * to the args' pointers (or the handle's own buffers).
 *
 * mev_gather_result (root): the gather buffer of the last gathered step,
 * [world][bytes] in rank order, and makes the handle's stream wait for that
 * gather (stream-ordered consumers on that stream then see every rank's rows).
 * mev_gather_wait: host wait for every gather issued so far, at most
 * timeout_ms (<= 0: no limit); on timeout the communicator is aborted and
 * MEV_E_HIP returned, so a lost peer cannot hang the caller forever. */
int mev_gather_result(mev_handle* h, void** stacked, uint64_t* bytes_per_rank, int32_t* world);
int mev_gather_wait(mev_handle* h, int32_t timeout_ms);
/* Root (any gather format): the float observation rows of a gathered buffer
 * `stacked` (device, [world][bytes] as mev_gather_result returns it, in the
 * handle's gather format and slots) into obs (device, [world][slots][N][D]), on
 * the handle's stream -- the rows each rank's plain step would have written, bit
 * for bit (F32: copied; LIDAR_U8: heads + decoded codes; STATE: heads rebuilt from
 * the shipped state).  Slots beyond a rank's envs hold whatever their (zeroed)
 * message decodes to.  Reward, done, status, terminated and truncated are read
 * from the buffer directly (mev_packed_layout2). */
int mev_unpack_gathered(mev_handle* h, const void* stacked, int32_t world, float* obs);

/* ---- Zero-copy export (DLPack) -----------------------------------------
 * the handle's device output buffers as DLPack tensors for
 * torch-free consumers (and torch.from_dlpack).  The structs below are the
 * DLPack v0.8 ABI (dlpack.h: DLDevice, DLDataType, DLTensor, DLManagedTensor),
 * restated so this header stays self-contained.  The tensor views memory the
 * handle owns: it is valid until mev_destroy; call its deleter when done (it
 * frees only the descriptor). */
typedef struct { int32_t device_type; int32_t device_id; } mev_dl_device; /* kDLROCM = 10 */
typedef struct { uint8_t code; uint8_t bits; uint16_t lanes; } mev_dl_dtype; /* kDLInt 0, kDLUInt 1, kDLFloat 2 */
typedef struct {
    void* data;
    mev_dl_device device;
    int32_t ndim;
    mev_dl_dtype dtype;
    int64_t* shape;
    int64_t* strides; /* NULL = compact row-major */
    uint64_t byte_offset;
} mev_dl_tensor;
typedef struct mev_dl_managed {
    mev_dl_tensor dl_tensor;
    void* manager_ctx;
    void (*deleter)(struct mev_dl_managed* self);
} mev_dl_managed;
enum { MEV_OUT_OBS = 0, MEV_OUT_REWARD, MEV_OUT_DONE, MEV_OUT_STATUS, MEV_OUT_TERMINATED, MEV_OUT_TRUNCATED,
       MEV_OUT_AGENTS_ALIVE, MEV_OUT_STEP, MEV_OUT_GATHERED /* root: [world][bytes] u8 of the last gather */,
       MEV_OUT_COUNT };
/* The handle's internal output buffer `which` (what mev_device_outputs returns,
 * brought up to the last outputs the same way) as a DLPack tensor:
 * obs [E][N][D] f32, reward [E][N] f32, done/status [E][N] u8,
 * terminated/truncated [E] u8, agents_alive/step [E] i32.  MEV_OUT_GATHERED
 * (root): the last gather's buffer; the handle's stream is made to wait for its
 * RCCL receives, as mev_gather_result does. */
int mev_output_dlpack(mev_handle* h, int32_t which, mev_dl_managed** out);

#ifdef __cplusplus
}
#endif

#endif /* MARLENV_H */
