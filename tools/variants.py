"""Experiment builds of libmarlenv_hip.so (never built or shipped by __graft_entry__.build()).

Timing-only variants (wrong results by construction) and exact A/B variants measured during the
kernel work; DESIGN.md §9 records what each showed.  Build one with

    python tools/variants.py NAME [NAME ...]      (or --all)

and select it at run time with MEV_LIB_VARIANT=NAME (marl_traffic_intersection_amd/_capi.py).
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "marl-traffic-intersection_amd"))
import _build  # noqa: E402

# Round 4 removed the source-level experiment variants (exact A/B variants and
# timing-only cuts measured and rejected in rounds 1-3: DESIGN.md §9 keeps their
# numbers; the code is in git history up to commit 00b72c8).  What remains: the
# diagnostic stamp builds, the timing-only stop builds of the phase budgets and
# compiler-flag variants (no source macros).
EXPERIMENTS = {"stampsr": ["-DMEV_STAMPS", "-DMEV_STAMPS_R"],
               # stampsr with slot 2 = end of cars_post (the split kernel's car wave)
               "stampsrp": ["-DMEV_STAMPS", "-DMEV_STAMPS_R", "-DMEV_STAMPS_POSTEND=1"],
               "stampsn": ["-DMEV_STAMPS_N"],  # NPC phase parts (tools/npc_profile.py --parts)
               "stampsq": ["-DMEV_STAMPS_Q"],  # eight LDS-held stamps per step (tools/qstamp_profile.py)
               # timing-only: k_step stopped after the car part / LiDAR phase 1 / 2 / 3 (instruction budgets)
               "stop1": ["-DMEV_EXP_STOP=1"], "stop2": ["-DMEV_EXP_STOP=2"], "stop3": ["-DMEV_EXP_STOP=3"],
               "stop4": ["-DMEV_EXP_STOP=4"], "stop0": ["-DMEV_EXP_STOP=0"],
               # (round 5's traffic / early-split variants -- timing cuts ts1-3, tsb64, ts2env, tswpe*,
               # tsilp2, tslp*, tsad*, esr*, esc3 -- were removed from the sources after measuring; their
               # results are in DESIGN.md §9 / §3.1e, the macros in git history up to commit 55a6684)
               # compiler options (exact): SLP vectorization back on, no loop vectorization, the max-ilp
               # scheduler, kernel-argument preloading, AMDGPU register-pressure trackers, no unclustered
               # high-pressure reschedule stage, latency over occupancy, relaxed occupancy
               "slp": ["-fslp-vectorize"], "novec": ["-fno-vectorize"],
               "sch_maxilp": ["-mllvm", "--amdgpu-sched-strategy=max-ilp"],
               "kpreload": ["-mllvm", "-amdgpu-kernarg-preload-count=16"],
               "trk": ["-mllvm", "-amdgpu-use-amdgpu-trackers=1"],
               "nounclust": ["-mllvm", "-amdgpu-disable-unclustered-high-rp-reschedule=1"],
               "bias0": ["-mllvm", "-amdgpu-schedule-metric-bias=0"],
               "relaxocc": ["-mllvm", "--amdgpu-schedule-relaxed-occupancy"],
               # the dense phase-1 walk (R not a multiple of 64) at 3 / 4 chunks per pass instead of 2
               "dilp3": ["-DMEV_DENSE_ILP=3"], "dilp4": ["-DMEV_DENSE_ILP=4"],
               # the traffic early split with 2 / 4 envs (car waves) per workgroup
               "ts2": ["-DMEV_TSPLIT_ENVS=2"], "ts4": ["-DMEV_TSPLIT_ENVS=4"],
               # ... with its LiDAR wave at issue level 0 / 2 / 3 before barrier H (1 otherwise)
               "ts2p0": ["-DMEV_TSPLIT_ENVS=2", "-DMEV_TSPLIT_LPRIO=0"],
               "ts2p2": ["-DMEV_TSPLIT_ENVS=2", "-DMEV_TSPLIT_LPRIO=2"],
               "ts2p3": ["-DMEV_TSPLIT_ENVS=2", "-DMEV_TSPLIT_LPRIO=3"],
               # ... with its car waves starting at issue level 1 / 3 (2 otherwise)
               "tsc1": ["-DMEV_TSPLIT_CPRIO=1"], "tsc3": ["-DMEV_TSPLIT_CPRIO=3"],
               # timing-only: LiDAR phase 1's beam directions by the hardware sin/cos instead of the
               # glibc-exact double-precision sincosf (the upper bound of a cheaper exact one)
               "fastsin": ["-DMEV_EXP_FASTSIN"],
               # the NPC controller's issue level = NPCs / 1 or / 3 (2 otherwise)
               "npcp1": ["-DMEV_NPC_PRIO=1"], "npcp3": ["-DMEV_NPC_PRIO=3"],
               # timing-only: the early splits' LiDAR waves without their road march before barrier H / B
               # (what the light workgroups' wait for it costs config 4 at most)
               "tsnomarch": ["-DMEV_EXP_TSNOMARCH"],
               # timing-only: the NPC controller without its round B (round A's moves final): its share
               "noroundb": ["-DMEV_EXP_NOROUNDB"],
               # k_step's phase-1 ILP (agents per pass) 3 / 4, the early split's 2, LiDAR probes per ray 1 / 4
               "p1ilp3": ["-DMEV_PHASE1_ILP=3"], "p1ilp4": ["-DMEV_PHASE1_ILP=4"], "eilp2": ["-DMEV_ESPLIT_ILP=2"],
               "npr1": ["-DMEV_LIDAR_NPR=1"], "npr4": ["-DMEV_LIDAR_NPR=4"]}


def build(name: str, force: bool = False) -> str:
    if name in _build.VARIANTS:
        return _build.build(force=force, verbose=True, variant=name)
    return _build.build(force=force, verbose=True, variant=name, flags=EXPERIMENTS[name])


if __name__ == "__main__":
    names = list(EXPERIMENTS) if "--all" in sys.argv else [a for a in sys.argv[1:] if not a.startswith("-")]
    for n in names:
        print(build(n, force="--force" in sys.argv))
