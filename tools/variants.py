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
               # the traffic early split (mev_set_step_split(3)): timing-only cuts -- the LiDAR wave
               # without its work after barrier B / without any work, the car waves without cars_post
               # -- and the LiDAR wave's phase 1 at two agents per pass (exact)
               "ts1": ["-DMEV_EXP_TS=1"], "ts2": ["-DMEV_EXP_TS=2"], "ts3": ["-DMEV_EXP_TS=3"],
               "tsilp2": ["-DMEV_TS_ILP=2"], "ts2env": ["-DMEV_TS_ENVS=2"], "tswpe5": ["-DMEV_TS_WPE=5"], "tslp3": ["-DMEV_TS_LPRIO=3"], "tslp2": ["-DMEV_TS_LPRIO=2"],
               "tslp0": ["-DMEV_TS_LPRIO=0"], "tslp1c3": ["-DMEV_TS_CPRIO=3"],
               # the LiDAR wave of workgroups whose envs all hold fewer than T NPCs at level L
               "tsad2l2": ["-DMEV_TS_ADAPT=2", "-DMEV_TS_ALPRIO=2"], "tsad2l3": ["-DMEV_TS_ADAPT=2", "-DMEV_TS_ALPRIO=3"],
               "tsad1l3": ["-DMEV_TS_ADAPT=1", "-DMEV_TS_ALPRIO=3"],
               # the early split without traffic: the road march's / the car wave's issue level
               "esr2": ["-DMEV_ES_RPRIO=2"], "esr1": ["-DMEV_ES_RPRIO=1"], "esc3": ["-DMEV_ES_CPRIO=3"], "tswpe7": ["-DMEV_TS_WPE=7"],
               "tsb64": ["-DMEV_TS_BEAMS=64"], "ts2b64": ["-DMEV_TS_BEAMS=64", "-DMEV_EXP_TS=2"],
               # compiler options (exact): SLP vectorization back on, no loop vectorization, the max-ilp
               # scheduler, kernel-argument preloading, AMDGPU register-pressure trackers, no unclustered
               # high-pressure reschedule stage, latency over occupancy, relaxed occupancy
               "slp": ["-fslp-vectorize"], "novec": ["-fno-vectorize"],
               "sch_maxilp": ["-mllvm", "--amdgpu-sched-strategy=max-ilp"],
               "kpreload": ["-mllvm", "-amdgpu-kernarg-preload-count=16"],
               "trk": ["-mllvm", "-amdgpu-use-amdgpu-trackers=1"],
               "nounclust": ["-mllvm", "-amdgpu-disable-unclustered-high-rp-reschedule=1"],
               "bias0": ["-mllvm", "-amdgpu-schedule-metric-bias=0"],
               "relaxocc": ["-mllvm", "--amdgpu-schedule-relaxed-occupancy"]}


def build(name: str, force: bool = False) -> str:
    if name in _build.VARIANTS:
        return _build.build(force=force, verbose=True, variant=name)
    return _build.build(force=force, verbose=True, variant=name, flags=EXPERIMENTS[name])


if __name__ == "__main__":
    names = list(EXPERIMENTS) if "--all" in sys.argv else [a for a in sys.argv[1:] if not a.startswith("-")]
    for n in names:
        print(build(n, force="--force" in sys.argv))
