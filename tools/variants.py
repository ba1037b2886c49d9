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

EXPERIMENTS = {"exp_noroad": ["-DMEV_EXP_NOROAD"], "exp_nocars": ["-DMEV_EXP_NOCARS"],
               "exp_none": ["-DMEV_EXP_NOROAD", "-DMEV_EXP_NOCARS"], "exp_iters": ["-DMEV_ITERS"],
               "stampsx": ["-DMEV_STAMPS", "-DMEV_STAMPS_X"], "stampsy": ["-DMEV_STAMPS", "-DMEV_STAMPS_Y"],
               "stampsr": ["-DMEV_STAMPS", "-DMEV_STAMPS_R"],
               # stampsr with slot 2 = end of cars_post (the split kernel's car wave)
               "stampsrp": ["-DMEV_STAMPS", "-DMEV_STAMPS_R", "-DMEV_STAMPS_POSTEND=1"],
               "stampsn": ["-DMEV_STAMPS_N"],  # NPC phase parts (tools/npc_profile.py --parts)
               # exact variants: probes per road-march step (product: 2)
               "npr1": ["-DMEV_LIDAR_NPR=1"], "npr3": ["-DMEV_LIDAR_NPR=3"],
               # exact variants: k_step issue priorities (product: cars 3, LiDAR phase 1 3 -> 2 after a
               # quarter of its agents, phase 2 1, phase 3 0); prio10 = the earlier cars 1 / LiDAR 0
               "prio10": ["-DMEV_PRIO_CARS=1", "-DMEV_PRIO_LIDAR=0", "-DMEV_PRIO_P1B=-1", "-DMEV_PRIO_P2=-1",
                          "-DMEV_PRIO_P3=-1"],
               "prio3210": ["-DMEV_PRIO_CARS=3", "-DMEV_PRIO_LIDAR=2", "-DMEV_PRIO_P1B=-1"],
               "prio_half": ["-DMEV_PRIO_P1B_AT=2"],
               "p2prio0": ["-DMEV_PRIO_P2=0"], "p2prio2": ["-DMEV_PRIO_P2=2"], "p3prio1": ["-DMEV_PRIO_P3=1"],
               "priohbm0": ["-DMEV_PRIO_HBM=0"],  # k_lidar without the LiDAR phases' priorities
               # the compiler's default machine scheduler instead of SCHED (k_step 41.6 -> 41.9 us)
               "sch_maxilp": ["-mllvm", "--amdgpu-sched-strategy=max-ilp"], "ilp1": ["-DMEV_PHASE1_ILP=1"],
               # k_cars' NPC-count priorities (product: level = NPCs left / 2): off / per NPC / per 3 NPCs
               # exact variant: the NPC controller's first move pass loads its path windows before the plans
               "npcprewin": ["-DMEV_NPC_PREWIN=1"],
               "npcpf": ["-DMEV_NPC_PREFETCH=1"],
               # exact variant: fdlibm's branchy atan2f in the observation head and NPC steering
               "noatanbf": ["-DMEV_ATAN_BF=0"],
               "noprefilter": ["-DMEV_NPC_PREFILTER=0"],
               # fused traffic: the rest of the step at a level by the env's NPC count (product: 3)
               "trafprio0": ["-DMEV_TRAFFIC_PRIO=0"], "trafprio2": ["-DMEV_TRAFFIC_PRIO=2"],
               "npcprio1": ["-DMEV_NPC_PRIO=1"], "npcprio3": ["-DMEV_NPC_PRIO=3"],
               "npcprio0": ["-DMEV_NPC_PRIO=0"],
               # timing-only (wrong results): NPC controller without ghost scans / without round B
               "x_noscan": ["-DMEV_X_NOSCAN"], "x_nob": ["-DMEV_X_NOB"], "x_noplan": ["-DMEV_X_NOPLAN"],
               "x_noseq": ["-DMEV_X_NOSEQ"],
               # (-fno-slp-vectorize is the product's since round 3; "slp" re-enables it)
               "slp": ["-fslp-vectorize"], "novec": ["-fno-vectorize"],
               # timing-only: k_step stopped after the car part / LiDAR phase 1 / 2 / 3 (instruction budgets)
               "stop1": ["-DMEV_EXP_STOP=1"], "stop2": ["-DMEV_EXP_STOP=2"], "stop3": ["-DMEV_EXP_STOP=3"],
               "stop4": ["-DMEV_EXP_STOP=4"], "stop0": ["-DMEV_EXP_STOP=0"],
               # timing-only: k_step without the observation head / the car-car SAT
               "nohead": ["-DMEV_EXP_NOHEAD"], "nosat": ["-DMEV_EXP_NOSAT"], "nowb": ["-DMEV_EXP_NOWB"],
               # exact variant: k_step's ego state write-back at its end (product: in cars_post)
               "wblate": ["-DMEV_WB_LATE=1"],
               # the road march's tail (product: helper groups from 16 beams, 3 probes per lane)
               "bfphys0": ["-DMEV_BF_PHYS=0"], "nostraight": ["-DMEV_LIDAR_STRAIGHT=0"],
               "nokeepskip": ["-DMEV_NPC_KEEPSKIP=0"], "solo": ["-DMEV_NPC_SOLO=1"], "nocircle": ["-DMEV_SAT_CIRCLE=0"], "noodc": ["-DMEV_NPC_ODC=0"], "far": ["-DMEV_NPC_FAR=1"], "probeint": ["-DMEV_PROBE_INT=1", "-DMEV_PROBE_PK=1"],
               "probepk": ["-DMEV_PROBE_PK=1"], "probeint1": ["-DMEV_PROBE_INT=1"],
               "earlypath": ["-DMEV_EARLY_PATH=1"], "scanpf": ["-DMEV_NPC_SCANPF=1"],
               "nosplit": ["-DMEV_SPLIT_MAX_WG=0"], "nohelptraf": ["-DMEV_HELP_TRAFFIC=0"],
               "skew1": ["-DMEV_EXP_SKEW=1"], "skew2": ["-DMEV_EXP_SKEW=2"], "skew4": ["-DMEV_EXP_SKEW=4"],
               "skewprio": ["-DMEV_EXP_SKEWPRIO"],
               "nohelp": ["-DMEV_MARCH_HELP=0"], "nprt6": ["-DMEV_MARCH_HELP=0", "-DMEV_LIDAR_NPR_TAIL=6"],
               "h8_3": ["-DMEV_MARCH_HELP=8"], "h32_3": ["-DMEV_MARCH_HELP=32"],
               "h16_2": ["-DMEV_NPT_HELP=2"], "h16_4": ["-DMEV_NPT_HELP=4"],
               # phase 1's first probes (product: 2)
               "npr1_1": ["-DMEV_LIDAR_NPR1=1"], "npr1_3": ["-DMEV_LIDAR_NPR1=3"],
               # the road march's steps with 3 probes before the tail (product: 2)
               "npr3": ["-DMEV_LIDAR_NPR=3"],
               # exact variants: k_step's cars_post after the LiDAR (product: before it), at the LiDAR's last
               # issue priority or a fixed one
               "postlate": ["-DMEV_POST_AFTER_LIDAR=1"], "postlate2": ["-DMEV_POST_AFTER_LIDAR=1", "-DMEV_PRIO_POST=2"],
               "headprio2": ["-DMEV_PRIO_HEAD=2"], "headprio1": ["-DMEV_PRIO_HEAD=1"],
               # exact variant: k_step's plain block -> env order (product: XCD-aware)
               "noxcd": ["-DMEV_XCD_REMAP=0"],
               "post1": ["-DMEV_POST_AFTER_LIDAR=1", "-DMEV_PRIO_POST=1"],
               "post3": ["-DMEV_POST_AFTER_LIDAR=1", "-DMEV_PRIO_POST=3"],
               # exact variant: k_step stages every output in LDS and writes whole rows at the end
               "staged": ["-DMEV_FUSED_STAGED=1"],
               # exact variant: the leading kernel arguments preloaded into SGPRs at wave launch (no kernarg
               # s_load round trip in front of the parameter loads)
               "kpreload": ["-mllvm", "-amdgpu-kernarg-preload-count=16"],
               # machine-scheduler options (exact): AMDGPU register-pressure trackers, no unclustered
               # high-pressure reschedule stage, latency over occupancy
               "trk": ["-mllvm", "-amdgpu-use-amdgpu-trackers=1"],
               "nounclust": ["-mllvm", "-amdgpu-disable-unclustered-high-rp-reschedule=1"],
               "bias0": ["-mllvm", "-amdgpu-schedule-metric-bias=0"],
               # the split kernel (car wave + LiDAR wave per workgroup) with 8 / 6 waves per SIMD
               "split8": ["-DMEV_SPLIT_WPE=8"], "split8i1": ["-DMEV_SPLIT_WPE=8", "-DMEV_PHASE1_ILP=1"],
               "split6": ["-DMEV_SPLIT_WPE=6"], "split5": ["-DMEV_SPLIT_WPE=5"],
               # the early split (mev_set_step_split(3)) without the car part's round-A group loads
               "eswpe6": ["-DMEV_ESPLIT_WPE=6"],
               "esilp2": ["-DMEV_ESPLIT_ILP=2"], "esroad2": ["-DMEV_PRIO_ESPLIT_ROAD=2"], "escars3": ["-DMEV_PRIO_ESPLIT_CARS=3"],
               "escars1": ["-DMEV_PRIO_ESPLIT_CARS=1"], "escp0": ["-DMEV_PRIO_ESPLIT_CARPHASE=0"], "x_es_nolidar": ["-DMEV_X_ES_NOLIDAR"],
               "stampses": ["-DMEV_STAMPS_ES"],
               # mixed order: odd residency slots march the road right after the kinematics
               "mix": ["-DMEV_MIX=1"], "mixp0": ["-DMEV_MIX=1", "-DMEV_PRIO_MIX_ROAD=0"],
               "mixp2": ["-DMEV_MIX=1", "-DMEV_PRIO_MIX_ROAD=2"], "mixs11": ["-DMEV_MIX=1", "-DMEV_MIX_SHIFT=11"],
               "mixs0": ["-DMEV_MIX=1", "-DMEV_MIX_SHIFT=0"],
               # traffic: the NPC write-back and the deal's append at the end of k_step (product: where the
               # NPC phase / the car part ends)
               # k_step's register allocation aimed at exactly 4 waves per SIMD (up to 128 VGPRs)
               "wpe44": ["-DMEV_KSTEP_ATTR=__attribute__((amdgpu_waves_per_eu(4,4)))"],
               "relaxocc": ["-mllvm", "--amdgpu-schedule-relaxed-occupancy"],
               "npcwblate": ["-DMEV_NPC_DEFER_WB=1"], "deallate": ["-DMEV_DEAL_LATE=1"],
               "bothlate": ["-DMEV_NPC_DEFER_WB=1", "-DMEV_DEAL_LATE=1"],
               # deliberately wrong: beam spans narrowed, to show the stress test catches it
               "exp_badrange": ["-DMEV_EXP_BADRANGE"]}


def build(name: str, force: bool = False) -> str:
    if name in _build.VARIANTS:
        return _build.build(force=force, verbose=True, variant=name)
    return _build.build(force=force, verbose=True, variant=name, flags=EXPERIMENTS[name])


if __name__ == "__main__":
    names = list(EXPERIMENTS) if "--all" in sys.argv else [a for a in sys.argv[1:] if not a.startswith("-")]
    for n in names:
        print(build(n, force="--force" in sys.argv))
