"""Build the gfx950 extension in-tree: marl-traffic-intersection_amd/libmarlenv_hip.so.

hipcc cross-compiles for gfx950 without a GPU, so this runs in the build
container (``__graft_entry__.build()``) and the resulting .so travels to the GPU
box with the repository snapshot.  All simulator code is compiled with
-ffp-contract=off: the reference is an SSE (no-FMA) x86-64 build and the
device path must round exactly like it ("Bit-exactness").
"""
from __future__ import annotations

import os
import shutil
import subprocess
import sys

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG_DIR)
CSRC = os.path.join(PKG_DIR, "csrc")
INCLUDE = os.path.join(ROOT, "include")
LIB_NAME = "libmarlenv_hip.so"
LIB_PATH = os.path.join(PKG_DIR, LIB_NAME)
SOURCES = ["mev_kernels.hip", "mev_capi.cpp"]
ARCH = os.environ.get("MEV_OFFLOAD_ARCH", "gfx950")


def _hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found (ROCm required to build libmarlenv_hip.so)")


def _inputs():
    files = [os.path.join(CSRC, f) for f in os.listdir(CSRC)] + [os.path.join(INCLUDE, "marlenv.h"), __file__]
    return [f for f in files if os.path.isfile(f)]


VARIANTS = {"": [], "stamps": ["-DMEV_STAMPS"]}
# machine scheduling: LLVM's default strategy (max-ilp was +0.7 % in round 1; with the round-2 kernel the
# default is +0.5 % at config 3, even at config 4: variant sch_maxilp)
SCHED = []
# timing-only experiment builds (wrong results by construction; never used by the product)
EXPERIMENTS = {"exp_noroad": ["-DMEV_EXP_NOROAD"], "exp_nocars": ["-DMEV_EXP_NOCARS"],
               "exp_none": ["-DMEV_EXP_NOROAD", "-DMEV_EXP_NOCARS"], "exp_iters": ["-DMEV_ITERS"],
               "stampsx": ["-DMEV_STAMPS", "-DMEV_STAMPS_X"], "stampsy": ["-DMEV_STAMPS", "-DMEV_STAMPS_Y"],
               "stampsr": ["-DMEV_STAMPS", "-DMEV_STAMPS_R"],
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
               "sch_maxilp": [], "ilp1": ["-DMEV_PHASE1_ILP=1"],
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
               # deliberately wrong: beam spans narrowed, to show the stress test catches it
               "exp_badrange": ["-DMEV_EXP_BADRANGE"]}
VARIANTS.update(EXPERIMENTS)


def lib_path(variant: str = "") -> str:
    return LIB_PATH if not variant else os.path.join(PKG_DIR, f"libmarlenv_hip_{variant}.so")


def up_to_date(variant: str = "") -> bool:
    path = lib_path(variant)
    if not os.path.exists(path):
        return False
    t = os.path.getmtime(path)
    return all(os.path.getmtime(f) <= t for f in _inputs())


def build(force: bool = False, verbose: bool = False, variant: str = "") -> str:
    path = lib_path(variant)
    if not force and up_to_date(variant):
        return path
    tmp = path + ".tmp"
    sched = ["-mllvm", "--amdgpu-sched-strategy=max-ilp"] if variant == "sch_maxilp" else SCHED
    cmd = [_hipcc(), "-O3", "-std=c++17", f"--offload-arch={ARCH}", "-ffp-contract=off", "-fPIC", "-shared",
           "-Wall", "-Wno-unused-function", "-I", INCLUDE, "-I", CSRC] + sched + VARIANTS[variant]
    cmd += [os.path.join(CSRC, s) for s in SOURCES]
    # RCCL for the multi-GPU gather (mev_comm_*); when torch is imported first its
    # bundled librccl.so (same SONAME librccl.so.1) satisfies this dependency,
    # as its libamdhip64.so satisfies libamdhip64.so.7: one runtime per process
    cmd += ["-L", "/opt/rocm/lib", "-lrccl", "-o", tmp]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed ({r.returncode}):\n{r.stderr[-6000:]}")
    os.replace(tmp, path)
    return path


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
    if "--all" in sys.argv or "--exp" in sys.argv:
        for v in VARIANTS:
            if v and (v in EXPERIMENTS) == ("--exp" in sys.argv):
                print(build(force="--force" in sys.argv, verbose=True, variant=v))
