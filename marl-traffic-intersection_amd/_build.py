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


# the product library ("") and the diagnostic timestamp build ("stamps", tools/phase_profile.py).
# Experiment builds (timing-only and exact A/B variants) live in tools/variants.py and pass their
# flags to build(..., flags=...); they are never built by __graft_entry__.build().
VARIANTS = {"": [], "stamps": ["-DMEV_STAMPS"]}


def lib_path(variant: str = "") -> str:
    return LIB_PATH if not variant else os.path.join(PKG_DIR, f"libmarlenv_hip_{variant}.so")


def up_to_date(variant: str = "") -> bool:
    path = lib_path(variant)
    if not os.path.exists(path):
        return False
    t = os.path.getmtime(path)
    return all(os.path.getmtime(f) <= t for f in _inputs())


def build(force: bool = False, verbose: bool = False, variant: str = "", flags=None) -> str:
    """Compile variant `variant` (VARIANTS, or an experiment whose hipcc `flags` the caller passes)."""
    path = lib_path(variant)
    if not force and up_to_date(variant):
        return path
    if flags is None:
        if variant not in VARIANTS:
            raise KeyError(f"unknown library variant {variant!r} (experiment builds: tools/variants.py)")
        flags = VARIANTS[variant]
    tmp = path + ".tmp"
    # LLVM's default machine scheduler (max-ilp was +0.7 % in round 1, 0.5 % slower on the round-2 kernel).
    # No SLP vectorization: packed v_pk_mul/add_f32 cost gfx950 more issue cycles than the scalar pairs
    # they replace, plus the v_mov shuffles and hazard s_nops around them (config 3 35.0 -> 33.9 us,
    # config 5 55.5 -> 53.0 us per step; config 2 -1.4 %: profiles/r3_ab_noslp.txt).  Exact: the same
    # IEEE operations, unfused.
    cmd = [_hipcc(), "-O3", "-std=c++17", f"--offload-arch={ARCH}", "-ffp-contract=off", "-fno-slp-vectorize",
           "-fPIC", "-shared", "-Wall", "-Wno-unused-function", "-I", INCLUDE, "-I", CSRC] + list(flags)
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
    if "--all" in sys.argv:
        print(build(force="--force" in sys.argv, verbose=True, variant="stamps"))
