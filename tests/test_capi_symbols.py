"""The C-ABI library builds, loads without a GPU, and exports every function
include/marlenv.h declares (no compute calls: this runs on the CPU box)."""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared():
    src = open(os.path.join(ROOT, "include", "marlenv.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(mev_[a-z_0-9]+)\s*\(", src)))


def test_header_declares_the_boundary():
    names = declared()
    for must in ("mev_create", "mev_destroy", "mev_reset", "mev_step", "mev_get_state", "mev_set_state",
                 "mev_set_ego_routes", "mev_set_traffic_routes", "mev_last_error"):
        assert must in names


def test_library_exports_every_declared_symbol(mev):
    lib = mev.load_library()
    missing = [n for n in declared() if not hasattr(lib, n)]
    assert not missing, missing
    assert set(mev._capi.EXPORTED) == set(declared())


def test_abi_and_defaults_without_gpu(mev):
    lib = mev.load_library()
    assert lib.mev_abi_version() == 3  # 3: per-car sizes, beam angles, snapshot format 2
    assert lib.mev_path_len() == 160
    cfg = mev._capi.default_config()
    # reference defaults: 96 beams (IntersectionEnv.cpp:113), RewardConfig (Reward.h:5-14), max_steps 2000
    assert cfg["lidar_rays"] == 96 and cfg["max_steps"] == 2000 and cfg["num_lanes"] == 3
    assert [round(x, 4) for x in cfg["reward"]] == [10.0, 1.0, -0.01, -10.0, -5.0, 10.0, -0.02, 0.2]


def test_create_fails_loudly_without_device(mev):
    if mev.device_count() > 0:
        pytest.skip("a HIP device is present")
    with pytest.raises(mev.MevError):
        mev.Handle(num_envs=2)


def test_invalid_config_is_rejected(mev):
    lib = mev.load_library()
    c = mev._capi.MevConfig()
    lib.mev_config_default(ctypes.byref(c))
    c.num_agents = 65
    h = ctypes.c_void_p()
    assert lib.mev_create(ctypes.byref(c), ctypes.byref(h)) == -1
    assert b"num_agents" in lib.mev_last_error()


def test_one_hip_runtime_with_torch():
    """With PyTorch installed, loading the library leaves ONE HIP runtime in the
    process: torch's libamdhip64 / librccl (imported first by _capi) satisfy the
    library's NEEDED libamdhip64.so.7 / librccl.so.1 (checked in a fresh
    process, from /proc/self/maps; no GPU call)."""
    import subprocess
    import sys
    code = ("import sys; sys.path.insert(0, %r); import pkgload; pkgload.load()._capi.load_library(); "
            "libs = sorted({l.split()[-1] for l in open('/proc/self/maps') if 'libamdhip64' in l or 'librccl' in l}); "
            "print('\\n'.join(libs))") % ROOT
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300, check=True).stdout
    hip = [l for l in out.split() if "libamdhip64" in l]
    rccl = [l for l in out.split() if "librccl" in l]
    assert len(hip) == 1, hip
    assert len(rccl) == 1, rccl
