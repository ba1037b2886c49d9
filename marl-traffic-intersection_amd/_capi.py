"""ctypes binding of libmarlenv_hip.so (include/marlenv.h).

The product path: every simulator computation happens in the gfx950 library;
this module only marshals buffers.  Importing works without a GPU (the CPU
test-suite checks the exported symbols), but creating a handle requires the
HIP runtime and a device — there is NO CPU fallback: a missing library or
device raises.
"""
from __future__ import annotations

import ctypes
import operator
import os
from typing import Dict, Optional

import numpy as np

from . import _build

LIB_PATH = _build.LIB_PATH

MEV_DEVICE_PTRS = 0x1
MEV_AUTO_RESET = 0x2
MEV_GATHER_TO_ROOT = 0x4
MEV_COMM_ID_BYTES = 128
MEV_GATHER_F32 = 0
MEV_GATHER_LIDAR_U8 = 1
MEV_GATHER_STATE = 2
STATE_BYTES_PER_AGENT = 22
# packed-output fields (mev_packed_layout2) and DLPack outputs (mev_output_dlpack), include/marlenv.h order
PACKED_FIELDS = ("obs", "reward", "done", "status", "terminated", "truncated", "lidar", "state")
DLPACK_OUTPUTS = ("obs", "reward", "done", "status", "terminated", "truncated", "agents_alive", "step", "gathered")

STATUS_NAMES = ("ALIVE", "DEAD", "SUCCESS", "CRASH_WALL", "CRASH_LINE", "CRASH_CAR")
PATH_LEN = 160  # every lane-layout route
MAX_PATH_LEN = 4096  # a written path (mev_add_route_n)

# exported symbols that include/marlenv.h declares (checked by tests/test_capi_symbols.py)
EXPORTED = (
    "mev_last_error", "mev_abi_version", "mev_device_count", "mev_config_default", "mev_create", "mev_destroy",
    "mev_get_config", "mev_obs_dim", "mev_set_stream", "mev_sync", "mev_num_points", "mev_point_xy",
    "mev_route_id", "mev_route_info", "mev_route_len", "mev_path_len", "mev_set_ego_routes", "mev_set_traffic_routes",
    "mev_default_traffic_routes", "mev_reset", "mev_step", "mev_get_outputs", "mev_get_state", "mev_set_state",
    "mev_device_outputs", "mev_npc_overflow", "mev_npc_stats", "mev_use_own_stream", "mev_debug_stamps",
    "mev_configure", "mev_configure_traffic", "mev_set_reward", "mev_car_update", "mev_car_check_collision",
    "mev_kernel_timing", "mev_kernel_times", "mev_set_reset_routes", "mev_snapshot_size", "mev_snapshot",
    "mev_restore", "mev_set_step_kernel", "mev_get_step_kernel", "mev_set_step_pack", "mev_get_step_pack",
    "mev_set_step_split", "mev_get_step_split", "mev_set_env_deal", "mev_set_serve", "mev_serve_stats",
    "mev_packed_layout", "mev_comm_unique_id", "mev_comm_init", "mev_comm_destroy", "mev_gather_result",
    "mev_gather_wait", "mev_output_dlpack", "mev_packed_layout2", "mev_set_gather_format", "mev_lidar_decode_table",
    "mev_unpack_gathered", "mev_add_route", "mev_add_route_n", "mev_set_car_dims", "mev_get_car_dims", "mev_car_dims_active",
    "mev_set_beam_angles", "mev_get_beam_angles", "mev_decode_errors",
)


class MevConfig(ctypes.Structure):
    _fields_ = [
        ("num_envs", ctypes.c_int32), ("num_agents", ctypes.c_int32), ("num_lanes", ctypes.c_int32),
        ("lidar_rays", ctypes.c_int32), ("lidar_fov_deg", ctypes.c_float), ("lidar_max_dist", ctypes.c_float),
        ("lidar_step", ctypes.c_float), ("obs_dim", ctypes.c_int32), ("traffic_flow", ctypes.c_int32),
        ("traffic_density", ctypes.c_float), ("use_team_reward", ctypes.c_int32), ("respawn_enabled", ctypes.c_int32),
        ("max_steps", ctypes.c_int32), ("reward", ctypes.c_float * 8), ("max_npcs", ctypes.c_int32),
        ("seed", ctypes.c_uint64), ("device", ctypes.c_int32),
    ]


_vp = ctypes.c_void_p


class MevStepArgs(ctypes.Structure):
    _fields_ = [
        ("actions", _vp), ("dt", ctypes.c_float), ("spawn_route", _vp), ("obs", _vp), ("reward", _vp),
        ("done", _vp), ("status", _vp), ("terminated", _vp), ("truncated", _vp), ("agents_alive", _vp),
        ("step", _vp), ("flags", ctypes.c_uint32),
    ]


# (name, dtype, per) — per: "ego" [E*N], "npc" [E*K], "env" [E]; order == struct mev_state
STATE_FIELDS = (
    ("x", np.float32, "ego"), ("y", np.float32, "ego"), ("v", np.float32, "ego"), ("heading", np.float32, "ego"),
    ("acc", np.float32, "ego"), ("steering", np.float32, "ego"), ("prev_dist", np.float32, "ego"),
    ("prev_a0", np.float32, "ego"), ("prev_a1", np.float32, "ego"), ("spawn_x", np.float32, "ego"),
    ("spawn_y", np.float32, "ego"), ("spawn_v", np.float32, "ego"), ("spawn_heading", np.float32, "ego"),
    ("path_index", np.int32, "ego"), ("route", np.int32, "ego"), ("intention", np.int32, "ego"),
    ("alive", np.uint8, "ego"),
    ("npc_x", np.float32, "npc"), ("npc_y", np.float32, "npc"), ("npc_v", np.float32, "npc"),
    ("npc_heading", np.float32, "npc"), ("npc_acc", np.float32, "npc"), ("npc_steering", np.float32, "npc"),
    ("npc_path_index", np.int32, "npc"), ("npc_route", np.int32, "npc"), ("npc_intention", np.int32, "npc"),
    ("npc_alive", np.uint8, "npc"), ("npc_count", np.int32, "env"), ("step_count", np.int32, "env"),
)


class MevState(ctypes.Structure):
    _fields_ = [(name, _vp) for name, _, _ in STATE_FIELDS]


_libs = {}
VARIANT = os.environ.get("MEV_LIB_VARIANT", "")  # "" = product library; "stamps" = diagnostic build


def lib_available() -> bool:
    return os.path.exists(LIB_PATH)


def load_library(variant: str = None):
    """Load libmarlenv_hip.so (building it first when hipcc is present)."""
    variant = VARIANT if variant is None else variant
    if variant in _libs:
        return _libs[variant]
    path = _build.lib_path(variant)
    _one_runtime()
    if not _build.up_to_date(variant) and variant in _build.VARIANTS:  # experiments: tools/variants.py builds them
        try:
            _build.build(variant=variant)
        except Exception as exc:  # no hipcc on this machine: use a prebuilt library if it is there
            if not os.path.exists(path):
                raise RuntimeError(f"{os.path.basename(path)} is missing and could not be built: {exc}") from exc
    L = ctypes.CDLL(path)
    i32p = ctypes.POINTER(ctypes.c_int32)
    f32p = ctypes.POINTER(ctypes.c_float)
    L.mev_last_error.restype = ctypes.c_char_p
    L.mev_config_default.argtypes = [ctypes.POINTER(MevConfig)]
    L.mev_create.argtypes = [ctypes.POINTER(MevConfig), ctypes.POINTER(_vp)]
    L.mev_destroy.argtypes = [_vp]
    L.mev_get_config.argtypes = [_vp, ctypes.POINTER(MevConfig)]
    L.mev_obs_dim.argtypes = [_vp, i32p]
    L.mev_set_stream.argtypes = [_vp, _vp]
    L.mev_sync.argtypes = [_vp]
    L.mev_num_points.argtypes = [_vp, i32p]
    L.mev_point_xy.argtypes = [_vp, ctypes.c_int32, f32p]
    L.mev_route_id.argtypes = [_vp, ctypes.c_int32, ctypes.c_int32, i32p]
    L.mev_route_info.argtypes = [_vp, ctypes.c_int32, f32p, i32p, f32p]
    L.mev_set_ego_routes.argtypes = [_vp, i32p]
    L.mev_set_traffic_routes.argtypes = [_vp, i32p, ctypes.c_int32]
    L.mev_default_traffic_routes.argtypes = [_vp, i32p, i32p]
    L.mev_reset.argtypes = [_vp, _vp, _vp, ctypes.c_uint32]
    L.mev_step.argtypes = [_vp, ctypes.POINTER(MevStepArgs)]
    L.mev_get_outputs.argtypes = [_vp] + [_vp] * 8 + [ctypes.c_uint32]
    L.mev_get_state.argtypes = [_vp, ctypes.POINTER(MevState)]
    L.mev_set_state.argtypes = [_vp, ctypes.POINTER(MevState)]
    L.mev_device_outputs.argtypes = [_vp] + [ctypes.POINTER(_vp)] * 6
    L.mev_npc_overflow.argtypes = [_vp, ctypes.POINTER(ctypes.c_int64)]
    L.mev_npc_stats.argtypes = [_vp, ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_int64)]
    L.mev_device_count.argtypes = [i32p]
    L.mev_use_own_stream.argtypes = [_vp]
    L.mev_debug_stamps.argtypes = [_vp, ctypes.POINTER(ctypes.c_uint64)]
    L.mev_kernel_timing.argtypes = [_vp, ctypes.c_int32]
    L.mev_set_reset_routes.argtypes = [_vp, i32p, ctypes.c_int32]
    L.mev_snapshot_size.argtypes = [_vp, ctypes.POINTER(ctypes.c_uint64)]
    L.mev_snapshot.argtypes = [_vp, _vp, ctypes.c_uint32]
    L.mev_restore.argtypes = [_vp, _vp, _vp, ctypes.c_uint32]
    L.mev_kernel_times.argtypes = [_vp, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double),
                                   ctypes.POINTER(ctypes.c_int64)]
    L.mev_set_step_kernel.argtypes = [_vp, ctypes.c_int32]
    L.mev_get_step_kernel.argtypes = [_vp, i32p]
    L.mev_set_step_pack.argtypes = [_vp, ctypes.c_int32]
    L.mev_get_step_pack.argtypes = [_vp, i32p]
    L.mev_set_step_split.argtypes = [_vp, ctypes.c_int32]
    L.mev_set_env_deal.argtypes = [_vp, ctypes.c_int32]
    L.mev_get_step_split.argtypes = [_vp, i32p]
    L.mev_set_serve.argtypes = [_vp, ctypes.c_int32]
    L.mev_serve_stats.argtypes = [_vp, ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64), i32p]
    L.mev_configure.argtypes = [_vp, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32]
    L.mev_configure_traffic.argtypes = [_vp, ctypes.c_int32, ctypes.c_float]
    L.mev_set_reward.argtypes = [_vp, f32p]
    L.mev_car_update.argtypes = [f32p, ctypes.c_float, ctypes.c_float, ctypes.c_float]
    L.mev_car_check_collision.argtypes = [f32p, f32p, i32p]
    u64p = ctypes.POINTER(ctypes.c_uint64)
    L.mev_packed_layout.argtypes = [ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, u64p, u64p]
    L.mev_packed_layout2.argtypes = [ctypes.c_int32] * 5 + [u64p, u64p]
    L.mev_set_gather_format.argtypes = [_vp, ctypes.c_int32]
    L.mev_lidar_decode_table.argtypes = [_vp, f32p]
    L.mev_comm_unique_id.argtypes = [ctypes.c_char_p]
    L.mev_comm_init.argtypes = [_vp, ctypes.c_char_p, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32]
    L.mev_comm_destroy.argtypes = [_vp]
    L.mev_gather_result.argtypes = [_vp, ctypes.POINTER(_vp), u64p, i32p]
    L.mev_gather_wait.argtypes = [_vp, ctypes.c_int32]
    L.mev_unpack_gathered.argtypes = [_vp, _vp, ctypes.c_int32, _vp]
    L.mev_add_route.argtypes = [_vp, f32p, ctypes.c_int32, i32p]
    L.mev_add_route_n.argtypes = [_vp, f32p, ctypes.c_int32, ctypes.c_int32, i32p]
    L.mev_route_len.argtypes = [_vp, ctypes.c_int32, i32p]
    L.mev_output_dlpack.argtypes = [_vp, ctypes.c_int32, ctypes.POINTER(_vp)]
    L.mev_set_car_dims.argtypes = [_vp, f32p, f32p]
    L.mev_get_car_dims.argtypes = [_vp, f32p, f32p]
    L.mev_car_dims_active.argtypes = [_vp, i32p]
    L.mev_set_beam_angles.argtypes = [_vp, f32p]
    L.mev_get_beam_angles.argtypes = [_vp, f32p]
    L.mev_decode_errors.argtypes = [_vp, ctypes.POINTER(ctypes.c_int64)]
    _libs[variant] = L
    return L


class MevError(RuntimeError):
    pass


class IndexRangeError(MevError, IndexError):
    """MEV_E_RANGE: mirrors the reference's std::out_of_range -> IndexError."""


def _check(rc: int):
    if rc != 0:
        msg = load_library().mev_last_error().decode(errors="replace")  # thread-local in the product lib
        if rc == -4:
            raise IndexRangeError(msg)
        raise MevError(f"libmarlenv_hip error {rc}: {msg}")


_OUT_KEYS = ("obs", "reward", "done", "status", "terminated", "truncated", "agents_alive", "step")


class _DLTensor(ctypes.Structure):  # mev_dl_tensor (include/marlenv.h), DLPack's DLTensor
    _fields_ = [("data", ctypes.c_void_p), ("device_type", ctypes.c_int32), ("device_id", ctypes.c_int32),
                ("ndim", ctypes.c_int32), ("dtype_code", ctypes.c_uint8), ("dtype_bits", ctypes.c_uint8),
                ("dtype_lanes", ctypes.c_uint16), ("shape", ctypes.c_void_p), ("strides", ctypes.c_void_p),
                ("byte_offset", ctypes.c_uint64)]


_DL_DELETER = ctypes.CFUNCTYPE(None, ctypes.c_void_p)


class _DLManaged(ctypes.Structure):  # mev_dl_managed, DLPack's DLManagedTensor
    _fields_ = [("dl_tensor", _DLTensor), ("manager_ctx", ctypes.c_void_p), ("deleter", ctypes.c_void_p)]


_DLTENSOR = b"dltensor"


@ctypes.CFUNCTYPE(None, ctypes.c_void_p)
def _capsule_destructor(capsule):
    """PyCapsule destructor: a capsule still named "dltensor" was never consumed (a consumer renames
    it "used_dltensor" and takes over the deleter), so call the managed tensor's deleter."""
    api = ctypes.pythonapi
    api.PyCapsule_IsValid.restype = ctypes.c_int
    api.PyCapsule_IsValid.argtypes = [ctypes.c_void_p, ctypes.c_char_p]
    if not api.PyCapsule_IsValid(capsule, _DLTENSOR):
        return
    api.PyCapsule_GetPointer.restype = ctypes.c_void_p
    api.PyCapsule_GetPointer.argtypes = [ctypes.c_void_p, ctypes.c_char_p]
    ptr = api.PyCapsule_GetPointer(capsule, _DLTENSOR)
    if ptr:
        m = _DLManaged.from_address(ptr)
        if m.deleter:
            _DL_DELETER(m.deleter)(ptr)


def _ptr(a) -> Optional[int]:
    if a is None:
        return None
    if isinstance(a, np.ndarray):
        assert a.flags.c_contiguous, "arrays passed to libmarlenv_hip must be C-contiguous"
        return a.__array_interface__["data"][0]
    if hasattr(a, "data_ptr"):  # torch tensor (device pointer mode)
        return int(a.data_ptr())
    return int(a)


_torch_first_done = False


def _one_runtime():
    """One HIP runtime per process.  PyTorch-ROCm ships its own runtime
    (torch/lib/libamdhip64.so, SONAME libamdhip64.so.7, loaded by path) next to
    the /opt/rocm one this library links by that SONAME.  Imported first, torch's
    copy is already loaded when ours is, and the dynamic linker binds our
    NEEDED libamdhip64.so.7 / librccl.so.1 to it: a single runtime serves both
    (tests/test_capi_symbols.py::test_one_hip_runtime_with_torch).  Loaded the
    other way round, torch would bring its copy in beside ours -- two runtimes in
    one process -- so torch, when installed, is imported before the library.
    MEV_TORCH_FIRST=0 skips this for torch-free processes."""
    if os.environ.get("MEV_TORCH_FIRST", "1") == "0":
        return
    try:
        import torch  # noqa: F401
    except ImportError:
        pass


def _torch_runtime_first():
    """With torch present, let its runtime initialise the device before the
    library's first HIP call (the same single runtime, see _one_runtime).
    Set MEV_TORCH_FIRST=0 for torch-free processes."""
    global _torch_first_done
    if _torch_first_done:
        return
    _torch_first_done = True
    if os.environ.get("MEV_TORCH_FIRST", "1") == "0":
        return
    try:
        import torch
    except ImportError:
        return
    try:
        if torch.cuda.is_available():
            torch.cuda.init()
    except Exception:
        pass


def default_config() -> Dict:
    c = MevConfig()
    _check(load_library().mev_config_default(ctypes.byref(c)))
    d = {name: getattr(c, name) for name, _ in MevConfig._fields_}
    d["reward"] = list(c.reward)
    return d


class Handle:
    """One device-resident batch of E intersection envs (owner of a mev_handle)."""

    def __init__(self, **cfg):
        _torch_runtime_first()
        L = load_library()
        c = MevConfig()
        _check(L.mev_config_default(ctypes.byref(c)))
        for k, v in cfg.items():
            if k == "reward":
                for j, x in enumerate(v):
                    c.reward[j] = float(x)
            elif not hasattr(c, k):
                raise TypeError(f"unknown config key {k!r}")
            else:
                setattr(c, k, v)
        h = _vp()
        _check(L.mev_create(ctypes.byref(c), ctypes.byref(h)))
        self._args_cache = None
        self._h = h
        self._lib = L
        out = MevConfig()
        _check(L.mev_get_config(h, ctypes.byref(out)))
        self.config = {name: getattr(out, name) for name, _ in MevConfig._fields_}
        self.config["reward"] = list(out.reward)
        self.E = out.num_envs
        self.N = out.num_agents
        self.K = out.max_npcs
        self.R = out.lidar_rays
        self.D = out.obs_dim
        n = ctypes.c_int32()
        _check(L.mev_num_points(h, ctypes.byref(n)))
        self.num_points = n.value

    # -- lifetime ---------------------------------------------------------
    def close(self):
        if getattr(self, "_h", None):
            self._lib.mev_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def handle(self):
        return self._h

    def set_stream(self, stream_ptr: Optional[int]):
        """Order this handle's work on a hipStream_t (int handle; 0/None = legacy default stream)."""
        _check(self._lib.mev_set_stream(self._h, stream_ptr or None))

    def use_own_stream(self):
        _check(self._lib.mev_use_own_stream(self._h))

    def debug_stamps(self) -> np.ndarray:
        out = np.zeros((self.E, 8), np.uint64)
        _check(self._lib.mev_debug_stamps(self._h, out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64))))
        return out

    def sync(self):
        _check(self._lib.mev_sync(self._h))

    # -- routes -----------------------------------------------------------
    def route_id(self, start_point: int, end_point: int) -> int:
        r = ctypes.c_int32()
        _check(self._lib.mev_route_id(self._h, int(start_point), int(end_point), ctypes.byref(r)))
        return r.value

    def route_info(self, route: int):
        """(path [max(n, 160), 2] -- a shorter path padded with its last point --, intent, spawn)."""
        path = np.zeros((max(PATH_LEN, self.route_len(route)), 2), np.float32)
        intent = ctypes.c_int32()
        spawn = np.zeros(3, np.float32)
        _check(self._lib.mev_route_info(self._h, int(route), path.ctypes.data_as(ctypes.POINTER(ctypes.c_float)),
                                        ctypes.byref(intent), spawn.ctypes.data_as(ctypes.POINTER(ctypes.c_float))))
        return path, intent.value, spawn

    def route_len(self, route: int) -> int:
        """Points of a route's path (160, or a written path's own n; mev_route_len)."""
        n = ctypes.c_int32()
        _check(self._lib.mev_route_len(self._h, int(route), ctypes.byref(n)))
        return n.value

    def add_route(self, path, intent: int) -> int:
        """Append a route of the caller's own (path [n, 2] f32 with 2 <= n <= 4096, intent 0 straight /
        1 left / 2 right) to the route table (mev_add_route_n); returns its id."""
        a = np.ascontiguousarray(path, np.float32)
        if a.ndim != 2 or a.shape[1] != 2 or not 2 <= a.shape[0] <= MAX_PATH_LEN:
            raise ValueError(f"a route path has 2 .. {MAX_PATH_LEN} points (x, y), got shape {a.shape}")
        r = ctypes.c_int32()
        _check(self._lib.mev_add_route_n(self._h, a.ctypes.data_as(ctypes.POINTER(ctypes.c_float)), a.shape[0],
                                         int(intent), ctypes.byref(r)))
        return r.value

    def point_xy(self, point: int):
        xy = np.zeros(2, np.float32)
        _check(self._lib.mev_point_xy(self._h, int(point), xy.ctypes.data_as(ctypes.POINTER(ctypes.c_float))))
        return xy

    def set_ego_routes(self, routes):
        r = np.ascontiguousarray(np.broadcast_to(np.asarray(routes, np.int32), (self.E, self.N)), np.int32)
        _check(self._lib.mev_set_ego_routes(self._h, r.ctypes.data_as(ctypes.POINTER(ctypes.c_int32))))

    def set_traffic_routes(self, routes):
        r = np.ascontiguousarray(np.asarray(routes, np.int32).reshape(-1))
        _check(self._lib.mev_set_traffic_routes(self._h, r.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), len(r)))

    def default_traffic_routes(self):
        cnt = ctypes.c_int32()
        buf = np.zeros(1024, np.int32)
        _check(self._lib.mev_default_traffic_routes(self._h, buf.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)),
                                                    ctypes.byref(cnt)))
        return buf[: cnt.value].copy()

    # -- reset / step -----------------------------------------------------
    def reset(self, env_mask=None, obs=None, device: bool = False):
        mask = None if env_mask is None else (env_mask if device else np.ascontiguousarray(env_mask, np.uint8))
        _check(self._lib.mev_reset(self._h, _ptr(mask), _ptr(obs), MEV_DEVICE_PTRS if device else 0))
        return obs

    def alloc_outputs(self):
        E, N, D = self.E, self.N, self.D
        return dict(obs=np.zeros((E, N, D), np.float32), reward=np.zeros((E, N), np.float32),
                    done=np.zeros((E, N), np.uint8), status=np.zeros((E, N), np.uint8),
                    terminated=np.zeros(E, np.uint8), truncated=np.zeros(E, np.uint8),
                    agents_alive=np.zeros(E, np.int32), step=np.zeros(E, np.int32))

    def step(self, actions, dt: float = 1.0 / 60.0, out: Optional[dict] = None, spawn_route=None,
             auto_reset: bool = False, device: bool = False, gather: bool = False):
        """Host mode (default): numpy in/out, synchronous.  device=True: every
        array is a device tensor/pointer on this handle's device; asynchronous.
        gather=True (needs comm_init): the outputs are written packed and
        gathered to the root rank over RCCL (gather_result); `out` may then
        only hold agents_alive / step."""
        if not device:
            actions = np.ascontiguousarray(actions, np.float32)
            if actions.size != self.E * self.N * 2:
                raise ValueError(f"actions must have {self.E}x{self.N}x2 elements, got {actions.shape}")
            if spawn_route is not None:
                spawn_route = np.ascontiguousarray(np.broadcast_to(np.asarray(spawn_route, np.int32), (self.E,)))
            if out is None and not gather:
                out = self.alloc_outputs()
        out = out or {}
        # the output pointers of the args struct are reused while `out` holds the same
        # arrays (a step loop passes one dict): numpy pointer lookups cost ~1.6 us each
        c = self._args_cache
        if c is None or c[0] is not out or not all(map(operator.is_, c[1], map(out.get, _OUT_KEYS))):
            a = MevStepArgs()
            for k in _OUT_KEYS:
                setattr(a, k, _ptr(out.get(k)))
            c = self._args_cache = (out, tuple(map(out.get, _OUT_KEYS)), a, None)
        a = c[2]
        if actions is not c[3]:  # (a loop that refills one actions array skips the pointer lookup)
            a.actions = _ptr(actions)
            c = self._args_cache = (c[0], c[1], a, actions)
        a.dt = float(dt)
        a.spawn_route = _ptr(spawn_route)
        a.flags = ((MEV_DEVICE_PTRS if device else 0) | (MEV_AUTO_RESET if auto_reset else 0) |
                   (MEV_GATHER_TO_ROOT if gather else 0))
        _check(self._lib.mev_step(self._h, ctypes.byref(a)))
        return out

    # -- multi-GPU gather (mev_comm_*) -------------------------------------
    def comm_init(self, unique_id: bytes, world: int, rank: int, root: int = 0, slots: int = 0):
        """Join the RCCL communicator (collective over all ranks); slots = envs of the largest shard."""
        if len(unique_id) != MEV_COMM_ID_BYTES:
            raise ValueError("unique_id must be MEV_COMM_ID_BYTES bytes")
        _check(self._lib.mev_comm_init(self._h, bytes(unique_id), int(world), int(rank), int(root), int(slots)))
        self.comm = dict(world=int(world), rank=int(rank), root=int(root), slots=int(slots) or self.E)

    def set_gather_format(self, fmt: int):
        """MEV_GATHER_F32 (plain obs rows), MEV_GATHER_LIDAR_U8 (31-float heads + one LiDAR code per
        beam) or MEV_GATHER_STATE (post-step state + LiDAR codes, the heads rebuilt on the root);
        all lossless; before comm_init."""
        _check(self._lib.mev_set_gather_format(self._h, int(fmt)))
        self.gather_format = int(fmt)

    def lidar_decode_table(self) -> np.ndarray:
        """The compact gather format's 256-entry code -> LiDAR float table (mev_lidar_decode_table)."""
        t = np.zeros(256, np.float32)
        _check(self._lib.mev_lidar_decode_table(self._h, t.ctypes.data_as(ctypes.POINTER(ctypes.c_float))))
        return t

    def lidar_slots(self) -> int:
        return min(self.R, self.D - 31)

    def comm_destroy(self):
        _check(self._lib.mev_comm_destroy(self._h))
        self.comm = None

    def gather_result(self):
        """Root: (device pointer, bytes per rank, world) of the last gathered step's [world][bytes] buffer;
        the handle's stream is made to wait for that gather."""
        p, n, w = _vp(), ctypes.c_uint64(), ctypes.c_int32()
        _check(self._lib.mev_gather_result(self._h, ctypes.byref(p), ctypes.byref(n), ctypes.byref(w)))
        return p.value, n.value, w.value

    def gather_wait(self, timeout_ms: int = 0):
        """Host wait for every gather issued so far (timeout: the communicator is aborted, MevError)."""
        _check(self._lib.mev_gather_wait(self._h, int(timeout_ms)))

    def unpack_gathered(self, stacked_ptr: int, world: int, obs_ptr: int):
        """Root: the float observation rows [world][slots][N][D] (device, obs_ptr) of a gathered
        [world][bytes] device buffer in this handle's format (mev_unpack_gathered, on its stream)."""
        _check(self._lib.mev_unpack_gathered(self._h, _vp(int(stacked_ptr)), int(world), _vp(int(obs_ptr))))

    # -- zero-copy export (DLPack) ----------------------------------------
    def output_dlpack(self, which: str):
        """PyCapsule ("dltensor") viewing the handle's internal output buffer `which` (DLPACK_OUTPUTS);
        valid while the handle lives; torch.from_dlpack() consumes it.  A capsule dropped unconsumed
        frees its descriptor through the capsule destructor (DLPack's producer contract)."""
        m = _vp()
        _check(self._lib.mev_output_dlpack(self._h, DLPACK_OUTPUTS.index(which), ctypes.byref(m)))
        new = ctypes.pythonapi.PyCapsule_New
        new.restype = ctypes.py_object
        new.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_void_p]
        return new(m.value, _DLTENSOR, ctypes.cast(_capsule_destructor, ctypes.c_void_p))

    def output_tensors(self, names=("obs", "reward", "done", "status", "terminated", "truncated",
                                    "agents_alive", "step")):
        """The internal output buffers as torch tensors (zero copy, through DLPack)."""
        import torch.utils.dlpack as tdl
        return {k: tdl.from_dlpack(self.output_dlpack(k)) for k in names}

    def get_outputs(self, out: Optional[dict] = None, device: bool = False):
        """Outputs of the last step/reset/restore; device=True: `out` holds device buffers (D2D copies)."""
        out = out or self.alloc_outputs()
        _check(self._lib.mev_get_outputs(self._h, *[_ptr(out.get(k)) for k in (
            "obs", "reward", "done", "status", "terminated", "truncated", "agents_alive", "step")],
            MEV_DEVICE_PTRS if device else 0))
        return out

    def observations(self) -> np.ndarray:
        obs = np.zeros((self.E, self.N, self.D), np.float32)
        _check(self._lib.mev_get_outputs(self._h, _ptr(obs), None, None, None, None, None, None, None, 0))
        return obs

    # -- state ------------------------------------------------------------
    def _shape(self, per):
        return {"ego": (self.E, self.N), "npc": (self.E, self.K), "env": (self.E,)}[per]

    def get_state(self) -> Dict[str, np.ndarray]:
        st = MevState()
        arrays = {}
        for name, dt, per in STATE_FIELDS:
            a = np.zeros(self._shape(per), dt)
            arrays[name] = a
            setattr(st, name, _ptr(a) if a.size else None)
        _check(self._lib.mev_get_state(self._h, ctypes.byref(st)))
        return arrays

    def set_state(self, state: Dict[str, np.ndarray]):
        st = MevState()
        keep = []
        for name, dt, per in STATE_FIELDS:
            if name in state and state[name] is not None:
                a = np.ascontiguousarray(np.broadcast_to(np.asarray(state[name], dt), self._shape(per)))
                if a.size == 0:
                    continue
                keep.append(a)
                setattr(st, name, _ptr(a))
        _check(self._lib.mev_set_state(self._h, ctypes.byref(st)))

    def configure(self, use_team: bool, respawn: bool, max_steps: int):
        _check(self._lib.mev_configure(self._h, int(use_team), int(respawn), int(max_steps)))
        self.config.update(use_team_reward=int(use_team), respawn_enabled=int(respawn), max_steps=int(max_steps))

    def configure_traffic(self, enabled: bool, density: float):
        _check(self._lib.mev_configure_traffic(self._h, int(enabled), float(density)))
        self.config.update(traffic_flow=int(enabled), traffic_density=max(0.0, float(density)))

    def set_reward(self, reward):
        rc = np.ascontiguousarray(reward, np.float32)
        assert rc.size == 8
        _check(self._lib.mev_set_reward(self._h, rc.ctypes.data_as(ctypes.POINTER(ctypes.c_float))))
        self.config["reward"] = [float(x) for x in rc]

    def kernel_timing(self, every: int = 1):
        """Record per-kernel HIP events on every `every`-th step (0/False: off)."""
        _check(self._lib.mev_kernel_timing(self._h, int(every)))

    def kernel_times(self):
        """(k_cars ms summed, k_lidar ms summed, timed steps) since the previous call."""
        a, b, n = ctypes.c_double(), ctypes.c_double(), ctypes.c_int64()
        _check(self._lib.mev_kernel_times(self._h, ctypes.byref(a), ctypes.byref(b), ctypes.byref(n)))
        return a.value, b.value, n.value

    def set_step_kernel(self, kernel: int = 0):
        """0: automatic, 1: k_cars + k_lidar, 2: the fused k_step (scheduling only; results identical)."""
        _check(self._lib.mev_set_step_kernel(self._h, int(kernel)))

    def step_kernel(self) -> int:
        """The kernel path the next step uses: 1 (k_cars + k_lidar) or 2 (fused k_step)."""
        v = ctypes.c_int32()
        _check(self._lib.mev_get_step_kernel(self._h, ctypes.byref(v)))
        return v.value

    def set_step_pack(self, envs_per_wave: int = 0):
        """Envs per fused k_step wave: 0 automatic, 1, 2, 4 or 8 (scheduling only; results identical)."""
        _check(self._lib.mev_set_step_pack(self._h, int(envs_per_wave)))

    def step_pack(self) -> int:
        """Envs per wave the next step uses (1 on the two-kernel path)."""
        v = ctypes.c_int32()
        _check(self._lib.mev_get_step_pack(self._h, ctypes.byref(v)))
        return v.value

    def set_step_split(self, mode: int = 0):
        """Two waves per fused workgroup: 0 automatic, 1 off, 2 on, 3 early split (scheduling only;
        results identical)."""
        _check(self._lib.mev_set_step_split(self._h, int(mode)))

    def set_env_deal(self, on: bool = True):
        """The fused traffic kernel's NPC-aware env deal on / off (scheduling only; results identical)."""
        _check(self._lib.mev_set_env_deal(self._h, 1 if on else 0))

    def step_split(self) -> int:
        """Two waves per fused workgroup in the next step: 0 no, 1 split, 2 early split."""
        v = ctypes.c_int32()
        _check(self._lib.mev_get_step_split(self._h, ctypes.byref(v)))
        return int(v.value)

    def set_serve(self, mode: int = 1):
        """Host-mode steps through the persistent step server: 0 off, 1 automatic (results identical)."""
        _check(self._lib.mev_set_serve(self._h, int(mode)))

    def serve_stats(self) -> dict:
        """Steps the persistent server answered, its launches, and whether one is running."""
        st, la, ru = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_int32()
        _check(self._lib.mev_serve_stats(self._h, ctypes.byref(st), ctypes.byref(la), ctypes.byref(ru)))
        return {"steps": int(st.value), "launches": int(la.value), "running": bool(ru.value)}

    def set_reset_routes(self, routes):
        """Draw every agent's route from `routes` at each reset (empty: fixed routes)."""
        r = np.ascontiguousarray(np.asarray(routes, np.int32).reshape(-1))
        _check(self._lib.mev_set_reset_routes(self._h, r.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)) if r.size
                                              else None, int(r.size)))

    def snapshot_size(self) -> int:
        n = ctypes.c_uint64()
        _check(self._lib.mev_snapshot_size(self._h, ctypes.byref(n)))
        return n.value

    def snapshot(self, dst=None, device: bool = False):
        """Whole-state snapshot into `dst` (host uint8 array, or a device buffer/tensor with device=True)."""
        if dst is None:
            if device:
                raise ValueError("device snapshots need a caller-provided device buffer")
            dst = np.zeros(self.snapshot_size(), np.uint8)
        _check(self._lib.mev_snapshot(self._h, _ptr(dst), MEV_DEVICE_PTRS if device else 0))
        return dst

    def restore(self, src, env_mask=None, device: bool = False):
        mask = None if env_mask is None else (env_mask if device else np.ascontiguousarray(env_mask, np.uint8))
        _check(self._lib.mev_restore(self._h, _ptr(src), _ptr(mask), MEV_DEVICE_PTRS if device else 0))

    def npc_stats(self):
        """(dropped spawns, NPC turns run sequentially after a parallel-round disagreement), cumulative."""
        a, b = ctypes.c_int64(), ctypes.c_int64()
        _check(self._lib.mev_npc_stats(self._h, ctypes.byref(a), ctypes.byref(b)))
        return a.value, b.value

    def decode_errors(self) -> int:
        """Route ids of state-format gather messages this handle's route table lacks (cumulative)."""
        v = ctypes.c_int64()
        _check(self._lib.mev_decode_errors(self._h, ctypes.byref(v)))
        return v.value

    # -- per-car sizes and beam angles -------------------------------------
    def set_car_dims(self, ego=None, npc=None):
        """Car::length / Car::width of every ego ([E][N][2]) and NPC slot ([E][K][2]) in px (mev_set_car_dims);
        None leaves that array as it is."""
        f32p = ctypes.POINTER(ctypes.c_float)
        e = None if ego is None else np.ascontiguousarray(np.broadcast_to(np.asarray(ego, np.float32),
                                                                          (self.E, self.N, 2)))
        n = None if npc is None else np.ascontiguousarray(np.broadcast_to(np.asarray(npc, np.float32),
                                                                          (self.E, self.K, 2)))
        _check(self._lib.mev_set_car_dims(self._h, None if e is None else e.ctypes.data_as(f32p),
                                          None if n is None or n.size == 0 else n.ctypes.data_as(f32p)))

    def car_dims(self):
        """(ego [E][N][2], NPC [E][K][2]) (length, width) of every car."""
        f32p = ctypes.POINTER(ctypes.c_float)
        e = np.zeros((self.E, self.N, 2), np.float32)
        n = np.zeros((self.E, self.K, 2), np.float32)
        _check(self._lib.mev_get_car_dims(self._h, e.ctypes.data_as(f32p), n.ctypes.data_as(f32p) if n.size else None))
        return e, n

    def car_dims_active(self) -> bool:
        """Whether some car differs from the reference's 54 x 24 px (the steps then run the runtime-layout kernels)."""
        v = ctypes.c_int32()
        _check(self._lib.mev_car_dims_active(self._h, ctypes.byref(v)))
        return bool(v.value)

    def set_beam_angles(self, rel):
        """LiDAR beam offsets [R] in radians (Lidar::rel_angles; evenly spaced)."""
        a = np.ascontiguousarray(np.asarray(rel, np.float32).reshape(-1))
        if a.size != self.R:
            raise ValueError(f"{self.R} beam angles expected, got {a.size}")
        _check(self._lib.mev_set_beam_angles(self._h, a.ctypes.data_as(ctypes.POINTER(ctypes.c_float))))

    def beam_angles(self) -> np.ndarray:
        a = np.zeros(self.R, np.float32)
        _check(self._lib.mev_get_beam_angles(self._h, a.ctypes.data_as(ctypes.POINTER(ctypes.c_float))))
        return a

    def npc_overflow(self) -> int:
        v = ctypes.c_int64()
        _check(self._lib.mev_npc_overflow(self._h, ctypes.byref(v)))
        return v.value


def car_update(kin, throttle: float, steer: float, dt: float):
    """Host Car::update with the reference's exact arithmetic; kin = [x, y, v, heading, acc, steering]."""
    k = np.ascontiguousarray(kin, np.float32).copy()
    _check(load_library().mev_car_update(k.ctypes.data_as(ctypes.POINTER(ctypes.c_float)), float(throttle),
                                         float(steer), float(dt)))
    return k


def car_check_collision(box_a, box_b) -> bool:
    """Host Car::check_collision; box = [x, y, heading, length, width]."""
    a = np.ascontiguousarray(box_a, np.float32)
    b = np.ascontiguousarray(box_b, np.float32)
    r = ctypes.c_int32()
    _check(load_library().mev_car_check_collision(a.ctypes.data_as(ctypes.POINTER(ctypes.c_float)),
                                                  b.ctypes.data_as(ctypes.POINTER(ctypes.c_float)), ctypes.byref(r)))
    return bool(r.value)


def packed_layout(slots: int, agents: int, obs_dim: int, fmt: int = MEV_GATHER_F32, lidar_slots: int = 0):
    """(offsets by field, total bytes) of one rank's packed outputs (mev_packed_layout2; host-only, no GPU).
    fmt MEV_GATHER_LIDAR_U8: "obs" holds [slots][N][31] heads and "lidar" [slots][N][lidar_slots] codes;
    MEV_GATHER_STATE: "obs" is empty, "state" holds the post-step state arrays (22 B per agent)."""
    off = (ctypes.c_uint64 * len(PACKED_FIELDS))()
    n = ctypes.c_uint64()
    _check(load_library().mev_packed_layout2(int(slots), int(agents), int(obs_dim), int(lidar_slots), int(fmt), off,
                                             ctypes.byref(n)))
    return dict(zip(PACKED_FIELDS, (int(x) for x in off))), int(n.value)


def comm_unique_id() -> bytes:
    """ncclGetUniqueId (call on ONE rank, share the bytes with all)."""
    _torch_runtime_first()
    buf = ctypes.create_string_buffer(MEV_COMM_ID_BYTES)
    _check(load_library().mev_comm_unique_id(buf))
    return buf.raw


def device_count() -> int:
    _torch_runtime_first()
    n = ctypes.c_int32()
    load_library().mev_device_count(ctypes.byref(n))
    return n.value
