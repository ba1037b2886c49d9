"""MI355X-native batched intersection environment (drop-in for the reference's
env.py / cpp_backend.py / MARLEnv on the IntersectionEnv step path).

The simulator runs in libmarlenv_hip.so (hand-written gfx950 HIP kernels behind
a C ABI, include/marlenv.h).  Python only marshals buffers.
"""
from . import _capi  # noqa: F401
from ._capi import Handle, MevError, STATUS_NAMES, device_count, lib_available, load_library  # noqa: F401
from . import utils, cpp_backend, env, vec_env  # noqa: F401,E402
from .env import IntersectionEnv  # noqa: F401,E402
from .vec_env import VecIntersectionEnv  # noqa: F401,E402

__all__ = ["Handle", "MevError", "STATUS_NAMES", "device_count", "lib_available", "load_library",
           "IntersectionEnv", "VecIntersectionEnv", "cpp_backend", "env", "vec_env", "utils"]
