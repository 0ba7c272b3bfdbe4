"""Device ops: ctypes bindings of the gfx950 HIP kernels + CPU references."""
from . import kernels, reference  # noqa: F401
from ._native import NativeError, cpu_lib, hip_lib, loaded_libraries  # noqa: F401
