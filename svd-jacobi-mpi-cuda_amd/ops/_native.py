"""ctypes bindings of the two in-tree native libraries.

``libsvdj_cpu.so`` (host C++) is always required.  ``libsvdj_hip.so`` (gfx950
kernels) is required for any CUDA/HIP tensor: if it is missing or fails to
load on a GPU box the call raises -- there is no silent PyTorch fallback for
device tensors.  CPU tensors use the torch reference implementations in
``ops/reference.py`` (the oracle path used by CPU tests).
"""
from __future__ import annotations

import ctypes as C
import os
import threading
from pathlib import Path

_PKG = Path(__file__).resolve().parent.parent
_LIBDIR = _PKG / "lib"
_lock = threading.Lock()
_cpu = None
_hip = None
_dist = None

c_int = C.c_int
c_double = C.c_double
c_size_t = C.c_size_t
c_void_p = C.c_void_p
c_u32_p = C.POINTER(C.c_uint32)
c_i32_p = C.POINTER(C.c_int32)
c_f64_p = C.POINTER(C.c_double)


class NativeError(RuntimeError):
    pass


def _ensure_built(which: str) -> Path:
    from .. import _build

    path = _build.CPU_LIB if which == "cpu" else _build.HIP_LIB
    if os.environ.get("SVDJ_NO_AUTOBUILD") == "1":
        if not path.exists():
            raise NativeError(f"{path} missing and SVDJ_NO_AUTOBUILD=1")
        return path
    if which == "cpu":
        return _build.build_cpu()
    return _build.build_hip()


def _sig(lib, name, restype, argtypes):
    fn = getattr(lib, name)
    fn.restype = restype
    fn.argtypes = argtypes
    return fn


def cpu_lib():
    """Host library (schedules, oracle, RNG, verification)."""
    global _cpu
    if _cpu is not None:
        return _cpu
    with _lock:
        if _cpu is not None:
            return _cpu
        override = os.environ.get("SVDJ_CPU_LIB")  # e.g. the host-ASan build
        lib = C.CDLL(override if override else str(_ensure_built("cpu")))
        _sig(lib, "svdj_sameh_num_steps", c_int, [c_int])
        _sig(lib, "svdj_sameh_schedule", c_int, [c_int, c_i32_p])
        _sig(lib, "svdj_round_robin", c_int, [c_int, c_i32_p])
        _sig(lib, "svdj_bipartite", c_int, [c_int, c_i32_p])
        _sig(lib, "svdj_quad_round_robin", c_int, [c_int, c_i32_p])
        _sig(lib, "svdj_quad_bipartite", c_int, [c_int, c_i32_p, c_i32_p, c_i32_p])
        _sig(lib, "svdj_tournament", c_int, [c_int, c_i32_p, c_i32_p, c_i32_p, c_i32_p])
        for name, ptr in (("svdj_cpu_jacobi_f64", C.POINTER(C.c_double)),
                          ("svdj_cpu_jacobi_f32", C.POINTER(C.c_float))):
            _sig(lib, name, c_int, [c_int, c_int, c_int, c_int, ptr, c_int, ptr, ptr, c_int,
                                    c_int, c_int, c_double, c_int, c_f64_p, c_int])
        _sig(lib, "svdj_ref_triu_input", None, [c_int, c_int, c_f64_p, c_int, C.c_uint32])
        _sig(lib, "svdj_ref_dense_input", None, [c_int, c_int, c_f64_p, c_int, C.c_uint32])
        _sig(lib, "svdj_ref_uniform_stream", None, [C.c_uint32, c_int, c_f64_p])
        _sig(lib, "svdj_cpu_residual_f64", c_double,
             [c_int, c_int, c_int, c_f64_p, c_int, c_f64_p, c_int, c_f64_p, c_f64_p, c_int, c_int])
        _sig(lib, "svdj_cpu_orth_f64", c_double, [c_int, c_int, c_f64_p, c_int, c_int])
        _sig(lib, "svdj_sweep_converged", c_int,
             [c_double, c_double, c_double, c_double, c_double, c_int, c_int])
        _sig(lib, "svdj_cpu_version", C.c_char_p, [])
        _cpu = lib
        return lib


def hip_lib():
    """gfx950 kernel library.  Raises NativeError if unavailable."""
    global _hip
    if _hip is not None:
        return _hip
    with _lock:
        if _hip is not None:
            return _hip
        import torch  # noqa: F401  -- load torch's HIP runtime first (shared soname)

        override = os.environ.get("SVDJ_HIP_LIB")  # e.g. an A/B build of the kernels
        path = Path(override) if override else _ensure_built("hip")
        try:
            lib = C.CDLL(str(path))
        except OSError as e:  # pragma: no cover - GPU box only
            raise NativeError(f"cannot load {path}: {e}") from e
        _sig(lib, "svdj_hip_version", C.c_char_p, [])
        _sig(lib, "svdj_hip_last_error", C.c_char_p, [])
        _sig(lib, "svdj_scalar_step", c_int,
             [c_int, c_int, c_void_p, c_int, c_void_p, c_int, c_int, c_void_p, c_int, c_double,
              c_int, c_void_p, c_void_p])
        _sig(lib, "svdj_scalar_solve", c_int,
             [c_int, c_int, c_void_p, c_int, c_void_p, c_int, c_int, c_void_p, c_int, c_int,
              c_double, c_int, c_int, c_void_p, c_f64_p, c_void_p])
        _sig(lib, "svdj_block_workspace_bytes", c_size_t, [c_int, c_int, c_int, c_int, c_int])
        _sig(lib, "svdj_choose_inner_order", c_int, [c_int, c_int, c_int])
        _sig(lib, "svdj_block_steps", c_int,
             [c_int, c_int, c_int, c_void_p, c_int, c_void_p, c_int, c_int, c_void_p, c_void_p,
              c_int, c_int, c_i32_p, c_double, c_int, c_int, c_void_p, c_size_t, c_void_p, c_int,
              c_void_p])
        _sig(lib, "svdj_block_solve", c_int,
             [c_int, c_int, c_int, c_void_p, c_int, c_void_p, c_int, c_int, c_void_p, c_int,
              c_double, c_int, c_int, c_int, c_int, c_void_p, c_size_t, c_void_p, c_f64_p, c_int,
              c_int, c_void_p])
        _sig(lib, "svdj_reset_metric", c_int, [c_void_p, c_void_p])
        _sig(lib, "svdj_gram_cross", c_int,
             [c_int, c_int, c_void_p, c_int, c_int, c_void_p, c_int, c_int, c_void_p, c_void_p])
        _sig(lib, "svdj_gram_quad", c_int,
             [c_void_p, c_int, c_int, c_void_p, c_int, c_int, c_void_p, c_int, c_void_p])
        _sig(lib, "svdj_apply_q", c_int,
             [c_int, c_int, c_int, c_void_p, c_int, c_int, c_void_p, c_void_p])
        _sig(lib, "svdj_set_identity", c_int,
             [c_int, c_void_p, c_int, c_int, c_int, c_int, c_void_p])
        _sig(lib, "svdj_col_norms2", c_int, [c_int, c_void_p, c_int, c_int, c_int, c_void_p, c_void_p])
        _sig(lib, "svdj_finalize", c_int,
             [c_int, c_void_p, c_int, c_int, c_int, c_void_p, c_int, c_void_p])
        _sig(lib, "svdj_spin_ns", c_int, [c_double, c_void_p])
        _hip = lib
        return lib


class DistProblem(C.Structure):
    """svdj_dist_problem (csrc/include/svdj_dist.h), field for field."""
    _fields_ = [("rank", c_int), ("world", c_int), ("comm", c_void_p), ("dtype", c_int),
                ("W", c_int), ("m_pad", c_int), ("n_v", c_int), ("B", c_int),
                ("At", c_void_p), ("Vt", c_void_p), ("D", c_void_p), ("held", C.c_int32 * 2),
                ("tol", c_double), ("tol_mode", c_int), ("max_sweeps", c_int), ("mma", c_int),
                ("inner_order", c_int), ("exchange", c_int),
                ("stream_a", c_void_p),
                ("stream_b", c_void_p), ("stream_comm", c_void_p), ("timeout_s", c_double),
                ("comm_timing", c_int), ("fault_rank", c_int), ("fault_sweep", c_int),
                ("handle", c_void_p), ("hist", c_f64_p), ("sweeps", c_int),
                ("converged", c_int), ("comm_ms", c_double), ("exposed_comm_ms", c_double),
                ("exchanges", C.c_longlong), ("bytes_sent", C.c_longlong),
                ("progress", c_int), ("inner_order_used", c_int), ("exchange_used", c_int),
                ("stop_rule", c_int), ("quad", c_int), ("quad_used", c_int),
                ("merged_used", c_int), ("calib_direct_ms", c_double),
                ("calib_spread_ms", c_double)]


def dist_lib_path() -> Path:
    """Path of libsvdj_dist.so, (re)built unless SVDJ_NO_AUTOBUILD=1.  Always
    the shared object, never the ``bin/svdj_dist_main`` launcher."""
    from .. import _build

    override = os.environ.get("SVDJ_DIST_LIB")  # e.g. the host-ASan build
    if override:
        return Path(override)
    if os.environ.get("SVDJ_NO_AUTOBUILD") != "1":
        _build.build_dist()
    return _build.DIST_LIB


def dist_lib():
    """Native distributed solver (libsvdj_dist.so: RCCL tournament over the
    HIP block kernels, no Python in the sweep).  Loaded after torch, so its
    librccl.so.1 / libamdhip64 resolve to the runtime torch already loaded."""
    global _dist
    if _dist is not None:
        return _dist
    hip_lib()  # (takes _lock itself)
    with _lock:
        if _dist is not None:
            return _dist
        path = dist_lib_path()
        if not path.exists():
            raise NativeError(f"{path} missing")
        lib = C.CDLL(str(path))
        _sig(lib, "svdj_dist_comm_init", c_int,
             [c_int, c_int, C.c_char_p, c_double, C.POINTER(c_void_p)])
        _sig(lib, "svdj_dist_comm_destroy", c_int, [c_void_p])
        _sig(lib, "svdj_dist_id_file", c_int, [c_int, C.c_char_p, c_double, c_void_p, c_size_t])
        _sig(lib, "svdj_dist_geometry", c_int,
             [c_int, c_int, c_int, c_int, c_int, c_i32_p, c_i32_p, c_i32_p, c_i32_p])
        _sig(lib, "svdj_dist_choose_block", c_int, [c_int, c_int, c_int, c_int])
        _sig(lib, "svdj_dist_initial_held", c_int, [c_int, c_int, c_i32_p])
        _sig(lib, "svdj_dist_solve", c_int, [C.POINTER(DistProblem), c_void_p])
        _sig(lib, "svdj_dist_storage_cols", c_int, [c_int, c_int])
        _sig(lib, "svdj_dist_issue_rules", c_int,
             [c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_i32_p, c_i32_p])
        _sig(lib, "svdj_dist_merged_lists", c_int,
             [c_int, c_int, c_int, c_i32_p, c_int, c_i32_p, c_int, c_i32_p])
        _sig(lib, "svdj_dist_handle_create", c_int, [C.POINTER(DistProblem), C.POINTER(c_void_p)])
        _sig(lib, "svdj_dist_handle_destroy", c_int, [c_void_p])
        _sig(lib, "svdj_dist_last_error", C.c_char_p, [])
        _dist = lib
        return lib


def hip_check(rc: int, what: str) -> int:
    if rc < 0:
        msg = hip_lib().svdj_hip_last_error().decode(errors="replace")
        raise NativeError(f"{what} failed (rc={rc}): {msg}")
    return rc


def loaded_libraries() -> dict:
    """Which native libraries this process has loaded (for reports/tests)."""
    return {"cpu": _cpu is not None, "hip": _hip is not None,
            "cpu_path": str(_LIBDIR / "libsvdj_cpu.so"), "hip_path": str(_LIBDIR / "libsvdj_hip.so")}
