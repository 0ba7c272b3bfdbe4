"""Native build of the framework (no setuptools / no hipify / no JIT cache).

Two shared libraries are produced IN-TREE under ``lib/`` so they travel with
the repository snapshot to the GPU box:

* ``libsvdj_cpu.so`` -- host C++/OpenMP: schedules, CPU oracle, reference
  input generator, verification (g++).
* ``libsvdj_hip.so`` -- HIP kernels for gfx950 (CDNA4) + their host drivers
  (hipcc --offload-arch=gfx950).  Compiles on a CPU-only machine.

Reference parity: replaces the reference's CMake/nvcc build
(reference CMakeLists.txt:1-26, build/runSVDMPICUDAWithoutCMake.slurm:26).
"""
from __future__ import annotations

import concurrent.futures as cf
import os
import shutil
import subprocess
import sys
from pathlib import Path

PKG = Path(__file__).resolve().parent
CSRC = PKG / "csrc"
LIBDIR = PKG / "lib"
ARCH = os.environ.get("SVDJ_OFFLOAD_ARCH", "gfx950")

CPU_SOURCES = sorted((CSRC / "cpu").glob("*.cpp"))
HIP_SOURCES = sorted((CSRC / "hip").glob("*.hip"))
HEADERS = sorted((CSRC / "include").glob("*.h")) + sorted((CSRC / "hip").glob("*.hpp"))

CPU_LIB = LIBDIR / "libsvdj_cpu.so"
HIP_LIB = LIBDIR / "libsvdj_hip.so"


def _hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), shutil.which("hipcc"), "/opt/rocm/bin/hipcc"):
        if cand and Path(cand).exists():
            return cand
    raise FileNotFoundError("hipcc not found (set HIPCC)")


def _stale(target: Path, deps) -> bool:
    if not target.exists():
        return True
    t = target.stat().st_mtime
    return any(Path(d).stat().st_mtime > t for d in deps)


def _run(cmd, verbose):
    if verbose:
        print("[svdj-build]", " ".join(str(c) for c in cmd), flush=True)
    r = subprocess.run([str(c) for c in cmd], capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"build failed: {' '.join(map(str, cmd))}\n{r.stdout}\n{r.stderr}")
    return r


ASAN_CPU_LIB = LIBDIR / "asan" / "libsvdj_cpu.so"


def build_cpu(force: bool = False, verbose: bool = False, asan: bool = False) -> Path:
    """Host library.  ``asan``: AddressSanitizer + UBSan build into lib/asan/
    (host code only -- GPU sanitizers are not available); load it with
    SVDJ_CPU_LIB=<path> and the interpreter started under
    LD_PRELOAD=$(gcc -print-file-name=libasan.so) (tools/asan_cpu_tests.sh)."""
    target = ASAN_CPU_LIB if asan else CPU_LIB
    target.parent.mkdir(parents=True, exist_ok=True)
    if not force and not _stale(target, CPU_SOURCES + HEADERS + [Path(__file__)]):
        return target
    cxx = os.environ.get("CXX", "g++")
    tmp = target.with_suffix(".so.tmp")
    san = ["-fsanitize=address,undefined", "-fno-omit-frame-pointer", "-O1", "-g"] if asan else ["-O3"]
    cmd = [cxx, *san, "-std=c++17", "-fopenmp", "-fPIC", "-shared", "-Wall",
           f"-I{CSRC / 'include'}", *CPU_SOURCES, "-o", tmp]
    _run(cmd, verbose)
    os.replace(tmp, target)
    return target


def build_hip(force: bool = False, verbose: bool = False, jobs: int = 4) -> Path:
    LIBDIR.mkdir(exist_ok=True)
    if not force and not _stale(HIP_LIB, HIP_SOURCES + HEADERS + [Path(__file__)]):
        return HIP_LIB
    hipcc = _hipcc()
    objdir = LIBDIR / "obj"
    objdir.mkdir(exist_ok=True)
    flags = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-Wall",
             "-Wno-unused-result", f"-I{CSRC / 'include'}", f"-I{CSRC / 'hip'}"]
    objs = []

    def compile_one(src: Path):
        obj = objdir / (src.stem + ".o")
        if force or _stale(obj, [src] + HEADERS + [Path(__file__)]):
            _run([hipcc, *flags, "-c", src, "-o", obj], verbose)
        return obj

    with cf.ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
        objs = list(ex.map(compile_one, HIP_SOURCES))
    tmp = HIP_LIB.with_suffix(".so.tmp")
    _run([hipcc, f"--offload-arch={ARCH}", "-shared", "-fPIC", *objs, "-o", tmp], verbose)
    os.replace(tmp, HIP_LIB)
    return HIP_LIB


DRIVER_SRC = CSRC / "driver" / "svdj_main.cpp"
DRIVER_BIN = PKG / "bin" / "svdj_main"


def build_driver(force: bool = False, verbose: bool = False) -> Path:
    """Native single-GPU driver (reference `SVD_Jacobi_MPI_CUDA <n>` parity),
    linked against the in-tree libraries with an $ORIGIN rpath (its default
    block engine is libsvdj_dist's plan at world 1, no RCCL communicator)."""
    cpu, hip, dist = build_cpu(force, verbose), build_hip(force, verbose), build_dist(force, verbose)
    DRIVER_BIN.parent.mkdir(exist_ok=True)
    if not force and not _stale(DRIVER_BIN, [DRIVER_SRC, cpu, hip, dist] + HEADERS):
        return DRIVER_BIN
    tmp = DRIVER_BIN.with_suffix(".tmp")
    _run([_hipcc(), "-O2", "-std=c++17", f"--offload-arch={ARCH}", f"-I{CSRC / 'include'}",
          DRIVER_SRC, "-o", tmp, f"-L{LIBDIR}", "-lsvdj_dist", "-lsvdj_hip", "-lsvdj_cpu",
          "-lrccl", "-Wl,-rpath,$ORIGIN/../lib"], verbose)
    os.replace(tmp, DRIVER_BIN)
    return DRIVER_BIN


DIST_SRC = CSRC / "dist" / "svdj_dist.cpp"
DIST_LIB = LIBDIR / "libsvdj_dist.so"
DIST_DRIVER_SRC = CSRC / "driver" / "svdj_dist_main.cpp"
DIST_DRIVER_BIN = PKG / "bin" / "svdj_dist_main"


def build_dist(force: bool = False, verbose: bool = False) -> Path:
    """Native distributed solver (svdj_dist.h: RCCL tournament over the HIP
    block kernels) and its fork launcher ``bin/svdj_dist_main``.

    Returns the shared library ``DIST_LIB`` (the thing ``ctypes`` loads); the
    launcher is at ``DIST_DRIVER_BIN``."""
    cpu, hip = build_cpu(force, verbose), build_hip(force, verbose)
    deps = [DIST_SRC, cpu, hip, Path(__file__)] + HEADERS
    if force or _stale(DIST_LIB, deps):
        tmp = DIST_LIB.with_suffix(".so.tmp")
        _run([_hipcc(), "-O2", "-std=c++17", "-fPIC", "-shared", "-Wall", f"--offload-arch={ARCH}",
              f"-I{CSRC / 'include'}", DIST_SRC, "-o", tmp, f"-L{LIBDIR}", "-lsvdj_hip",
              "-lsvdj_cpu", "-lrccl", "-Wl,-rpath,$ORIGIN"], verbose)
        os.replace(tmp, DIST_LIB)
    DIST_DRIVER_BIN.parent.mkdir(exist_ok=True)
    if force or _stale(DIST_DRIVER_BIN, [DIST_DRIVER_SRC, DIST_LIB] + deps):
        tmp = DIST_DRIVER_BIN.with_suffix(".tmp")
        _run([_hipcc(), "-O2", "-std=c++17", "-Wall", f"--offload-arch={ARCH}",
              f"-I{CSRC / 'include'}", DIST_DRIVER_SRC, "-o", tmp, f"-L{LIBDIR}", "-lsvdj_dist",
              "-lsvdj_hip", "-lsvdj_cpu", "-lrccl", "-Wl,-rpath,$ORIGIN/../lib"], verbose)
        os.replace(tmp, DIST_DRIVER_BIN)
    return DIST_LIB


ASAN_DIST_LIB = LIBDIR / "asan" / "libsvdj_dist.so"


def build_dist_asan(force: bool = False, verbose: bool = False) -> Path:
    """AddressSanitizer + UBSan build of libsvdj_dist's host code (id-file
    handshake, plan and list builder, watchdog thread) into lib/asan/.  The
    file holds no device code, so g++ compiles it against the HIP runtime
    headers, with the same sanitizer runtime as ``build_cpu(asan=True)``;
    it links the ASan libsvdj_cpu next to it and the regular libsvdj_hip.
    Load with SVDJ_DIST_LIB=<path> (tools/asan_cpu_tests.sh)."""
    cpu, hip = build_cpu(force, verbose, asan=True), build_hip(force, verbose)
    target = ASAN_DIST_LIB
    if not force and not _stale(target, [DIST_SRC, cpu, hip, Path(__file__)] + HEADERS):
        return target
    rocm = os.environ.get("ROCM_PATH", "/opt/rocm")
    tmp = target.with_suffix(".so.tmp")
    _run([os.environ.get("CXX", "g++"), "-fsanitize=address,undefined", "-fno-omit-frame-pointer",
          "-O1", "-g", "-std=c++17", "-fPIC", "-shared", "-Wall", "-D__HIP_PLATFORM_AMD__",
          f"-I{rocm}/include", f"-I{CSRC / 'include'}", DIST_SRC, "-o", tmp,
          f"-L{target.parent}", "-lsvdj_cpu", f"-L{LIBDIR}", "-lsvdj_hip", f"-L{rocm}/lib",
          "-lamdhip64", "-lrccl", "-Wl,-rpath,$ORIGIN:$ORIGIN/.."], verbose)
    os.replace(tmp, target)
    return target


def build_all(force: bool = False, verbose: bool = False) -> dict:
    return {"cpu": str(build_cpu(force, verbose)), "hip": str(build_hip(force, verbose)),
            "driver": str(build_driver(force, verbose)),
            "dist": str(build_dist(force, verbose)), "dist_driver": str(DIST_DRIVER_BIN)}


if __name__ == "__main__":
    force = "--force" in sys.argv
    print(build_all(force=force, verbose=True))
