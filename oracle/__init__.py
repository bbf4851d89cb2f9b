"""ctypes wrapper of the CPU oracle (oracle/rt_oracle.c).  TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this package,
and only as the checker / CPU baseline — never as the product path.
Parity unpinned by reference artifacts (the reference has none); see rt_oracle.h.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
LIB_PATH = HERE / "build" / "librt_oracle.so"
# the same C source built for Zen with AVX-512 (make oracle: -march=znver3 + AVX-512; gcc 11
# has no znver4): the CPU baseline's build for the GPU box's AMD EPYC host cores (BASELINE.md:
# the CPU reference built for its own host); tests use the portable x86-64-v3 build
NATIVE_PATH = HERE / "build" / "librt_oracle_zen.so"

AOP_COMPUTE, AOP_POSTPROCESSING, AO_COMPUTE, P_COMPUTE, H_COMPUTE = 1, 2, 3, 4, 5


class rto_dims(C.Structure):
    _fields_ = [(n, C.c_int) for n in ("W", "H", "S", "AA", "F", "D", "gy0", "gh")]


_lib = None


def build():
    """Compile the oracle with gcc (Makefile target `oracle`)."""
    subprocess.run(["make", "-s", "oracle"], cwd=HERE.parent, check=True)


def select_native() -> bool:
    """Use the Zen AVX-512 build for this process when the host is an AVX-512 AMD CPU (before the
    first load; CPU-baseline timing only)."""
    global LIB_PATH
    if _lib is not None or not NATIVE_PATH.exists():
        return False
    try:
        info = Path("/proc/cpuinfo").read_text()
    except OSError:
        return False
    if "AuthenticAMD" in info and " avx512f" in info and " avx512vl" in info:
        LIB_PATH = NATIVE_PATH
        return True
    return False


def lib_name() -> str:
    return LIB_PATH.name


def load():
    global _lib
    if _lib is not None:
        return _lib
    if not LIB_PATH.exists():
        build()
    lib = C.CDLL(str(LIB_PATH))
    fp = C.POINTER(C.c_float)
    lib.rto_run_program.argtypes = [fp, C.POINTER(rto_dims), C.c_int, C.c_int, fp, C.c_int, C.c_int, C.c_int]
    lib.rto_run_program.restype = C.c_int
    lib.rto_run_program_window.argtypes = [fp, C.POINTER(rto_dims), C.c_int, C.c_int, fp, C.c_int, C.c_int, C.c_int,
                                           C.c_int, C.c_int]
    lib.rto_run_program_window.restype = C.c_int
    lib.rto_dispatch.argtypes = [fp, C.POINTER(rto_dims), C.c_int, C.c_int, fp, C.c_int]
    lib.rto_dispatch.restype = C.c_int
    lib.rto_sin.argtypes = [C.c_float]
    lib.rto_sin.restype = C.c_float
    if hasattr(lib, "rto_sin_check_range"):  # (absent from older builds, tools/sin_change_effect.py)
        lib.rto_sin_check_range.argtypes = [C.c_uint32, C.c_int64, fp, C.POINTER(C.c_uint32), C.c_int]
        lib.rto_sin_check_range.restype = C.c_int64
    lib.rto_set_contraction.argtypes = [C.c_int]
    lib.rto_set_contraction.restype = None
    lib.rto_get_contraction.argtypes = []
    lib.rto_get_contraction.restype = C.c_int
    lib.rto_random.argtypes = [C.c_float, C.c_float]
    lib.rto_random.restype = C.c_float
    lib.rto_sphere_eval.argtypes = [fp, fp, fp, C.c_float]
    lib.rto_sphere_eval.restype = C.c_float
    lib.rto_normalize3.argtypes = [fp, fp]
    lib.rto_normalize3.restype = None
    lib.rto_sphere_del.argtypes = [fp, fp, fp, C.c_float]
    lib.rto_sphere_del.restype = C.c_float
    lib.rto_primary_dir.argtypes = [fp, C.c_float, C.c_float, fp]
    lib.rto_primary_dir.restype = None
    _lib = lib
    return lib


def _fp(a):
    if a is None:
        return None
    assert a.dtype == np.float32 and a.flags["C_CONTIGUOUS"]
    return a.ctypes.data_as(C.POINTER(C.c_float))


def dims(W, H, S, AA, F=8, D=20, gy0=0, gh=None) -> rto_dims:
    return rto_dims(W, H, S, AA, F, D, gy0, H if gh is None else gh)


def run_program(ssbo: np.ndarray, d: rto_dims, program: int, frame: int, image=None, y0=None, y1=None,
                nthreads: int = 0, x0: int = 0, x1=None) -> None:
    """Rows [y0, y1) (default: the g-buffer band) x columns [x0, x1) (default: all)."""
    y0 = d.gy0 if y0 is None else y0
    y1 = d.gy0 + d.gh if y1 is None else y1
    x1 = d.W if x1 is None else x1
    rc = load().rto_run_program_window(_fp(ssbo), C.byref(d), program, frame, _fp(image), y0, y1, x0, x1, nthreads)
    if rc != 0:
        raise ValueError(f"rto_run_program rejected its arguments (program {program})")


def dispatch(ssbo: np.ndarray, d: rto_dims, mode: int, frame: int, image=None, nthreads: int = 0) -> int:
    rc = load().rto_dispatch(_fp(ssbo), C.byref(d), mode, frame, _fp(image), nthreads)
    if rc < 0:
        raise ValueError(f"rto_dispatch rejected its arguments (mode {mode})")
    return rc


# contraction variants of random()'s argument arithmetic (rto_set_contraction; measurement and
# test hook: 0 = the kernels' semantics)
C_UNFUSED_DOT, C_FUSED_SEEDS, C_FUSED_JITTER = 1, 2, 4


def set_contraction(flags: int) -> None:
    load().rto_set_contraction(int(flags))


def get_contraction() -> int:
    return int(load().rto_get_contraction())


# ---- primitives (vectorised over numpy inputs) --------------------------------------
def det_sin(x: np.ndarray) -> np.ndarray:
    f = load().rto_sin
    return np.array([f(float(v)) for v in np.asarray(x, np.float32).ravel()], np.float32)


def sin_check_range(start: int, got: np.ndarray, max_bad: int = 64):
    """(count, first bit patterns) where got[i] differs from rto_sin of bit pattern start + i."""
    got = np.ascontiguousarray(got, np.float32)
    bad = np.zeros(max_bad, np.uint32)
    n = load().rto_sin_check_range(start & 0xFFFFFFFF, got.size, _fp(got), bad.ctypes.data_as(C.POINTER(C.c_uint32)),
                                   max_bad)
    return int(n), bad[:min(n, max_bad)]


def random2(xy: np.ndarray) -> np.ndarray:
    f = load().rto_random
    xy = np.asarray(xy, np.float32).reshape(-1, 2)
    return np.array([f(float(a), float(b)) for a, b in xy], np.float32)


def _f32v(v) -> np.ndarray:
    return np.ascontiguousarray(np.asarray(v, np.float32).reshape(3))


def sphere_del(pos, dir_, center, r) -> np.float32:
    """The discriminant of sphere_eval_ray (p_compute.glsl:80-82) in the oracle's float semantics."""
    return np.float32(load().rto_sphere_del(_fp(_f32v(pos)), _fp(_f32v(dir_)), _fp(_f32v(center)), float(r)))


def sphere_eval(pos, dir_, center, r) -> np.float32:
    return np.float32(load().rto_sphere_eval(_fp(_f32v(pos)), _fp(_f32v(dir_)), _fp(_f32v(center)), float(r)))


def primary_dir(header: np.ndarray, hp, vp) -> np.ndarray:
    """normalize(llc + hp*horizontal + vp*vertical) (p_compute.glsl:233-235) of a header."""
    out = np.zeros(3, np.float32)
    load().rto_primary_dir(_fp(np.ascontiguousarray(header, np.float32)), float(np.float32(hp)), float(np.float32(vp)),
                           _fp(out))
    return out


def nthreads_default() -> int:
    return int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))
