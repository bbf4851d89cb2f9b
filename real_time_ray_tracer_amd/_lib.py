"""ctypes binding of librtrt.so (include/rt/abi.h).

The product path has no CPU fallback: if the HIP library is missing this module raises
on first use, with the build command in the message.
"""
from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

LIB_NAME = "librtrt.so"
LIB_PATH = Path(__file__).resolve().with_name(LIB_NAME)

# status codes / ids mirrored from include/rt/abi.h and include/rt/layout.h
RT_OK, RT_E_INVAL, RT_E_NOMEM, RT_E_HIP, RT_E_NODEV, RT_E_STATE = 0, -1, -2, -3, -4, -5
RT_PROG_AOP_COMPUTE = 1
RT_PROG_AOP_POSTPROCESSING = 2
RT_PROG_AO_COMPUTE = 3
RT_PROG_P_COMPUTE = 4
RT_PROG_H_COMPUTE = 5
RT_MODE_AO_PP, RT_MODE_AO, RT_MODE_PHONG, RT_MODE_PHONG_REFL = 1, 2, 3, 4
(RT_MATH_SIN, RT_MATH_RANDOM, RT_MATH_SQRT, RT_MATH_DIV, RT_MATH_NORMALIZE, RT_MATH_SPHERE, RT_MATH_SQRT_SWEEP,
 RT_MATH_RCP_SWEEP, RT_MATH_SQRT_TAIL_SWEEP, RT_MATH_SIN_RANGE, RT_MATH_SHADOW,
 RT_MATH_SIN_TABLE) = range(12)
RT_NUM_FRAMES = 8
RT_RECURSION_DEPTH = 20
RT_SHAPE_SPHERE, RT_SHAPE_RECTANGLE, RT_SHAPE_PLANE = 1, 3, 5
HDR_MODE, HDR_HORIZONTAL, HDR_VERTICAL, HDR_LLC, HDR_CAMERA, HDR_LIGHT, HDR_BACKGROUND = range(7)


class rt_config(C.Structure):
    _fields_ = [(n, C.c_int) for n in
                ("width", "height", "num_shapes", "spp", "num_frames", "max_depth", "row_begin", "row_end")]


_fp = C.POINTER(C.c_float)
_vp = C.c_void_p
_ctx = C.c_void_p
_grp = C.c_void_p

# name -> (restype, argtypes); every function declared in include/rt/abi.h
SIGNATURES = {
    "rt_create": (C.c_int, [C.c_int, C.POINTER(rt_config), C.POINTER(_ctx)]),
    "rt_destroy": (C.c_int, [_ctx]),
    "rt_set_stream": (C.c_int, [_ctx, _vp]),
    "rt_use_own_stream": (C.c_int, [_ctx]),
    "rt_get_stream": (_vp, [_ctx]),
    "rt_enable_pipelining": (C.c_int, [_ctx, C.c_int, _vp]),
    "rt_get_output_stream": (_vp, [_ctx]),
    "rt_image_stream": (_vp, [_ctx]),
    "rt_device_count": (C.c_int, []),
    "rt_synchronize": (C.c_int, [_ctx]),
    "rt_last_hip_error": (C.c_int, [_ctx]),
    "rt_upload_header": (C.c_int, [_ctx, _vp, C.c_size_t]),
    "rt_upload_rand_buffer": (C.c_int, [_ctx, _fp, C.c_size_t]),
    "rt_run_program": (C.c_int, [_ctx, C.c_int, C.c_int]),
    "rt_dispatch": (C.c_int, [_ctx, C.c_int, C.c_int]),
    "rt_compute_frames": (C.c_int, [_ctx, _fp, C.c_int, C.c_int, C.c_int, C.c_uint64, C.c_int]),
    "rt_set_frame_batch": (C.c_int, [_ctx, C.c_int]),
    "rt_set_tile_schedule": (C.c_int, [_ctx, C.c_int]),
    "rt_tile_schedule_state": (C.c_int, [_ctx]),
    "rt_tile_schedule_orders": (C.c_int, [_ctx]),
    "rt_download": (C.c_int, [_ctx, _fp, _fp, _fp, _fp]),
    "rt_download_rect": (C.c_int, [_ctx, C.c_int, C.c_int, C.c_int, C.c_int, _fp, _fp, _fp, _fp]),
    "rt_upload_gbuffer": (C.c_int, [_ctx, _fp, _fp, _fp]),
    "rt_image_device_ptr": (_vp, [_ctx]),
    "rt_bind_image": (C.c_int, [_ctx, _vp]),
    "rt_compute_one_shader": (C.c_int, [_ctx, _vp, C.c_int, C.c_int, _fp]),
    "rt_compute_two_shaders": (C.c_int, [_ctx, _vp, C.c_int, C.c_int, C.c_int, _fp]),
    "rt_group_create": (C.c_int, [C.c_int, C.POINTER(C.c_int), C.POINTER(rt_config), C.POINTER(C.c_int),
                                  C.POINTER(_grp)]),
    "rt_group_destroy": (C.c_int, [_grp]),
    "rt_group_size": (C.c_int, [_grp]),
    "rt_group_strip_copies": (C.c_int, [_grp, C.c_int]),
    "rt_group_force_copies": (C.c_int, [_grp, C.c_int]),
    "rt_group_bounds": (C.c_int, [_grp, C.POINTER(C.c_int)]),
    "rt_group_set_bounds": (C.c_int, [_grp, C.POINTER(C.c_int)]),
    "rt_group_strip": (_ctx, [_grp, C.c_int]),
    "rt_group_last_hip_error": (C.c_int, [_grp]),
    "rt_group_enable_pipelining": (C.c_int, [_grp, C.c_int]),
    "rt_group_bind_frame": (C.c_int, [_grp, _vp]),
    "rt_group_frame_device_ptr": (_vp, [_grp]),
    "rt_group_upload_header": (C.c_int, [_grp, _vp, C.c_size_t]),
    "rt_group_dispatch": (C.c_int, [_grp, C.c_int, C.c_int]),
    "rt_group_compute_frames": (C.c_int, [_grp, _fp, C.c_int, C.c_int, C.c_int, C.c_uint64, C.c_int]),
    "rt_group_synchronize": (C.c_int, [_grp]),
    "rt_group_download_image": (C.c_int, [_grp, _fp]),
    "rt_group_balance": (C.c_int, [_grp, _fp, C.c_int, C.c_int, C.POINTER(C.c_double)]),
    "rt_plan_strips": (C.c_int, [C.POINTER(C.c_double), C.c_int, C.c_int, C.POINTER(C.c_int)]),
    "rt_calibrate_row_cost": (C.c_int, [C.POINTER(C.c_double), C.c_int, C.POINTER(C.c_int), C.c_int,
                                        C.POINTER(C.c_double)]),
    "rt_plan_strips_gather": (C.c_int, [C.POINTER(C.c_double), C.c_int, C.c_int, C.c_int, C.c_double, C.c_double,
                                        C.POINTER(C.c_int), C.POINTER(C.c_int), C.POINTER(C.c_double)]),
    "rt_strip_gather_bound": (C.c_int, [C.POINTER(C.c_double), C.c_int, C.POINTER(C.c_int), C.c_int, C.c_int, C.c_int,
                                        C.c_double, C.c_double, C.POINTER(C.c_double)]),
    "rt_group_set_plan": (C.c_int, [_grp, C.POINTER(C.c_int), C.c_int]),
    "rt_group_root_strip": (C.c_int, [_grp]),
    "rt_group_strip_device": (C.c_int, [_grp, C.c_int]),
    "rt_group_set_link_model": (C.c_int, [_grp, C.c_double, C.c_double]),
    "rt_group_link_model": (C.c_int, [_grp, C.POINTER(C.c_double), C.POINTER(C.c_double)]),
    "rt_debug_fail_next_event_query": (C.c_int, [_ctx, C.c_int]),
    "rt_enable_timing": (C.c_int, [_ctx, C.c_int]),
    "rt_kernel_stats": (C.c_int, [_ctx, C.c_int, C.POINTER(C.c_int), C.POINTER(C.c_double)]),
    "rt_reset_stats": (C.c_int, [_ctx]),
    "rt_host_stats": (C.c_int, [_ctx, C.POINTER(C.c_double), C.POINTER(C.c_longlong)]),
    "rt_enable_counters": (C.c_int, [_ctx, C.c_int]),
    "rt_read_counters": (C.c_int, [_ctx, C.POINTER(C.c_uint64), C.c_int]),
    "rt_read_row_counters": (C.c_int, [_ctx, C.POINTER(C.c_uint64), C.c_int]),
    "rt_selftest_math": (C.c_int, [_ctx, C.c_int, _fp, _fp, C.c_size_t]),
    "rt_pack_sphere": (C.c_int, [_fp, C.c_int, C.c_int, _fp, C.c_float, _fp, C.c_float, C.c_int]),
    "rt_pack_plane": (C.c_int, [_fp, C.c_int, C.c_int, _fp, C.c_float, _fp, C.c_float, C.c_int]),
    "rt_pack_rectangle": (C.c_int, [_fp, C.c_int, C.c_int, _fp, _fp, _fp, _fp, C.c_float, C.c_int]),
    "rt_camera_basis": (C.c_int, [_fp, _fp, _fp, _fp, C.c_float]),
    "rt_set_mode": (C.c_int, [_fp, C.c_int, C.c_int]),
    "rt_fill_rand_buffer": (C.c_int, [_fp, C.c_int, C.c_int, C.c_uint64]),
    "rt_moving_light": (C.c_int, [_fp, C.c_int]),
    "rt_scenegen": (C.c_int, [_fp, C.c_int, C.c_int, C.c_int, C.c_uint64, C.c_float]),
    "rt_init_scene": (C.c_int, [_fp, C.c_int, C.c_int, C.c_int, C.c_float]),
    "rt_strerror": (C.c_char_p, [C.c_int]),
    "rt_version": (C.c_int, []),
}

_LIB = None


class RtError(RuntimeError):
    def __init__(self, status: int, what: str = "", hip: int = 0):
        msg = f"{what}: {strerror(status)} ({status})"
        if hip:
            msg += f", hipError {hip}"
        super().__init__(msg)
        self.status = status
        self.hip = hip


def load() -> C.CDLL:
    """Load librtrt.so (in-tree).  Raises if it has not been built — never falls back."""
    global _LIB
    if _LIB is not None:
        return _LIB
    path = Path(os.environ.get("RTRT_LIB", LIB_PATH))
    if not path.exists():
        raise RuntimeError(f"{path} not found: the HIP library is required (build it with `make lib` "
                           f"or __graft_entry__.build()); there is no CPU fallback")
    # One HIP runtime per process: PyTorch bundles its own libamdhip64 (same soname as
    # /opt/rocm's).  Whichever loads first serves both, and torch cannot start on the other
    # one, while torch streams handed to rt_set_stream must belong to the runtime the library
    # uses.  So when torch is installed it is imported (and its runtime loaded) first.
    if os.environ.get("RTRT_NO_TORCH_FIRST") != "1":
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
    lib = C.CDLL(str(path))
    # RTRT_LIB (A/B tools) may name an older build: entry points added since are left unbound
    tolerant = "RTRT_LIB" in os.environ
    for name, (res, args) in SIGNATURES.items():
        if tolerant and not hasattr(lib, name):
            continue
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _LIB = lib
    return lib


def strerror(status: int) -> str:
    try:
        return load().rt_strerror(status).decode()
    except Exception:  # library absent: still format the message
        return {0: "ok", -1: "invalid argument", -2: "out of memory", -3: "HIP runtime error",
                -4: "no HIP device", -5: "bad call order"}.get(status, "unknown status")


def fptr(a) -> "C._Pointer":
    """float* of a C-contiguous float32 numpy array (None -> NULL)."""
    if a is None:
        return None
    assert a.dtype.name == "float32" and a.flags["C_CONTIGUOUS"], "need C-contiguous float32"
    return a.ctypes.data_as(_fp)
