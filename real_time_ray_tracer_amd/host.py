"""Host-side mirror of the reference's compute interface, over the C ABI (librtrt.so).

Reference (src/main.cpp):
  class ssbo_data (49-85)            -> SSBO / header_size / ssbo_size
  loadShapeBuffer (395-469)          -> Header.pack_sphere / pack_plane / pack_rectangle
  fill_rand_buffer (535-539)         -> Header.fill_rand_buffer (seeded)
  moving_light (541-551)             -> Header.moving_light
  camera basis in render (772-779)   -> Header.camera_basis
  compute (553-578)                  -> Renderer.compute / Renderer.dispatch
  compute_one_shader (580-620)       -> Renderer.compute_one_shader
  compute_two_shaders (622-671)      -> Renderer.compute_two_shaders
Programs keep the reference's names: AOP_COMPUTE, AOP_POSTPROCESSING, AO_COMPUTE,
P_COMPUTE, H_COMPUTE.  Errors raise RtError (the reference exits on shader compile errors
and has no dispatch errors; here every bad argument is reported).
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

import numpy as np

from . import _lib
from ._lib import RtError, fptr

AOP_COMPUTE = _lib.RT_PROG_AOP_COMPUTE
AOP_POSTPROCESSING = _lib.RT_PROG_AOP_POSTPROCESSING
AO_COMPUTE = _lib.RT_PROG_AO_COMPUTE
P_COMPUTE = _lib.RT_PROG_P_COMPUTE
H_COMPUTE = _lib.RT_PROG_H_COMPUTE
PROGRAM_NAMES = {AOP_COMPUTE: "aop_compute", AOP_POSTPROCESSING: "aop_postprocessing",
                 AO_COMPUTE: "ao_compute", P_COMPUTE: "p_compute", H_COMPUTE: "h_compute"}

ASPECT_RATIO = 1.333333            # src/main.cpp:39
FULLSCREEN_ASPECT_RATIO = 1.777777  # src/main.cpp:40


def header_floats(S: int, AA: int) -> int:
    """floats in the SSBO prefix: 7 vec4 + S*5 vec4 + 2*AA vec4 (include/rt/layout.h)."""
    return 4 * (7 + 5 * S + 2 * AA)


def ssbo_floats(S: int, AA: int, W: int, H: int, F: int = 8) -> int:
    return header_floats(S, AA) + 3 * 4 * F * W * H


def aspect_for(width: int, height: int) -> float:
    return ASPECT_RATIO if width * 3 == height * 4 else FULLSCREEN_ASPECT_RATIO


def _check(rc: int, what: str, ctx=None) -> int:
    if rc < 0:
        hip = _lib.load().rt_last_hip_error(ctx) if ctx else 0
        raise RtError(rc, what, hip)
    return rc


def _f3(v):
    return (C.c_float * 3)(*[float(x) for x in v])


class Header:
    """The SSBO prefix (header + shapes + rand_buffer) as a float32 array; host-only helpers."""

    def __init__(self, num_shapes: int, spp: int, data: np.ndarray | None = None):
        self.S, self.AA = int(num_shapes), int(spp)
        n = header_floats(self.S, self.AA)
        self.data = np.zeros(n, np.float32) if data is None else np.ascontiguousarray(data, np.float32)
        assert self.data.size == n
        self._lib = _lib.load()

    # views
    def vec4(self, i: int) -> np.ndarray:
        return self.data[4 * i:4 * i + 4]

    @property
    def shapes(self) -> np.ndarray:
        return self.data[28:28 + 20 * self.S].reshape(self.S, 5, 4)

    @property
    def rand_buffer(self) -> np.ndarray:
        o = 28 + 20 * self.S
        return self.data[o:o + 8 * self.AA].reshape(2 * self.AA, 4)

    @property
    def num_objects(self) -> int:
        return int(self.data[2])

    def _p(self):
        return fptr(self.data)

    # loadShapeBuffer entries
    def pack_sphere(self, i, center, radius, color, reflectivity=1.0, emissive=False):
        _check(self._lib.rt_pack_sphere(self._p(), self.S, i, _f3(center), radius, _f3(color),
                                        reflectivity, int(emissive)), "rt_pack_sphere")

    def pack_plane(self, i, normal, dist, color, reflectivity=1.0, emissive=False):
        _check(self._lib.rt_pack_plane(self._p(), self.S, i, _f3(normal), dist, _f3(color),
                                       reflectivity, int(emissive)), "rt_pack_plane")

    def pack_rectangle(self, i, llc, right, up, color, reflectivity=1.0, emissive=False):
        _check(self._lib.rt_pack_rectangle(self._p(), self.S, i, _f3(llc), _f3(right), _f3(up), _f3(color),
                                           reflectivity, int(emissive)), "rt_pack_rectangle")

    def camera_basis(self, location, up, look_towards, aspect):
        _check(self._lib.rt_camera_basis(self._p(), _f3(location), _f3(up), _f3(look_towards), aspect),
               "rt_camera_basis")

    def set_mode(self, frame: int, num_objects: int):
        _check(self._lib.rt_set_mode(self._p(), frame, num_objects), "rt_set_mode")

    def fill_rand_buffer(self, seed: int):
        _check(self._lib.rt_fill_rand_buffer(self._p(), self.S, self.AA, seed), "rt_fill_rand_buffer")

    def moving_light(self, light_movement: bool = False):
        _check(self._lib.rt_moving_light(self._p(), int(light_movement)), "rt_moving_light")

    @classmethod
    def synthetic(cls, num_objects: int, spp: int, seed: int, aspect: float, num_shapes: int | None = None):
        h = cls(num_shapes if num_shapes is not None else num_objects, spp)
        _check(h._lib.rt_scenegen(h._p(), h.S, num_objects, spp, seed, aspect), "rt_scenegen")
        return h

    @classmethod
    def builtin(cls, which: int, spp: int, aspect: float = ASPECT_RATIO, num_shapes: int = 10):
        h = cls(num_shapes, spp)
        _check(h._lib.rt_init_scene(h._p(), h.S, spp, which, aspect), "rt_init_scene")
        return h

    def copy(self) -> "Header":
        return Header(self.S, self.AA, self.data.copy())


class SSBO:
    """A whole ssbo_data-layout host buffer (src/main.cpp:49-85) for the host-buffer path."""

    def __init__(self, header: Header, width: int, height: int, num_frames: int = 8):
        self.S, self.AA, self.W, self.H, self.F = header.S, header.AA, width, height, num_frames
        self.data = np.zeros(ssbo_floats(self.S, self.AA, width, height, num_frames), np.float32)
        self.data[:header.data.size] = header.data
        self.hn = header.data.size

    @property
    def header(self) -> Header:
        return Header(self.S, self.AA, self.data[:self.hn].copy())

    def set_header(self, header: Header):
        self.data[:self.hn] = header.data

    def _g(self, k):
        n = self.F * self.W * self.H * 4
        o = self.hn + k * n
        return self.data[o:o + n].reshape(self.F, self.W, self.H, 4)

    pixels = property(lambda self: self._g(0))
    normals = property(lambda self: self._g(1))
    depth = property(lambda self: self._g(2))


@dataclass
class GBuffer:
    pixels: np.ndarray   # [F][W][R][4]  reference layout
    normals: np.ndarray
    depth: np.ndarray
    image: np.ndarray    # [R][W][4]


class Renderer:
    """One rt_ctx: a device, a frame (or a row strip of it), a resident g-buffer ring."""

    def __init__(self, width: int, height: int, num_shapes: int, spp: int, num_frames: int = 8,
                 max_depth: int = 20, device: int = 0, rows: tuple[int, int] | None = None):
        self._lib = _lib.load()
        r0, r1 = rows if rows is not None else (0, height)
        self.cfg = _lib.rt_config(width, height, num_shapes, spp, num_frames, max_depth, r0, r1)
        self.W, self.H, self.S, self.AA, self.F, self.D = width, height, num_shapes, spp, num_frames, max_depth
        self.row_begin, self.row_end = r0, r1
        self.R = r1 - r0
        ctx = C.c_void_p()
        _check(self._lib.rt_create(device, C.byref(self.cfg), C.byref(ctx)), "rt_create")
        self.ctx = ctx

    # lifetime
    def close(self):
        if self.ctx:
            self._lib.rt_destroy(self.ctx)
            self.ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def _c(self, rc, what):
        return _check(rc, what, self.ctx)

    # streams
    def set_stream(self, stream):
        """Order the context's work on `stream`: a torch.cuda.Stream or an int hipStream_t
        (0 = the NULL stream, which is torch's default stream); None = the context's own stream."""
        if stream is None:
            self._c(self._lib.rt_use_own_stream(self.ctx), "rt_use_own_stream")
            return
        ptr = int(getattr(stream, "cuda_stream", stream))
        self._c(self._lib.rt_set_stream(self.ctx, C.c_void_p(ptr)), "rt_set_stream")

    def enable_pipelining(self, on: bool = True, output_stream=None):
        """Pipelined mode 1: frame k's post-process runs on `output_stream` (a torch.cuda.Stream
        or an int hipStream_t; None = a stream of the context's own) while frame k+1's AO pass
        runs on the main stream.  Bit-identical results; consumers of the image order their
        work on the output stream (or synchronize)."""
        ptr = None if output_stream is None else int(getattr(output_stream, "cuda_stream", output_stream))
        self._c(self._lib.rt_enable_pipelining(self.ctx, int(bool(on)), C.c_void_p(ptr) if ptr is not None else None),
                "rt_enable_pipelining")

    def synchronize(self):
        self._c(self._lib.rt_synchronize(self.ctx), "rt_synchronize")

    # device-resident path
    def upload_header(self, header: Header):
        assert header.S == self.S and header.AA == self.AA
        self._c(self._lib.rt_upload_header(self.ctx, header.data.ctypes.data_as(C.c_void_p),
                                           header.data.nbytes), "rt_upload_header")

    def upload_rand_buffer(self, rb: np.ndarray):
        rb = np.ascontiguousarray(rb, np.float32).reshape(-1)
        self._c(self._lib.rt_upload_rand_buffer(self.ctx, fptr(rb), rb.size // 4), "rt_upload_rand_buffer")

    def run_program(self, program: int, frame: int):
        self._c(self._lib.rt_run_program(self.ctx, program, frame), f"rt_run_program({program})")

    def dispatch(self, mode: int, frame: int) -> int:
        return self._c(self._lib.rt_dispatch(self.ctx, mode, frame), f"rt_dispatch(mode {mode})")

    def compute_frames(self, header: Header, mode: int, frame: int, n: int, rand_seed: int = 7000,
                       light_movement: bool = False) -> int:
        """n compute() rounds with the per-frame host updates done in C++ (rt_compute_frames):
        fill_rand_buffer(rand_seed + k) or moving_light, set_mode, upload, dispatch.  `header`
        is updated in place as the frame loop leaves it.  Returns the next frame slot."""
        return self._c(self._lib.rt_compute_frames(self.ctx, header._p(), mode, frame, n, rand_seed,
                                                   int(bool(light_movement))), "rt_compute_frames")

    def set_frame_batch(self, max_frames: int):
        """compute_frames' most frames per launch (modes 2-4); 1 (the default) = one launch and one
        image write per frame, the reference's dispatch shape; > 1 = multi-frame launches, the image
        by each launch's last frame (rt_set_frame_batch)."""
        self._c(self._lib.rt_set_frame_batch(self.ctx, int(max_frames)), "rt_set_frame_batch")

    def set_tile_schedule(self, on: bool):
        """Mode 4's longest-first tile order (rt_set_tile_schedule; on by default)."""
        self._c(self._lib.rt_set_tile_schedule(self.ctx, int(bool(on))), "rt_set_tile_schedule")

    def tile_schedule_state(self) -> int:
        """0 off, 1 on (row order so far), 2 a longest-first order in use (rt_tile_schedule_state)."""
        return self._c(self._lib.rt_tile_schedule_state(self.ctx), "rt_tile_schedule_state")

    def tile_schedule_orders(self) -> int:
        """Orders taken up so far (rt_tile_schedule_orders)."""
        return self._c(self._lib.rt_tile_schedule_orders(self.ctx), "rt_tile_schedule_orders")

    def download(self, pixels=True, normals=True, depth=True, image=True) -> GBuffer:
        shp = (self.F, self.W, self.R, 4)
        p = np.empty(shp, np.float32) if pixels else None
        n = np.empty(shp, np.float32) if normals else None
        d = np.empty(shp, np.float32) if depth else None
        im = np.empty((self.R, self.W, 4), np.float32) if image else None
        self._c(self._lib.rt_download(self.ctx, fptr(p), fptr(n), fptr(d), fptr(im)), "rt_download")
        return GBuffer(p, n, d, im)

    def download_rect(self, x0: int, x1: int, y0: int, y1: int, pixels=True, normals=True, depth=True,
                      image=True) -> GBuffer:
        """The window [x0, x1) x frame rows [y0, y1): g-buffer [F][w][h][4], image [h][w][4]."""
        shp = (self.F, x1 - x0, y1 - y0, 4)
        p = np.empty(shp, np.float32) if pixels else None
        n = np.empty(shp, np.float32) if normals else None
        d = np.empty(shp, np.float32) if depth else None
        im = np.empty((y1 - y0, x1 - x0, 4), np.float32) if image else None
        self._c(self._lib.rt_download_rect(self.ctx, x0, x1, y0, y1, fptr(p), fptr(n), fptr(d), fptr(im)),
                "rt_download_rect")
        return GBuffer(p, n, d, im)

    def image(self) -> np.ndarray:
        return self.download(False, False, False, True).image

    def upload_gbuffer(self, pixels=None, normals=None, depth=None):
        conv = [None if a is None else np.ascontiguousarray(a, np.float32) for a in (pixels, normals, depth)]
        self._c(self._lib.rt_upload_gbuffer(self.ctx, *[fptr(a) for a in conv]), "rt_upload_gbuffer")

    def image_device_ptr(self) -> int:
        return self._lib.rt_image_device_ptr(self.ctx) or 0

    def bind_image(self, device_ptr: int | None):
        self._c(self._lib.rt_bind_image(self.ctx, C.c_void_p(device_ptr) if device_ptr else None),
                "rt_bind_image")

    # host-buffer parity path (the reference's call shape)
    def compute_one_shader(self, ssbo: SSBO, frame_num: int, program: int, image: np.ndarray | None = None) -> int:
        return self._c(self._lib.rt_compute_one_shader(self.ctx, ssbo.data.ctypes.data_as(C.c_void_p), frame_num,
                                                       program, fptr(image)), "rt_compute_one_shader")

    def compute_two_shaders(self, ssbo: SSBO, frame_num: int, program1: int, program2: int,
                            image: np.ndarray | None = None) -> int:
        return self._c(self._lib.rt_compute_two_shaders(self.ctx, ssbo.data.ctypes.data_as(C.c_void_p), frame_num,
                                                        program1, program2, fptr(image)),
                       "rt_compute_two_shaders")

    # instrumentation
    def enable_timing(self, on: bool = True):
        self._c(self._lib.rt_enable_timing(self.ctx, int(on)), "rt_enable_timing")

    def kernel_stats(self, program: int) -> tuple[int, float]:
        n, ms = C.c_int(), C.c_double()
        self._c(self._lib.rt_kernel_stats(self.ctx, program, C.byref(n), C.byref(ms)), "rt_kernel_stats")
        return n.value, ms.value

    def reset_stats(self):
        self._c(self._lib.rt_reset_stats(self.ctx), "rt_reset_stats")

    def debug_fail_next_event_query(self, hip_error: int):
        """Test hook (rt_debug_fail_next_event_query): the next staging-buffer query reports hip_error."""
        self._c(self._lib.rt_debug_fail_next_event_query(self.ctx, int(hip_error)), "rt_debug_fail_next_event_query")

    def host_stats(self) -> tuple[float, int]:
        """(ms, count) of host waits for a free staging buffer since reset_stats (back-pressure)."""
        ms, n = C.c_double(), C.c_longlong()
        self._c(self._lib.rt_host_stats(self.ctx, C.byref(ms), C.byref(n)), "rt_host_stats")
        return ms.value, n.value

    def enable_counters(self, totals: bool = True, rows: bool = False):
        self._c(self._lib.rt_enable_counters(self.ctx, int(totals) | (2 if rows else 0)), "rt_enable_counters")

    def read_counters(self, reset: bool = True) -> dict:
        out = (C.c_uint64 * 8)()
        self._c(self._lib.rt_read_counters(self.ctx, out, int(reset)), "rt_read_counters")
        return {"samples": out[0], "segments": out[1], "shadow_rays": out[2], "tests": out[3],
                "executed_lane_tests": out[4], "filtered_pixels": out[5], "history_read": out[6],
                "history_accepted": out[7]}

    def read_row_counters(self, reset: bool = True) -> np.ndarray:
        out = np.zeros(self.R, np.uint64)
        self._c(self._lib.rt_read_row_counters(self.ctx, out.ctypes.data_as(C.POINTER(C.c_uint64)), int(reset)),
                "rt_read_row_counters")
        return out

    def selftest_math(self, fn: int, inputs: np.ndarray, n: int) -> np.ndarray:
        out_w = {_lib.RT_MATH_NORMALIZE: 3, _lib.RT_MATH_SHADOW: 5, _lib.RT_MATH_SIN_TABLE: 2}.get(fn, 1)
        in_w = {_lib.RT_MATH_RANDOM: 2, _lib.RT_MATH_DIV: 2, _lib.RT_MATH_NORMALIZE: 3, _lib.RT_MATH_SPHERE: 10,
                _lib.RT_MATH_SHADOW: 4}.get(fn, 1)
        inp = np.ascontiguousarray(inputs, np.float32).reshape(-1)
        sweep = fn in (_lib.RT_MATH_SQRT_SWEEP, _lib.RT_MATH_RCP_SWEEP, _lib.RT_MATH_SQRT_TAIL_SWEEP,
                       _lib.RT_MATH_SIN_RANGE, _lib.RT_MATH_SIN_TABLE)
        if inp.size < (1 if sweep else n * in_w):
            raise ValueError(f"selftest_math: {inp.size} input floats for n = {n} (need {1 if sweep else n * in_w})")
        out = np.empty(n * out_w, np.float32)
        self._c(self._lib.rt_selftest_math(self.ctx, fn, fptr(inp), fptr(out), n), "rt_selftest_math")
        return out


class StripGroup:
    """Row strips of one frame on several devices in one process (rt_group_*, the C-ABI
    counterpart of dist.py's one-process-per-GPU path): strip i = rows [bounds[i], bounds[i+1])
    on devices[i]; the image strips are assembled into one [H][W] frame on devices[0]."""

    def __init__(self, width: int, height: int, num_shapes: int, spp: int, devices, bounds=None,
                 num_frames: int = 8, max_depth: int = 20):
        self._lib = _lib.load()
        self.W, self.H, self.S, self.AA, self.F = width, height, num_shapes, spp, num_frames
        devs = [int(d) for d in devices]
        self.n = len(devs)
        cfg = _lib.rt_config(width, height, num_shapes, spp, num_frames, max_depth, 0, 0)
        dv = (C.c_int * self.n)(*devs)
        bd = None if bounds is None else (C.c_int * (self.n + 1))(*[int(b) for b in bounds])
        g = C.c_void_p()
        _check(self._lib.rt_group_create(self.n, dv, C.byref(cfg), bd, C.byref(g)), "rt_group_create")
        self.g = g

    def close(self):
        if self.g:
            self._lib.rt_group_destroy(self.g)
            self.g = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def _c(self, rc, what):
        if rc < 0:
            raise RtError(rc, what, self._lib.rt_group_last_hip_error(self.g) if self.g else 0)
        return rc

    @property
    def bounds(self) -> list[int]:
        b = (C.c_int * (self.n + 1))()
        self._c(self._lib.rt_group_bounds(self.g, b), "rt_group_bounds")
        return list(b)

    def set_bounds(self, bounds):
        self._c(self._lib.rt_group_set_bounds(self.g, (C.c_int * (self.n + 1))(*[int(b) for b in bounds])),
                "rt_group_set_bounds")

    def strip_copies(self, i: int) -> bool:
        """Whether strip i's image is copied into the frame (another device, or forced)."""
        return bool(self._c(self._lib.rt_group_strip_copies(self.g, i), "rt_group_strip_copies"))

    def set_plan(self, bounds, root_strip: int):
        """rt_group_set_plan: new bounds and root strip (the strip rendered on devices[0])."""
        b = (C.c_int * (self.n + 1))(*[int(x) for x in bounds])
        self._c(self._lib.rt_group_set_plan(self.g, b, int(root_strip)), "rt_group_set_plan")

    def root_strip(self) -> int:
        return self._c(self._lib.rt_group_root_strip(self.g), "rt_group_root_strip")

    def strip_device(self, i: int) -> int:
        return self._c(self._lib.rt_group_strip_device(self.g, i), "rt_group_strip_device")

    def set_link_model(self, link_gbps: float, ingest_gbps: float):
        self._c(self._lib.rt_group_set_link_model(self.g, float(link_gbps), float(ingest_gbps)),
                "rt_group_set_link_model")

    def link_model(self) -> tuple[float, float]:
        a, b = C.c_double(), C.c_double()
        self._c(self._lib.rt_group_link_model(self.g, C.byref(a), C.byref(b)), "rt_group_link_model")
        return a.value, b.value

    def force_copies(self, on: bool = True):
        """Test hook: every strip but strip 0 renders into its own image and copies it into the
        frame, as strips on other devices do (the copy path, exercised on one GPU)."""
        self._c(self._lib.rt_group_force_copies(self.g, int(bool(on))), "rt_group_force_copies")

    def strip_ctx(self, i: int):
        return self._lib.rt_group_strip(self.g, i)

    def strip_kernel_stats(self, i: int, program: int) -> tuple[int, float]:
        n, ms = C.c_int(), C.c_double()
        _check(self._lib.rt_kernel_stats(self.strip_ctx(i), program, C.byref(n), C.byref(ms)), "rt_kernel_stats")
        return n.value, ms.value

    def enable_pipelining(self, on: bool = True):
        self._c(self._lib.rt_group_enable_pipelining(self.g, int(bool(on))), "rt_group_enable_pipelining")

    def bind_frame(self, device_ptr: int | None):
        self._c(self._lib.rt_group_bind_frame(self.g, C.c_void_p(device_ptr) if device_ptr else None),
                "rt_group_bind_frame")

    def frame_device_ptr(self) -> int:
        return self._lib.rt_group_frame_device_ptr(self.g) or 0

    def upload_header(self, header: Header):
        assert header.S == self.S and header.AA == self.AA
        self._c(self._lib.rt_group_upload_header(self.g, header.data.ctypes.data_as(C.c_void_p), header.data.nbytes),
                "rt_group_upload_header")

    def dispatch(self, mode: int, frame: int) -> int:
        return self._c(self._lib.rt_group_dispatch(self.g, mode, frame), f"rt_group_dispatch(mode {mode})")

    def compute_frames(self, header: Header, mode: int, frame: int, n: int, rand_seed: int = 7000,
                       light_movement: bool = False) -> int:
        return self._c(self._lib.rt_group_compute_frames(self.g, header._p(), mode, frame, n, rand_seed,
                                                         int(bool(light_movement))), "rt_group_compute_frames")

    def synchronize(self):
        self._c(self._lib.rt_group_synchronize(self.g), "rt_group_synchronize")

    def image(self) -> np.ndarray:
        im = np.empty((self.H, self.W, 4), np.float32)
        self._c(self._lib.rt_group_download_image(self.g, fptr(im)), "rt_group_download_image")
        return im

    def balance(self, header: Header, mode: int, rounds: int = 3) -> list[float]:
        """Cost-balance the strips (probe frame + `rounds` timed plans); returns the kept plan's
        per-strip ms per frame.  The strips restart with fresh rings."""
        ms = (C.c_double * self.n)()
        self._c(self._lib.rt_group_balance(self.g, header._p(), mode, rounds, ms), "rt_group_balance")
        return list(ms)


def plan_strips(row_cost, n: int) -> list[int]:
    """rt_plan_strips: contiguous strips of nearly equal total cost (host only)."""
    c = np.ascontiguousarray(row_cost, np.float64)
    b = (C.c_int * (n + 1))()
    _check(_lib.load().rt_plan_strips(c.ctypes.data_as(C.POINTER(C.c_double)), c.size, n, b), "rt_plan_strips")
    return list(b)


def plan_strips_gather(row_ms, n: int, width: int, link_gbps: float, ingest_gbps: float):
    """rt_plan_strips_gather (host only): strips AND root strip minimising
    max(render, per-link copy, root ingest); returns (bounds, root_strip, {T, render, link, ingest} ms)."""
    c = np.ascontiguousarray(row_ms, np.float64)
    b = (C.c_int * (n + 1))()
    root = C.c_int()
    out = (C.c_double * 4)()
    _check(_lib.load().rt_plan_strips_gather(c.ctypes.data_as(C.POINTER(C.c_double)), c.size, n, width,
                                             float(link_gbps), float(ingest_gbps), b, C.byref(root), out),
           "rt_plan_strips_gather")
    return list(b), root.value, dict(zip(("bound_ms", "render_ms", "link_ms", "ingest_ms"), list(out)))


def strip_gather_bound(row_ms, bounds, root_strip: int, width: int, link_gbps: float, ingest_gbps: float) -> dict:
    """rt_strip_gather_bound: the frame bound of a given plan {T, render, link, ingest} (ms)."""
    c = np.ascontiguousarray(row_ms, np.float64)
    n = len(bounds) - 1
    b = (C.c_int * (n + 1))(*[int(x) for x in bounds])
    out = (C.c_double * 4)()
    _check(_lib.load().rt_strip_gather_bound(c.ctypes.data_as(C.POINTER(C.c_double)), c.size, b, n, int(root_strip),
                                             width, float(link_gbps), float(ingest_gbps), out),
           "rt_strip_gather_bound")
    return dict(zip(("bound_ms", "render_ms", "link_ms", "ingest_ms"), list(out)))


def calibrate_row_cost(bounds, row_cost, strip_ms) -> np.ndarray:
    """rt_calibrate_row_cost: rescale the profile so each strip's total is its measured time."""
    c = np.array(row_cost, np.float64)
    n = len(bounds) - 1
    b = (C.c_int * (n + 1))(*[int(x) for x in bounds])
    t = np.ascontiguousarray(strip_ms, np.float64)
    _check(_lib.load().rt_calibrate_row_cost(c.ctypes.data_as(C.POINTER(C.c_double)), c.size, b, n,
                                             t.ctypes.data_as(C.POINTER(C.c_double))), "rt_calibrate_row_cost")
    return c


class FrameDriver:
    """compute() of src/main.cpp:553-578 with its per-frame host updates: the frame ring
    (static frame_num, 555/619), fill_rand_buffer for AO modes (seeded: 7000 + frame count),
    moving_light for Phong modes."""

    def __init__(self, renderer: Renderer, header: Header, lighting: int, light_movement: bool = False,
                 rand_seed0: int = 7000):
        self.r, self.h, self.lighting = renderer, header, lighting
        self.light_movement = light_movement
        self.frame_num = 0
        self.frames_done = 0
        self.rand_seed0 = rand_seed0

    def compute_many(self, n: int) -> int:
        """n compute() calls in one C++ loop (rt_compute_frames): same frames, less host time."""
        self.frame_num = self.r.compute_frames(self.h, self.lighting, self.frame_num, n,
                                               self.rand_seed0 + self.frames_done, self.light_movement)
        self.frames_done += n
        return self.frame_num

    def compute(self) -> int:
        if self.lighting in (1, 2):
            self.h.fill_rand_buffer(self.rand_seed0 + self.frames_done)
        else:
            self.h.moving_light(self.light_movement)
        self.h.set_mode(self.frame_num, self.h.num_objects)
        self.r.upload_header(self.h)
        self.frame_num = self.r.dispatch(self.lighting, self.frame_num)
        self.frames_done += 1
        return self.frame_num
