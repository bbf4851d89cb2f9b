"""GPU parity: the HIP path through the C ABI against the CPU oracle on identical inputs.

Bar (BASELINE.json north star): every channel within |g-c| <= 1e-4*max(|g|,|c|) + 1e-6.
Control-flow-carrying values (normals, depth, and every pixel of modes whose output has no
pow) are additionally required to be bit-identical, which is what the shared float
semantics (oracle/rt_oracle.h) promise.
"""
import numpy as np
import pytest

import oracle
from conftest import assert_bitwise, assert_close
from real_time_ray_tracer_amd import (AO_COMPUTE, AOP_COMPUTE, AOP_POSTPROCESSING, H_COMPUTE, P_COMPUTE,
                                      SSBO, FrameDriver, Header, Renderer, _lib, aspect_for)

pytestmark = pytest.mark.gpu


def make_header(scene: str, W: int, H: int, spp: int) -> Header:
    a = aspect_for(W, H)
    if scene.startswith("s") and scene[1:].isdigit():
        return Header.builtin(int(scene[1:]), spp, a)
    if scene.startswith("syn") and scene.endswith("p"):  # synthetic spheres + one ground plane
        n = int(scene[3:-1])
        h = Header.synthetic(n, spp, 1234, a, num_shapes=n + 1)
        h.pack_plane(n, (0, 1, 0), -2.5, (0.45, 0.4, 0.35))
        h.set_mode(0, n + 1)
        return h
    if scene.startswith("syn"):
        return Header.synthetic(int(scene[3:]), spp, 1234, a)
    if scene == "planetie":  # scene1 + an identical copy of its plane: the lower index must win every tie
        h = Header.builtin(1, spp, a)
        h.pack_plane(5, (0, 1, 0), -4.0, (0.9, 0.9, 0.1))
        h.pack_sphere(6, (0, -0.5, 0), 2.0, (0.1, 0.9, 0.9), reflectivity=0.5)  # copy of sphere 0
        h.set_mode(0, 7)
        return h
    if scene == "manyplanes":  # 20 spheres + 70 planes (> 64: the unmasked plane tail), tilted,
        rng = np.random.default_rng(7)  # some with non-unit normals, some facing the camera
        h = Header.synthetic(20, spp, 1234, a, num_shapes=90)
        for k in range(70):
            n = rng.normal(size=3)
            n /= np.linalg.norm(n)
            if k % 7 == 0:
                n *= 2.0
            h.pack_plane(20 + k, n, -float(rng.uniform(25.0, 60.0)), rng.uniform(0.1, 0.9, 3),
                         reflectivity=float(rng.choice([1.0, 0.3])), emissive=bool(k % 11 == 0))
        h.set_mode(0, 90)
        return h
    if scene == "planes":  # spheres + planes + a (never hit) rectangle
        h = Header.builtin(1, spp, a)
        h.pack_plane(5, (1, 0, 0.2), -9.0, (0.2, 0.7, 0.3), reflectivity=0.3)
        h.pack_rectangle(6, (4, 6, 4), (0, 0, -8), (-8, 0, 0), (1.5, 1.5, 1.5), emissive=True)
        h.pack_sphere(7, (2, 3, -3), 1.0, (3, 3, 3), emissive=True)
        h.set_mode(0, 8)
        return h
    if scene == "empty":
        h = Header.builtin(1, spp, a)
        h.set_mode(0, 0)
        return h
    raise ValueError(scene)


def run_both(h: Header, W: int, H: int, mode: int, frames: int, max_depth: int = 20, light_movement=True):
    """Drive the GPU renderer and the oracle through the same frame sequence."""
    r = Renderer(W, H, h.S, h.AA, max_depth=max_depth)
    hg, ho = h.copy(), h.copy()
    s = SSBO(ho, W, H)
    d = oracle.dims(W, H, h.S, h.AA, D=max_depth)
    img = np.zeros((H, W, 4), np.float32)
    drv = FrameDriver(r, hg, mode, light_movement=light_movement)
    fo = 0
    for k in range(frames):
        drv.compute()
        if mode in (1, 2):
            ho.fill_rand_buffer(7000 + k)
        else:
            ho.moving_light(light_movement)
        ho.set_mode(fo, ho.num_objects)
        s.set_header(ho)
        fo = oracle.dispatch(s.data, d, mode, fo, img)
    assert drv.frame_num == fo
    g = r.download()
    r.close()
    return g, s, img


@pytest.mark.parametrize("mode", [1, 2, 3, 4])
@pytest.mark.parametrize("scene", ["s1", "s5", "s6", "syn16", "planes", "empty", "planetie", "manyplanes", "syn30p"])
def test_mode_parity_small(scene, mode):
    W, H, spp = 64, 48, 4
    h = make_header(scene, W, H, spp)
    frames = 3 if mode in (1, 2) else 2
    g, s, img = run_both(h, W, H, mode, frames)
    assert_close(g.image, img, f"{scene} mode {mode} image")
    assert_close(g.pixels, s.pixels, f"{scene} mode {mode} pixels")
    assert_bitwise(g.normals, s.normals, f"{scene} mode {mode} normals")
    assert_bitwise(g.depth, s.depth, f"{scene} mode {mode} depth")


@pytest.mark.parametrize("chunks", [(2, 3), (37, 1)])
@pytest.mark.parametrize("mode", [1, 2, 3, 4, 5])
def test_compute_frames_equals_frame_by_frame(mode, chunks):
    """rt_compute_frames (the C++ frame loop; sequential frames go in batches of up to 32 device
    header copies with one upload) renders the same frames as FrameDriver.compute() called once
    per frame: g-buffer ring, image, frame slot and the updated header, bit for bit — across a
    batch boundary too, and with one more per-frame call after the loop (the state it leaves).
    "mode 5": mode 2 on 200 spheres, so the multi-frame launches take the above-128-sphere
    instantiations (the word-by-word pre-test, per-frame rand_buffer read from global memory)."""
    W, H, spp = 48, 32, 4
    scene = {4: "syn16p", 5: "syn200"}.get(mode, "syn16")
    mode = 2 if mode == 5 else mode
    h = make_header(scene, W, H, spp)
    n = sum(chunks) + 1
    outs = []
    for many in (False, True, "one launch per frame"):
        r = Renderer(W, H, h.S, h.AA)
        if many == "one launch per frame":
            r.set_frame_batch(1)  # rt_set_frame_batch: the reference's dispatch shape (the default)
        elif many:
            r.set_frame_batch(32)  # multi-frame launches (opt-in): the same frames
        hh = h.copy()
        drv = FrameDriver(r, hh, mode, light_movement=True)
        if many:
            for c in chunks:
                drv.compute_many(c)
            drv.compute()
        else:
            for _ in range(n):
                drv.compute()
        outs.append((r.download(), hh.data.copy(), drv.frame_num))
        r.close()
    (g0, h0, f0) = outs[0]
    for g1, h1, f1 in outs[1:]:
        assert f0 == f1 == n % 8
        assert_bitwise(h1, h0, f"mode {mode} header")
        for name in ("image", "pixels", "normals", "depth"):
            assert_bitwise(getattr(g1, name), getattr(g0, name), f"mode {mode} {name}")


@pytest.mark.parametrize("scene", ["syn16", "syn16p"])
@pytest.mark.parametrize("spp", [1, 3, 4, 16, 64])
def test_ao_spp_variants(spp, scene):
    W, H = 40, 24
    h = make_header(scene, W, H, spp)
    g, s, img = run_both(h, W, H, 1, 2)
    assert_close(g.image, img, f"spp {spp} image")
    assert_bitwise(g.depth, s.depth, f"spp {spp} depth")
    assert_bitwise(g.normals, s.normals, f"spp {spp} normals")


@pytest.mark.parametrize("nobj", ["64", "100", "128", "129", "200", "63p", "127p", "150p", "200@4", "200@64", "150p@4",
                                  "300@64"])
def test_ao_scene_sizes(nobj):
    """Sphere counts around the kernel's 64-sphere words and the 128-object LDS table limit
    (split tail rounds + the first bounce's per-ray pre-test table up to 128; above, the pre-test
    rows one word at a time with rand_buffer read from global memory, RT_PT_WIDE); "p": plus a
    ground plane (the plane-testing instantiations, with and without the LDS table); "@n": n spp
    (the spp 4 and 64 instantiations; 16 otherwise)."""
    W, H = 48, 32
    scene, _, spp = nobj.partition("@")
    h = make_header(f"syn{scene}", W, H, int(spp) if spp else 16)
    for mode in (1, 2):
        g, s, img = run_both(h, W, H, mode, 2)
        assert_close(g.image, img, f"{nobj} spheres mode {mode} image")
        assert_bitwise(g.depth, s.depth, f"{nobj} spheres mode {mode} depth")
        assert_bitwise(g.normals, s.normals, f"{nobj} spheres mode {mode} normals")


@pytest.mark.parametrize("mode", [1, 4])
def test_max_depth_variants(mode):
    W, H = 48, 32
    h = make_header("s6", W, H, 4)
    for D in (1, 2, 5):
        g, s, img = run_both(h, W, H, mode, 2, max_depth=D)
        assert_close(g.image, img, f"D={D} image")
        assert_bitwise(g.depth, s.depth, f"D={D} depth")


def test_mode1_long_sequence_ring_wraps():
    """12 frames: the 8-slot ring wraps, so temporal history and stale-depth reads are exercised."""
    W, H = 48, 32
    h = make_header("s5", W, H, 4)
    g, s, img = run_both(h, W, H, 1, 12)
    assert_close(g.image, img, "image")
    assert_close(g.pixels, s.pixels, "pixels ring")
    assert_bitwise(g.depth, s.depth, "depth ring")
    assert_bitwise(g.normals, s.normals, "normals ring")


def camera_path(k: int):
    """A scripted fly-through (what the reference's keyboard camera does each frame,
    src/main.cpp:701-760): the camera moves forward and sideways and turns a little each frame."""
    a = 0.05 * k
    loc = (0.6 * np.sin(a) * k, 0.15 * k, 14.0 - 0.7 * k)
    look = (np.sin(a), -0.04 * k, np.cos(a))  # look_towards (w); the basis normalizes u and v
    return loc, (0.0, 1.0, 0.0), look


@pytest.mark.parametrize("mode,pipelined", [(1, False), (1, True), (2, False), (3, False), (4, False)])
def test_moving_camera_parity(mode, pipelined):
    """The camera basis (render(), src/main.cpp:772-779) changes every frame: the pool and tile
    cones follow it, and in mode 1 the temporal filter (aop_postprocessing.glsl:177-201) now
    rejects history wherever the scene moved across the pixel.  11 frames (the ring wraps)."""
    W, H, spp = 64, 48, 4
    h = make_header("syn16p", W, H, spp)
    r = Renderer(W, H, h.S, h.AA)
    if pipelined:
        r.enable_pipelining(True)
    ho = h.copy()
    s = SSBO(ho, W, H)
    d = oracle.dims(W, H, h.S, h.AA)
    img = np.zeros((H, W, 4), np.float32)
    fg = fo = 0
    for k in range(11):
        for hh in (h, ho):
            hh.camera_basis(*camera_path(k), aspect_for(W, H))
            if mode in (1, 2):
                hh.fill_rand_buffer(7000 + k)
            else:
                hh.moving_light(True)
        h.set_mode(fg, h.num_objects)
        r.upload_header(h)
        fg = r.dispatch(mode, fg)
        ho.set_mode(fo, ho.num_objects)
        s.set_header(ho)
        fo = oracle.dispatch(s.data, d, mode, fo, img)
        assert fg == fo
    g = r.download()
    r.close()
    assert_close(g.image, img, f"mode {mode} image")
    assert_close(g.pixels, s.pixels, f"mode {mode} pixels ring")
    assert_bitwise(g.normals, s.normals, f"mode {mode} normals ring")
    assert_bitwise(g.depth, s.depth, f"mode {mode} depth ring")


def test_mode_switching_shares_the_ring():
    """compute() keeps one static frame counter across modes (src/main.cpp:555)."""
    W, H = 40, 30
    h = make_header("s6", W, H, 4)
    r = Renderer(W, H, h.S, h.AA)
    ho = h.copy()
    s = SSBO(ho, W, H)
    d = oracle.dims(W, H, h.S, h.AA)
    img = np.zeros((H, W, 4), np.float32)
    f = 0
    for k, mode in enumerate([1, 2, 3, 1, 4, 1, 1, 2, 1, 1]):
        h.fill_rand_buffer(100 + k)
        h.set_mode(f, h.num_objects)
        r.upload_header(h)
        s.set_header(h)
        fg = r.dispatch(mode, f)
        f = oracle.dispatch(s.data, d, mode, f, img)
        assert fg == f
    gb = r.download()
    assert_close(gb.image, img, "image")
    assert_close(gb.pixels, s.pixels, "pixels")
    assert_bitwise(gb.depth, s.depth, "depth")


@pytest.mark.parametrize("two", [False, True])
def test_host_buffer_path_mirrors_compute_one_two_shader(two):
    W, H = 32, 24
    h = make_header("s1", W, H, 4)
    r = Renderer(W, H, h.S, h.AA)
    sg, so = SSBO(h, W, H), SSBO(h, W, H)
    d = oracle.dims(W, H, h.S, h.AA)
    ig, io = np.zeros((H, W, 4), np.float32), np.zeros((H, W, 4), np.float32)
    fg = fo = 0
    for k in range(3):
        if two:
            fg = r.compute_two_shaders(sg, fg, AOP_COMPUTE, AOP_POSTPROCESSING, ig)
            oracle.run_program(so.data, d, AOP_COMPUTE, fo, io)
            oracle.run_program(so.data, d, AOP_POSTPROCESSING, fo, io)
        else:
            fg = r.compute_one_shader(sg, fg, [AO_COMPUTE, P_COMPUTE, H_COMPUTE][k], ig)
            oracle.run_program(so.data, d, [AO_COMPUTE, P_COMPUTE, H_COMPUTE][k], fo, io)
        fo = (fo + 1) % 8
        assert fg == fo
    assert sg.data[1] == so.data[1]  # mode.y written back
    assert_close(ig, io, "image")
    assert_close(sg.data, so.data, "whole ssbo")


def test_strips_equal_full_frame_bitwise():
    """G row strips (each with its own ring + 1-row halo) reproduce the whole frame exactly."""
    W, H, G = 48, 37, 3
    h = make_header("syn16", W, H, 4)
    bounds = [round(i * H / G) for i in range(G + 1)]
    full = Renderer(W, H, h.S, h.AA)
    strips = [Renderer(W, H, h.S, h.AA, rows=(bounds[i], bounds[i + 1])) for i in range(G)]
    f = 0
    for k, mode in enumerate([1, 1, 2, 1, 3, 1]):
        h.fill_rand_buffer(7000 + k)
        h.set_mode(f, h.num_objects)
        for rr in [full] + strips:
            rr.upload_header(h)
            fn = rr.dispatch(mode, f)
        f = fn
    gf = full.download()
    parts = [s.download() for s in strips]
    assert_bitwise(np.concatenate([p.image for p in parts], 0), gf.image, "strip images")
    for name in ("pixels", "normals", "depth"):
        assert_bitwise(np.concatenate([getattr(p, name) for p in parts], 2), getattr(gf, name), f"strip {name}")


def test_math_primitives_bitwise():
    r = Renderer(8, 8, 1, 1)
    rng = np.random.default_rng(0)
    x = np.concatenate([rng.uniform(-5e5, 5e5, 20000), rng.uniform(-10, 10, 5000),
                        [0.0, -0.0, 1e-30, 3.14159265, 1.5707964, 1e6, 3e7],
                        # huge arguments: the Payne-Hanek path (|x| >= 2^22)
                        [3.3e9, -3.3e9, 3.4e9, -3.4e9, 1e10, -1e10, 3e38, -3e38, 4194304.0, -4194304.0]]).astype(np.float32)
    ref = oracle.det_sin(x)
    assert_bitwise(r.selftest_math(_lib.RT_MATH_SIN, x, x.size), ref, "det_sin")
    bad = np.array([np.inf, -np.inf, np.nan], np.float32)
    assert np.isnan(r.selftest_math(_lib.RT_MATH_SIN, bad, bad.size)).all() and np.isnan(oracle.det_sin(bad)).all()
    xy = rng.uniform(0, 8000, (20000, 2)).astype(np.float32)
    assert_bitwise(r.selftest_math(_lib.RT_MATH_RANDOM, xy, len(xy)), oracle.random2(xy), "random")
    v = np.concatenate([rng.uniform(0, 1e6, 100000), 10.0 ** rng.uniform(-45, 38.5, 100000),
                        [0.0, -0.0, 1e-45, 1e-40, 2.0 ** -96, 2.0 ** -97, np.inf, 3.4e38]]).astype(np.float32)
    assert_bitwise(r.selftest_math(_lib.RT_MATH_SQRT, v, v.size), np.sqrt(v), "sqrt")
    ab = rng.uniform(-1e3, 1e3, (100000, 2)).astype(np.float32)
    assert_bitwise(r.selftest_math(_lib.RT_MATH_DIV, ab, len(ab)), ab[:, 0] / ab[:, 1], "div")
    r.close()


def _shadow_occludes_b64(l, ln, t):
    """shadow_ray's occluder test in binary64 (p_compute.glsl:159-161, the oracle's
    rto_shadow sequence): t > 0.0001 and sqrt(fma(dz, dz, fma(dy, dy, dx * dx))) < len with
    d = t * l; each fma rounded once, by exact rationals."""
    from fractions import Fraction as Fr
    import math
    t = float(t)
    if not t > float(np.float32(0.0001)):
        return False
    dx, dy, dz = t * float(l[0]), t * float(l[1]), t * float(l[2])

    def fma(a, b, c):
        if not (math.isfinite(a) and math.isfinite(b) and math.isfinite(c)):
            return a * b + c
        return float(Fr(a) * Fr(b) + Fr(c))
    q = fma(dz, dz, fma(dy, dy, dx * dx))
    return (math.sqrt(q) if q >= 0 else math.nan) < float(ln)


def test_shadow_occluder_decision():
    """The production kernels decide every shadow occluder test with the binary64 sequence
    (RT_SHADOW_FAST = 0, rt_kernels_impl.h: shadow_bounds gives {0, inf}, so no decision is taken
    in float).  Its decision equals the binary64 sequence evaluated exactly on t drawn at and
    around len (1 -+ 2^-12) (the float fast path's bounds, kept as probe points), around len
    itself, and for degenerate light vectors (zero, tiny, huge).  The float fast path is an A/B
    variant only and is not compiled into librtrt.so."""
    r = Renderer(8, 8, 1, 1)
    rng = np.random.default_rng(11)
    n = 6000
    d = rng.normal(size=(n, 3))
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    lv = (d * 10.0 ** rng.uniform(-2, 3.5, (n, 1))).astype(np.float32)
    lv = np.concatenate([lv, np.array([[0, 0, 0], [1e-25, 2e-25, 0], [3e-20, 0, 1e-20], [1e25, 1e25, 0],
                                       [3e38, 3e38, 0], [np.nan, 0, 0], [np.inf, 1, 0]], np.float32)])
    m = len(lv)
    probe = r.selftest_math(_lib.RT_MATH_SHADOW, np.concatenate([lv, np.ones((m, 1), np.float32)], 1), m)
    ln = probe.reshape(m, 5)[:, 3]
    # t per light vector: both bounds and len itself, each -+ a few ulps, plus random and special values
    ts = []
    for f in (1 - 2.0 ** -12, 1 + 2.0 ** -12, 1.0, 1 - 2.0 ** -20, 1 + 2.0 ** -20):
        base = (ln.astype(np.float64) * f).astype(np.float32)
        for k in (-3, -1, 0, 1, 3):
            ts.append(np.nextafter(base, np.float32(np.inf) if k > 0 else np.float32(-np.inf)) if k else base)
            for _ in range(abs(k) - 1):
                ts[-1] = np.nextafter(ts[-1], np.float32(np.inf) if k > 0 else np.float32(-np.inf))
    ts.append((ln * rng.uniform(0, 2, m)).astype(np.float32))
    ts.append(np.full(m, np.float32(0.0001)))
    ts.append(np.full(m, np.nextafter(np.float32(0.0001), np.float32(1))))
    for v in (-1.0, np.inf, np.nan):
        ts.append(np.full(m, v, np.float32))
    T = np.stack(ts, 1).astype(np.float32)  # [m, k]
    k = T.shape[1]
    inp = np.concatenate([np.repeat(lv, k, 0), T.reshape(-1, 1)], 1)
    out = r.selftest_math(_lib.RT_MATH_SHADOW, inp, len(inp)).reshape(-1, 5)
    r.close()
    got = out[:, 4] == 1.0
    want = np.array([_shadow_occludes_b64(o[:3], o[3], t) for o, t in zip(out, inp[:, 3])])
    bad = np.flatnonzero(got != want)
    assert bad.size == 0, f"{bad.size} of {len(inp)} decisions differ; first: lv={inp[bad[0], :3]} t={inp[bad[0], 3]!r} " \
                          f"len={out[bad[0], 3]!r} kernel={got[bad[0]]} binary64={want[bad[0]]}"
    assert want.any() and (~want).any()


def test_sqrt_rn_exhaustive():
    """The kernels' explicit sqrt sequence equals sqrtf on every non-negative float
    (0 .. +inf: 2^31 - 2^23 + 1 bit patterns), on the device."""
    r = Renderer(8, 8, 1, 1)
    per, n = 2048, 1 << 20
    bad = r.selftest_math(_lib.RT_MATH_SQRT_SWEEP, np.array([per], np.float32), n)
    r.close()
    assert n * per > 0x7f800000
    assert float(bad.sum()) == 0.0, f"{int(bad.sum())} mismatching inputs"


def test_sqrt_tail_exhaustive():
    """The sphere hit tail's sqrt (v_rsq_f32 + Markstein's correction) equals sqrtf on every
    float in [2^-96, FLT_MAX] and stays in [0, 2^-47] below 2^-96, on the device."""
    r = Renderer(8, 8, 1, 1)
    per, n = 2048, 1 << 20
    bad = r.selftest_math(_lib.RT_MATH_SQRT_TAIL_SWEEP, np.array([per], np.float32), n)
    r.close()
    assert n * per > 0x7f7fffff
    assert float(bad.sum()) == 0.0, f"{int(bad.sum())} inputs break the contract"


def test_det_sin_exhaustive():
    """random()'s sin on the device (csrc/rt_sin.h: binary64 fast path, Payne-Hanek beyond
    2^22, exception table) equals the oracle's independent correctly rounded sin (glibc's binary64
    sin, quad-precision sinq where its rounding is ambiguous) on all 2^32 bit patterns, bit for
    bit (NaN == NaN, -0 included)."""
    import time
    r = Renderer(8, 8, 1, 1)
    chunk = 1 << 27
    total, firsts = 0, []
    t0 = time.time()
    for start in range(0, 1 << 32, chunk):
        got = r.selftest_math(_lib.RT_MATH_SIN_RANGE, np.array([start], np.uint32).view(np.float32), chunk)
        n, bad = oracle.sin_check_range(start, got, max_bad=8)
        total += n
        firsts += [f"0x{int(b):08x}" for b in bad]
        if start % (1 << 30) == 0:
            print(f"  sin sweep {start:#010x}: {total} mismatches so far, {time.time() - t0:.1f} s", flush=True)
    r.close()
    print(f"  sin sweep: all 2^32 bit patterns, {total} mismatches, {time.time() - t0:.1f} s")
    assert total == 0, f"{total} inputs differ from the correctly rounded sin, e.g. {firsts[:8]}"


def test_sin_table_entries_are_ambiguous_on_this_device_build():
    """rt_sin_table.h was generated from a host build of rt_sin.h (tools/sin_enum.hip).
    Every table entry must still be an input this build's DEVICE code flags ambiguous (else the
    device would round its binary64 value without the table), and the device's sin must return
    the table's correctly rounded value on each: a codegen change shows here in milliseconds,
    beside the all-2^32 sweep above."""
    import re
    from pathlib import Path

    txt = (Path(__file__).resolve().parents[1] / "real_time_ray_tracer_amd" / "csrc" / "rt_sin_table.h").read_text()
    ntab = int(re.search(r"kSinTableN\s*=\s*(\d+)", txt).group(1))
    arrays = re.findall(r"kSinTable([XY])\[\d+\]\s*=\s*\{([^}]*)\}", txt)
    tab = {k: np.array([int(v, 16) for v in re.findall(r"0x([0-9A-Fa-f]+)u", body)], np.uint32) for k, body in arrays}
    assert len(tab["X"]) == len(tab["Y"]) == ntab
    r = Renderer(8, 8, 1, 1)
    out = r.selftest_math(_lib.RT_MATH_SIN_TABLE, np.zeros(1, np.float32), ntab + 8).reshape(-1, 2)
    vals = r.selftest_math(_lib.RT_MATH_SIN, tab["X"].view(np.float32), ntab)
    r.close()
    flags = out[:, 0]
    assert np.all(flags[ntab:] == -1.0)
    assert np.array_equal(out[:ntab, 1].view(np.uint32), tab["X"])
    assert np.all(flags[:ntab] == 1.0), [f"0x{int(x):08x}" for x in tab["X"][flags[:ntab] != 1.0]]
    assert np.array_equal(vals.view(np.uint32), tab["Y"])


def test_rcp_rn_exhaustive():
    """normalize's 1/sqrt (sqrt_rn_tail + v_rcp_f32 + one Newton step, with the compiler's
    sequence for out-of-range inputs) equals 1.0f/sqrtf on every non-negative float, and the
    reciprocal step equals 1.0f/x on every normal x in [2^-126, 2^126], on the device."""
    r = Renderer(8, 8, 1, 1)
    per, n = 2048, 1 << 20
    bad = r.selftest_math(_lib.RT_MATH_RCP_SWEEP, np.array([per], np.float32), n)
    r.close()
    assert n * per > 0x7f800000
    assert float(bad.sum()) == 0.0, f"{int(bad.sum())} mismatching inputs"


def test_errors_are_reported():
    r = Renderer(16, 16, 4, 4)
    with pytest.raises(_lib.RtError):
        r.dispatch(1, 0)  # no header uploaded yet
    h = Header.synthetic(4, 4, 1, 1.0)
    r.upload_header(h)
    with pytest.raises(_lib.RtError):
        r.dispatch(7, 0)
    with pytest.raises(_lib.RtError):
        r.dispatch(1, 8)
    with pytest.raises(_lib.RtError):
        r.compute_frames(h, 7, 0, 1)  # unknown mode
    with pytest.raises(_lib.RtError):
        r.compute_frames(h, 1, 8, 1)  # frame slot out of range
    with pytest.raises(_lib.RtError):
        r.compute_frames(h, 1, 0, -1)  # negative frame count
    assert r.compute_frames(h, 3, 6, 0) == 6  # no frames: the slot is returned unchanged
    h.set_mode(0, 5)  # more objects than capacity
    with pytest.raises(_lib.RtError):
        r.upload_header(h)
    with pytest.raises(_lib.RtError):
        r.compute_frames(h, 3, 0, 1)
    r.close()
    with pytest.raises(_lib.RtError):
        Renderer(16, 16, 4, 300)  # spp above the supported 256


@pytest.mark.parametrize("mode,pipelined", [(1, False), (1, True), (2, False), (3, False), (4, False)])
@pytest.mark.parametrize("W,H", [(1, 1), (1, 6), (9, 1), (2, 3), (17, 5)])
def test_degenerate_frame_sizes(W, H, mode, pipelined):
    """Frames of one row / one column / a few pixels: partial pools and tiles everywhere, and
    every post-process neighbour test (aop_postprocessing.glsl:82-171) at its border value,
    over 10 frames so the 8-slot history ring wraps (the post-process reads every slot)."""
    spp = 4
    h0 = make_header("s1", W, H, spp)
    r = Renderer(W, H, h0.S, spp)
    if pipelined:
        r.enable_pipelining(True)
    hg, ho = h0.copy(), h0.copy()
    s = SSBO(ho, W, H)
    d = oracle.dims(W, H, h0.S, spp)
    img = np.zeros((H, W, 4), np.float32)
    fg = fo = 0
    for k in range(10 if mode in (1, 2) else 3):
        for hh, f in ((hg, fg), (ho, fo)):
            if mode in (1, 2):
                hh.fill_rand_buffer(7000 + k)
            else:
                hh.moving_light(True)
            hh.set_mode(f, hh.num_objects)
        r.upload_header(hg)
        fg = r.dispatch(mode, fg)
        s.set_header(ho)
        fo = oracle.dispatch(s.data, d, mode, fo, img)
        assert fg == fo
    g = r.download()
    r.close()
    what = f"{W}x{H} mode {mode}{' pipelined' if pipelined else ''}"
    assert_close(g.image, img, f"{what} image")
    assert_close(g.pixels, s.pixels, f"{what} pixels")
    assert_bitwise(g.normals, s.normals, f"{what} normals")
    assert_bitwise(g.depth, s.depth, f"{what} depth")
