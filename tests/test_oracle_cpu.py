"""Pinning the CPU oracle (oracle/rt_oracle.c) without a runnable reference:
  * analytic known-answer tests: empty scene -> background, centre ray vs one
    sphere -> t = |c - cam| - r, shadowed point -> colour * 0.06, miss depth/normal zeros;
  * an independent numpy restatement written from the GLSL (oracle/numpy_ref.py), compared on
    small frames for every program, built-in and synthetic scenes, multi-frame sequences;
  * random()'s sin, correctly rounded (<= 0.5 ulp against mpmath; more in test_sin_cpu.py).
"""
import sys

import numpy as np
import pytest

import oracle
from conftest import assert_close
from oracle import numpy_ref
from real_time_ray_tracer_amd import SSBO, Header, aspect_for

GAMMA = np.float32(1.0) / np.float32(2.2)


def test_det_sin_is_a_sin():
    """random()'s sin is the correctly rounded binary32 sin: <= 0.5 ulp on every sample (the
    full check against mpmath and the plain binary64 re-execution is tests/test_sin_cpu.py)."""
    import mpmath as mp
    rng = np.random.default_rng(1)
    x = np.concatenate([rng.uniform(-5e5, 5e5, 1500), rng.uniform(-4, 4, 500)]).astype(np.float32)
    ours = oracle.det_sin(x)
    for xi, yi in zip(x, ours):
        with mp.workprec(200):
            s = mp.sin(mp.mpf(float(xi)))
            err = abs(mp.mpf(float(yi)) - s)
        ulp = 2.0 ** (np.frexp(abs(float(s)))[1] - 24)
        assert float(err) <= 0.5 * ulp, (float(xi), float(yi))
    plain = numpy_ref.det_sin(x)  # (float)sin((double)x): equal here (no double-rounding input drawn)
    np.testing.assert_array_equal(ours, plain)


def test_random_hash_matches_numpy_restatement_and_is_in_unit_interval():
    rng = np.random.default_rng(2)
    xy = rng.uniform(0, 8000, (3000, 2)).astype(np.float32)
    c = oracle.random2(xy)
    n = numpy_ref.grandom(xy[:, 0], xy[:, 1])
    np.testing.assert_array_equal(c, n)
    assert (c >= 0).all() and (c < 1).all()


def test_sphere_kat_centre_ray():
    # ray from the camera straight at a sphere centre: t = |c - cam| - r
    pos = np.float32([0, 0, 14])
    d = np.float32([0, 0, -1])
    c = np.float32([0, 0, 0])
    lib = oracle.load()
    fp = lambda a: a.ctypes.data_as(oracle.C.POINTER(oracle.C.c_float))  # noqa: E731
    assert lib.rto_sphere_eval(fp(pos), fp(d), fp(c), 2.0) == pytest.approx(12.0, abs=0)
    # behind / inside
    assert lib.rto_sphere_eval(fp(pos), fp(-d), fp(c), 2.0) == -1.0
    assert lib.rto_sphere_eval(fp(c), fp(d), fp(c), 2.0) == pytest.approx(2.0)
    # miss
    c2 = np.float32([5, 0, 0])
    assert lib.rto_sphere_eval(fp(pos), fp(d), fp(c2), 2.0) == -1.0


def _render(h, W, H, mode, frames=1):
    s = SSBO(h, W, H)
    d = oracle.dims(W, H, h.S, h.AA)
    img = np.zeros((H, W, 4), np.float32)
    f = 0
    for _ in range(frames):
        s.data[1] = f
        f = oracle.dispatch(s.data, d, mode, f, img, nthreads=2)
    return s, img


@pytest.mark.parametrize("mode", [1, 2, 3, 4])
def test_empty_scene_is_background(mode):
    h = Header.builtin(1, 4)
    h.set_mode(0, 0)
    s, img = _render(h, 16, 12, mode)
    bg = h.vec4(6)
    expect = np.concatenate([np.power(bg[:3], GAMMA), [0]]).astype(np.float32)
    assert_close(img, np.broadcast_to(expect, img.shape), "background")
    if mode in (1, 2):
        assert not s.normals.any() and not s.depth.any()  # primary miss -> zero g-buffer


def test_shadowed_point_is_colour_times_006():
    # a big ground sphere lit from straight below the ground: every visible ground point is in
    # the ground sphere's own shadow -> colour * 0.06 (p_compute.glsl:218)
    W, H = 16, 12
    h = Header(2, 1)
    h.camera_basis((0, 0, 14), (0, 1, 0), (0, 0, 1), 1.333333)
    h.vec4(5)[:] = (0, -100, 0, 0)  # light below the ground sphere
    h.vec4(6)[:] = (0.1, 0.2, 0.3, 0)
    h.pack_sphere(0, (0, -35, 0), 33.0, (0.5, 0.25, 1.0))
    h.set_mode(0, 1)
    s, img = _render(h, W, H, 3)
    col = np.float32([0.5, 0.25, 1.0]) * np.float32(0.06)
    ground = img[0, W // 2, :3]
    assert_close(ground, np.power(col, GAMMA).astype(np.float32), "shadowed ground")  # pow: tolerance


def _scene(name, W, H, spp):
    a = aspect_for(W, H)
    if name[0] == "s" and name[1:].isdigit():
        return Header.builtin(int(name[1:]), spp, a)
    if name == "planes":
        h = Header.builtin(1, spp, a)
        h.pack_plane(5, (1, 0, 0.2), -9.0, (0.2, 0.7, 0.3), reflectivity=0.3)
        h.pack_sphere(6, (2, 3, -3), 1.0, (3, 3, 3), emissive=True)
        h.set_mode(0, 7)
        return h
    return Header.synthetic(int(name[3:]), spp, 1234, a)


@pytest.mark.parametrize("mode", [1, 2, 3, 4])
@pytest.mark.parametrize("scene", ["s1", "s6", "syn12", "planes"])
def test_c_oracle_matches_numpy_restatement(scene, mode):
    W, H, spp = 24, 18, 3
    h = _scene(scene, W, H, spp)
    frames = 3 if mode == 1 else 2
    sc = SSBO(h, W, H)
    sn = SSBO(h, W, H)
    d = oracle.dims(W, H, h.S, h.AA)
    ic = np.zeros((H, W, 4), np.float32)
    inn = np.zeros((H, W, 4), np.float32)
    f = 0
    for k in range(frames):
        hk = h.copy()
        hk.fill_rand_buffer(7000 + k)
        hk.set_mode(f, hk.num_objects)
        sc.set_header(hk)
        sn.set_header(hk)
        oracle.dispatch(sc.data, d, mode, f, ic, nthreads=2)
        f = numpy_ref.dispatch(sn.data, W, H, h.S, h.AA, mode, f, inn)
    assert_close(inn, ic, f"{scene} mode {mode} image")
    assert_close(sn.data, sc.data, f"{scene} mode {mode} ssbo")
    # everything but pow() outputs is computed identically
    assert np.array_equal(sn.depth.view(np.uint32), sc.depth.view(np.uint32))
    assert np.array_equal(sn.normals.view(np.uint32), sc.normals.view(np.uint32))


@pytest.mark.parametrize("mode", [1, 2, 3, 4])
def test_oracle_window_equals_whole_frame(mode):
    """rto_run_program_window (the full-size tile checker): a window's trace passes over the window
    plus a 1-pixel halo and its post-process over the window give the whole-frame run's values
    inside the window, over a multi-frame sequence (temporal ring included)."""
    W, H, spp, frames = 40, 30, 4, 4
    x0, x1, y0, y1 = 9, 27, 6, 19
    h0 = Header.builtin(1, spp, aspect_for(W, H))
    progs = {1: [oracle.AOP_COMPUTE, oracle.AOP_POSTPROCESSING], 2: [oracle.AO_COMPUTE], 3: [oracle.P_COMPUTE],
             4: [oracle.H_COMPUTE]}[mode]
    outs = []
    for window in (False, True):
        h = h0.copy()
        d = oracle.dims(W, H, h.S, h.AA)
        buf = np.zeros(h.data.size + 3 * 8 * W * H * 4, np.float32)
        img = np.zeros((H, W, 4), np.float32)
        f = 0
        for k in range(frames):
            h.fill_rand_buffer(7000 + k) if mode in (1, 2) else h.moving_light(True)
            h.set_mode(f, h.num_objects)
            buf[:h.data.size] = h.data
            for p in progs:
                if not window:
                    oracle.run_program(buf, d, p, f, img)
                elif p in (oracle.AOP_COMPUTE, oracle.AO_COMPUTE):
                    oracle.run_program(buf, d, p, f, img, y0 - 1, y1 + 1, x0=x0 - 1, x1=x1 + 1)
                else:
                    oracle.run_program(buf, d, p, f, img, y0, y1, x0=x0, x1=x1)
            f = (f + 1) % 8
        ring = buf[h.data.size:].reshape(3, 8, W, H, 4)[:, :, x0:x1, y0:y1]
        outs.append((img[y0:y1, x0:x1].copy(), ring.copy()))
    np.testing.assert_array_equal(outs[1][0].view(np.uint32), outs[0][0].view(np.uint32))
    np.testing.assert_array_equal(outs[1][1].view(np.uint32), outs[0][1].view(np.uint32))


def _dup_scene(W, H, spp):
    """24 synthetic spheres, then exact duplicates of some of them at indices that land in the
    same lane of a later vector block (i + 8, i + 16) and in a neighbouring lane (i + 1): the
    vectorised sphere scan (8 or 16 spheres per step) must keep the reference's lowest-index
    winner of every tie (p_compute.glsl:177-188)."""
    a = aspect_for(W, H)
    base = Header.synthetic(24, spp, 1234, a, num_shapes=40)
    h = base.copy()
    shapes = h.data[28:28 + 40 * 20].reshape(40, 5, 4)
    src = shapes[:24].copy()
    order = list(range(24)) + [3, 1, 5, 9, 0, 4, 13, 2, 17, 6, 10, 11, 7, 12, 8, 14]
    for i, j in enumerate(order):
        shapes[i] = src[j]
    h.set_mode(0, 40)
    return h


@pytest.mark.parametrize("mode", [1, 2, 3, 4])
@pytest.mark.parametrize("scene", ["syn40", "dups"])
def test_vector_scan_matches_numpy_restatement(scene, mode):
    """The oracle's closest-hit and shadow scans run 8 (AVX2) or 16 (AVX-512) spheres per step
    (rt_oracle.c closest_hit / shadow_ray); the numpy restatement scans one sphere at a time in
    the reference's order.  Several vector blocks, padding, and ties across lanes and blocks."""
    W, H, spp = 20, 16, 2
    h = _dup_scene(W, H, spp) if scene == "dups" else _scene(scene, W, H, spp)
    sc, sn = SSBO(h, W, H), SSBO(h, W, H)
    d = oracle.dims(W, H, h.S, h.AA)
    ic, inn = np.zeros((H, W, 4), np.float32), np.zeros((H, W, 4), np.float32)
    f = 0
    for k in range(2):
        hk = h.copy()
        hk.fill_rand_buffer(7000 + k) if mode in (1, 2) else hk.moving_light(True)
        hk.set_mode(f, hk.num_objects)
        sc.set_header(hk)
        sn.set_header(hk)
        oracle.dispatch(sc.data, d, mode, f, ic, nthreads=2)
        f = numpy_ref.dispatch(sn.data, W, H, h.S, h.AA, mode, f, inn)
    assert_close(inn, ic, f"{scene} mode {mode} image")
    assert np.array_equal(sn.depth.view(np.uint32), sc.depth.view(np.uint32))
    assert np.array_equal(sn.normals.view(np.uint32), sc.normals.view(np.uint32))


def test_native_build_equals_portable_build():
    """The oracle's two builds (x86-64-v3 AVX2, and the Zen AVX-512 build the GPU box's checker and
    CPU baseline use) give bit-identical frames: same source, same binary32 operations."""
    import subprocess
    if not oracle.NATIVE_PATH.exists():
        pytest.skip("no native build")
    flags = open("/proc/cpuinfo").read()
    if not all(f" {x}" in flags for x in ("avx512f", "avx512vl", "avx512bw", "avx512dq")):
        pytest.skip("host has no AVX-512")
    code = r'''
import sys, numpy as np, ctypes as C
sys.path.insert(0, sys.argv[1])
import oracle
oracle.LIB_PATH = oracle.NATIVE_PATH if sys.argv[2] == "native" else oracle.LIB_PATH
from real_time_ray_tracer_amd import SSBO, Header, aspect_for
W, H = 24, 18
out = []
for S, spp, mode in ((40, 3, 1), (37, 2, 2), (21, 1, 4), (19, 1, 3)):
    h = Header.synthetic(S, spp, 99 + S, aspect_for(W, H))
    s = SSBO(h, W, H); d = oracle.dims(W, H, h.S, h.AA); img = np.zeros((H, W, 4), np.float32); f = 0
    for k in range(3):
        hk = h.copy(); hk.fill_rand_buffer(7000 + k) if mode < 3 else hk.moving_light(True)
        hk.set_mode(f, hk.num_objects); s.set_header(hk); f = oracle.dispatch(s.data, d, mode, f, img, nthreads=2)
    out.append(s.data.view(np.uint32).copy()); out.append(img.view(np.uint32).copy())
np.save(sys.argv[3], np.concatenate([o.ravel() for o in out]))
'''
    import tempfile
    from pathlib import Path
    root = str(Path(__file__).resolve().parents[1])
    with tempfile.TemporaryDirectory() as td:
        res = []
        for which in ("portable", "native"):
            p = f"{td}/{which}.npy"
            subprocess.run([sys.executable, "-c", code, root, which, p], check=True)
            res.append(np.load(p))
    np.testing.assert_array_equal(res[0], res[1])
