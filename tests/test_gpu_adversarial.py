"""GPU parity on adversarial geometry (tests/adversarial_scenes.py): the cone-culled kernels
against the CPU oracle where their culling proofs have their margins — the camera inside a
sphere, spheres straddling or behind the camera plane, first-bounce origins inside spheres,
exactly tangent primaries (del == 0), radius-1e4 and radius-1e-3 spheres, duplicate /
overlapping / concentric spheres, the light inside a sphere, and 256 spheres (past the
128-object LDS tables).

Every scene runs in all four modes (mode 1 sequential and pipelined) at 64x48 (spp 4 and 16)
and as 64x64 tiles of a 3840x2160 frame (spp 16): the tiles of tests/test_gpu_fullsize.py's
choice plus tiles around each scene's constructed features.  Normals and depth bit-identical,
colours within the north-star tolerance.

Reference: resources/p_compute.glsl:77-109 (every root branch), 145-166 (shadow_ray),
177-188 (closest hit), ao_compute.glsl:183-194, h_compute.glsl:199-210.
"""
import numpy as np
import pytest

import oracle
from adversarial_scenes import NAMES, scene
from conftest import assert_bitwise, assert_close
from real_time_ray_tracer_amd import SSBO, Renderer
from test_gpu_fullsize import PROGS, T, pick_tiles, whole_frame_properties

pytestmark = pytest.mark.gpu


def advance(h, mode: int, k: int, frame: int):
    """The render loop's per-frame host update (src/main.cpp:553-578)."""
    if mode in (1, 2):
        h.fill_rand_buffer(7000 + k)
    else:
        h.moving_light(True)
    h.set_mode(frame, h.num_objects)


@pytest.mark.parametrize("mode,pipelined", [(1, False), (1, True), (2, False), (3, False), (4, False)])
@pytest.mark.parametrize("name", NAMES)
def test_adversarial_small(name, mode, pipelined):
    W, H = 64, 48
    for spp in ((4, 16) if mode in (1, 2) else (1,)):
        h0, _ = scene(name, W, H, spp)
        r = Renderer(W, H, h0.S, spp)
        if pipelined:
            r.enable_pipelining(True)
        hg, ho = h0.copy(), h0.copy()
        s = SSBO(ho, W, H)
        d = oracle.dims(W, H, h0.S, spp)
        img = np.zeros((H, W, 4), np.float32)
        fg = fo = 0
        for k in range(4 if mode in (1, 2) else 3):
            advance(hg, mode, k, fg)
            r.upload_header(hg)
            fg = r.dispatch(mode, fg)
            advance(ho, mode, k, fo)
            s.set_header(ho)
            fo = oracle.dispatch(s.data, d, mode, fo, img)
            assert fg == fo
        g = r.download()
        r.close()
        what = f"{name} mode {mode}{' pipelined' if pipelined else ''} spp {spp}"
        assert_close(g.image, img, f"{what} image")
        assert_close(g.pixels, s.pixels, f"{what} pixels")
        assert_bitwise(g.normals, s.normals, f"{what} normals")
        assert_bitwise(g.depth, s.depth, f"{what} depth")


FW, FH = 3840, 2160
FRAMES = {1: 3, 2: 2, 3: 2, 4: 2}


def oracle_window(h0, spp: int, mode: int, frames: int, x0, x1, y0, y1):
    """The oracle over columns [x0, x1) x rows [y0, y1) of the same frame sequence (trace passes
    over the window plus a 1-pixel halo, which the post-process reads)."""
    h = h0.copy()
    gy0, gy1 = max(0, y0 - 1), min(FH, y1 + 1)
    gx0, gx1 = max(0, x0 - 1), min(FW, x1 + 1)
    gh = gy1 - gy0
    d = oracle.dims(FW, FH, h.S, spp, gy0=gy0, gh=gh)
    buf = np.zeros(h.data.size + 3 * 8 * FW * gh * 4, np.float32)
    img = np.zeros((gh, FW, 4), np.float32)
    nt = oracle.nthreads_default()
    f = 0
    for k in range(frames):
        advance(h, mode, k, f)
        buf[:h.data.size] = h.data
        for p in PROGS[mode]:
            if p in (oracle.AOP_COMPUTE, oracle.AO_COMPUTE):
                oracle.run_program(buf, d, p, f, img, gy0, gy1, nthreads=nt, x0=gx0, x1=gx1)
            else:
                oracle.run_program(buf, d, p, f, img, y0, y1, nthreads=nt, x0=x0, x1=x1)
        f = (f + 1) % 8
    o = h.data.size
    n = 8 * FW * gh * 4
    ring = [buf[o + i * n:o + (i + 1) * n].reshape(8, FW, gh, 4)[:, x0:x1, y0 - gy0:y1 - gy0] for i in range(3)]
    return img[y0 - gy0:y1 - gy0, x0:x1], ring


@pytest.mark.parametrize("mode", [1, 2, 3, 4])
@pytest.mark.parametrize("name", NAMES)
def test_adversarial_full_size_tiles(name, mode):
    spp = 16 if mode in (1, 2) else 1
    frames = FRAMES[mode]
    h0, poi = scene(name, FW, FH, spp)
    r = Renderer(FW, FH, h0.S, spp)
    if mode == 1:
        r.enable_pipelining(True)
    h = h0.copy()
    f = 0
    for k in range(frames):
        advance(h, mode, k, f)
        r.upload_header(h)
        f = r.dispatch(mode, f)
    r.synchronize()
    img = r.image()
    tiles = pick_tiles(img)
    clamp = lambda x, y: (min(max(0, x - T // 2), FW - T), min(max(0, y - T // 2), FH - T))  # noqa: E731
    for i, (x, y) in enumerate(poi):
        tiles[f"feature{i}"] = clamp(x, y)
    for i, (x, y) in enumerate(whole_frame_properties(img, name)):
        tiles[f"odd{i}"] = clamp(x, y)
    for tname, (x0, y0) in tiles.items():
        want_img, (wp, wn, wd) = oracle_window(h0, spp, mode, frames, x0, x0 + T, y0, y0 + T)
        g = r.download_rect(x0, x0 + T, y0, y0 + T)
        what = f"{name} mode {mode} tile {tname} at ({x0}, {y0})"
        assert_close(g.image, want_img, f"{what} image")
        assert_close(g.pixels[:frames], wp[:frames], f"{what} pixels")
        if mode in (1, 2):
            assert_bitwise(g.normals[:frames], wn[:frames], f"{what} normals")
            assert_bitwise(g.depth[:frames], wd[:frames], f"{what} depth")
    r.close()
