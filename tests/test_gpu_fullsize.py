"""Parity at BASELINE.json's full sizes ("sampled 64x64 tiles plus full strips").

The GPU renders the whole frame for a sequence of frames; the CPU oracle re-executes only a
window of it on the same inputs and frame sequence:
  - 64x64 tiles chosen from the rendered image: the four corners, the flattest sky tile, the
    tile with the most silhouette edges, the brightest (emissive) tile and a ground tile;
  - whole frames: config (a) 640x480, (b) and (c) 1920x1080 (3 frames each) and the headline
    config (d) 3840x2160 over 10 pipelined frames (the temporal ring wraps);
  - full strips: a 270-row strip of config (d) (one eighth of the frame, the N = 8 strip
    height) and a 540-row strip of config (e) (8K, 256 spheres, 64 spp: the north star's
    8-GPU config, one rank's strip) over 10 frames, so its ring wraps and frames 8 and 9 read
    slots 0 and 1's stale depth (ao_compute.glsl:196-208).
Trace passes run over the window plus a 1-pixel halo (the post-process reads its 4
neighbours), the post-process over the window itself.  Normals and depth must agree bit for
bit, colours within the north-star tolerance |g-c| <= 1e-4 max(|g|,|c|) + 1e-6 (conftest).
Mode-1 configs run >= 10 frames, so the 8-slot temporal ring (aop_postprocessing.glsl:177-201)
wraps and every history slot holds a filtered frame.  Plus size-independent properties of the
whole frame: finite, non-negative, alpha 0.
"""
import sys
import time

import numpy as np
import pytest

import oracle
from bench import CONFIGS, config_header
from conftest import assert_bitwise, assert_close
from real_time_ray_tracer_amd import Renderer

pytestmark = pytest.mark.gpu

T = 64  # tile size
PROGS = {1: [oracle.AOP_COMPUTE, oracle.AOP_POSTPROCESSING], 2: [oracle.AO_COMPUTE], 3: [oracle.P_COMPUTE],
         4: [oracle.H_COMPUTE]}


def advance(h, mode: int, k: int, frame: int, moving: bool = False):
    """The render loop's per-frame host update (src/main.cpp:553-578): rand_buffer for the AO
    modes, moving_light for the Phong modes; then mode.y = frame slot.  moving: the camera also
    flies (a scripted path, as the keyboard camera of src/main.cpp:701-760 would move it)."""
    if moving:
        from real_time_ray_tracer_amd import aspect_for
        a = 0.03 * k
        h.camera_basis((0.5 * k, 0.1 * k, 14.0 - 0.5 * k), (0.0, 1.0, 0.0), (np.sin(a), -0.02 * k, np.cos(a)),
                       aspect_for(*CONFIGS["d"][:2]))
    if mode in (1, 2):
        h.fill_rand_buffer(7000 + k)
    else:
        h.moving_light(True)
    h.set_mode(frame, h.num_objects)


def gpu_render(cfg: str, frames: int, pipelined: bool = False, moving: bool = False) -> Renderer:
    W, H, S, spp, mode, _ = CONFIGS[cfg]
    h = config_header(cfg)
    r = Renderer(W, H, S, spp)
    if pipelined:
        r.enable_pipelining(True)
    f = 0
    for k in range(frames):
        advance(h, mode, k, f, moving)
        r.upload_header(h)
        f = r.dispatch(mode, f)
    r.synchronize()
    return r


def oracle_window(cfg: str, frames: int, x0: int, x1: int, y0: int, y1: int, moving: bool = False):
    """The oracle over columns [x0, x1) x rows [y0, y1) for the same frame sequence: image
    window [h][w][4] and the ring's window ([F][w][h][4] each: pixels, normals, depth)."""
    W, H, S, spp, mode, _ = CONFIGS[cfg]
    h = config_header(cfg)
    gy0, gy1 = max(0, y0 - 1), min(H, y1 + 1)
    gx0, gx1 = max(0, x0 - 1), min(W, x1 + 1)
    gh = gy1 - gy0
    d = oracle.dims(W, H, S, spp, gy0=gy0, gh=gh)
    buf = np.zeros(h.data.size + 3 * 8 * W * gh * 4, np.float32)
    img = np.zeros((gh, W, 4), np.float32)
    nt = oracle.nthreads_default()
    f = 0
    t0 = time.perf_counter()
    for k in range(frames):
        if k and (x1 - x0) * (y1 - y0) > 1 << 20:  # long oracle runs show progress (pytest -s)
            print(f"  oracle {cfg} [{x0},{x1})x[{y0},{y1}): frame {k}/{frames}, {time.perf_counter() - t0:.1f} s",
                  file=sys.stderr, flush=True)
        advance(h, mode, k, f, moving)
        buf[:h.data.size] = h.data
        for p in PROGS[mode]:
            if p in (oracle.AOP_COMPUTE, oracle.AO_COMPUTE):  # g-buffer writers: the halo too
                oracle.run_program(buf, d, p, f, img, gy0, gy1, nthreads=nt, x0=gx0, x1=gx1)
            else:
                oracle.run_program(buf, d, p, f, img, y0, y1, nthreads=nt, x0=x0, x1=x1)
        f = (f + 1) % 8
    o = h.data.size
    n = 8 * W * gh * 4
    ring = [buf[o + i * n:o + (i + 1) * n].reshape(8, W, gh, 4)[:, x0:x1, y0 - gy0:y1 - gy0] for i in range(3)]
    return img[y0 - gy0:y1 - gy0, x0:x1], ring


def pick_tiles(img: np.ndarray) -> dict:
    """Tile origins (x0, y0) chosen from the rendered image (row 0 = bottom row)."""
    H, W = img.shape[:2]
    tiles = {"corner_bl": (0, 0), "corner_br": (W - T, 0), "corner_tl": (0, H - T), "corner_tr": (W - T, H - T),
             "ground": (W // 2 - T // 2, H // 16)}
    lum = img[..., :3].sum(-1).astype(np.float64)
    gy, gx = H // T, W // T
    g = lum[:gy * T, :gx * T].reshape(gy, T, gx, T)
    std = g.std(axis=(1, 3))
    peak = g.max(axis=(1, 3))
    ex = np.abs(np.diff(lum, axis=1))[:gy * T, :gx * T - T].reshape(gy, T, gx - 1, T).sum(axis=(1, 3))
    upper = std.copy()
    upper[:gy // 2] = np.inf  # sky: the flattest tile of the upper half
    cand = {"sky": np.unravel_index(np.argmin(upper), upper.shape),
            "silhouette": np.unravel_index(np.argmax(ex), ex.shape),
            "brightest": np.unravel_index(np.argmax(peak), peak.shape)}
    for name, (ty, tx) in cand.items():
        tiles[name] = (int(tx) * T, int(ty) * T)
    return tiles


def check_window(r: Renderer, cfg: str, frames: int, x0: int, x1: int, y0: int, y1: int, what: str,
                 moving: bool = False):
    mode = CONFIGS[cfg][4]
    want_img, (wp, wn, wd) = oracle_window(cfg, frames, x0, x1, y0, y1, moving)
    g = r.download_rect(x0, x1, y0, y1)
    assert_close(g.image, want_img, f"{what} image")
    nf = min(frames, 8)
    assert_close(g.pixels[:nf], wp[:nf], f"{what} pixels")
    if mode in (1, 2):
        assert_bitwise(g.normals[:nf], wn[:nf], f"{what} normals")
        assert_bitwise(g.depth[:nf], wd[:nf], f"{what} depth")


def whole_frame_properties(img: np.ndarray, what: str) -> list:
    """Pixels (x, y) breaking "finite, non-negative, alpha 0"; the caller checks them against the
    oracle (the reference's own arithmetic can produce NaN, e.g. normalize(vec2(0)) in the
    jitter, ao_compute.glsl:310-323)."""
    with np.errstate(invalid="ignore"):
        bad = ~np.isfinite(img).all(-1) | (img[..., :3] < 0).any(-1) | (img[..., 3] != 0)
    ys, xs = np.nonzero(bad)
    return [(int(x), int(y)) for x, y in zip(xs[:4], ys[:4])]


@pytest.mark.parametrize("cfg,frames,pipelined", [
    ("d", 10, True),    # headline config, pipelined as the bench runs it; the ring wraps
    ("p", 10, False),   # (d) + a ground plane
    ("s1", 10, True),   # the reference's scene1 (4 spheres + plane) at 4K
    ("e", 2, False),    # 8K, 256 spheres, 64 spp
    ("c", 2, False),
    ("b", 3, False),    # Phong + reflections, moving light
])
def test_full_size_tiles(cfg, frames, pipelined):
    r = gpu_render(cfg, frames, pipelined)
    img = r.image()
    odd = whole_frame_properties(img, cfg)
    tiles = pick_tiles(img)
    W, H = CONFIGS[cfg][:2]
    for i, (x, y) in enumerate(odd):  # any non-finite / negative pixel is checked against the oracle
        tiles[f"odd{i}"] = (min(max(0, x - T // 2), W - T), min(max(0, y - T // 2), H - T))
    for name, (x0, y0) in tiles.items():
        check_window(r, cfg, frames, x0, x0 + T, y0, y0 + T, f"config {cfg} tile {name} at ({x0}, {y0})")
    r.close()


def test_full_size_tiles_moving_camera():
    """Config (d), pipelined, 10 frames with the camera flying: the temporal filter rejects
    history where the scene moved, at 4K pixel coordinates; the same tile choice as above."""
    r = gpu_render("d", 10, pipelined=True, moving=True)
    img = r.image()
    tiles = pick_tiles(img)
    W, H = CONFIGS["d"][:2]
    for i, (x, y) in enumerate(whole_frame_properties(img, "d")):
        tiles[f"odd{i}"] = (min(max(0, x - T // 2), W - T), min(max(0, y - T // 2), H - T))
    for name, (x0, y0) in tiles.items():
        check_window(r, "d", 10, x0, x0 + T, y0, y0 + T, f"config d (moving camera) tile {name} at ({x0}, {y0})",
                     moving=True)
    r.close()


def test_full_strip_config_d():
    """One full N = 8 strip (rows [1080, 1350) of 2160) at config (d), 10 pipelined frames."""
    r = gpu_render("d", 10, pipelined=True)
    W = CONFIGS["d"][0]
    check_window(r, "d", 10, 0, W, 1080, 1350, "config (d) strip 4 of 8")
    r.close()


@pytest.mark.timeout(900)
def test_full_strip_config_e():
    """Config (e), 7680x4320, 256 spheres, AO 64 spp: one full N = 8 strip, rows [2160, 2700)
    (540 rows: the strip of rank 4 of an equal 8-way split, through the horizon where ground,
    spheres and sky meet), over 10 frames: the ring wraps, so frames 8 and 9 overwrite slots 0
    and 1 and read their stale depth for emissive first hits.  The culls skip most of the
    reference's tests here (>128-sphere global split tails, bounce-ray clusters); the oracle
    runs the reference's brute-force scan."""
    r = gpu_render("e", 10)
    W = CONFIGS["e"][0]
    check_window(r, "e", 10, 0, W, 2160, 2700, "config (e) strip 4 of 8")
    r.close()


@pytest.mark.timeout(900)
@pytest.mark.parametrize("cfg,frames,pipelined", [
    ("b", 3, False),    # Phong + mirror bounces (<= 20), moving light (moving_light(true))
    ("c", 3, False),    # AO 16 spp, 64 spheres
    ("d", 10, True),    # the headline: AO 16 spp + post-process, pipelined, the ring wraps
    ("e", 2, False),    # 8K, 256 spheres, AO 64 spp (the ring wrap: test_full_strip_config_e)
])
def test_whole_frame(cfg, frames, pipelined):
    """The whole frame against the oracle: image, every ring slot's pixels (tolerance), and for
    the AO modes every slot's normals and depth bit for bit."""
    r = gpu_render(cfg, frames, pipelined)
    W, H = CONFIGS[cfg][:2]
    check_window(r, cfg, frames, 0, W, 0, H, f"config ({cfg}) whole frame")
    r.close()


def test_config_a_whole_frame():
    """Config (a), 640x480, 4 spheres, Phong (mode 3): the whole frame, 3 frames with the light
    moving (moving_light, src/main.cpp:541-551)."""
    r = gpu_render("a", 3)
    W, H = CONFIGS["a"][:2]
    assert not whole_frame_properties(r.image(), "a")
    check_window(r, "a", 3, 0, W, 0, H, "config (a) whole frame")
    r.close()
