"""Mode 4's longest-first tile schedule (rt_set_tile_schedule, rt_shim HySched): the workgroups
of h_compute's dispatch (src/main.cpp:604, resources/h_compute.glsl) run their 16x16 tiles in the
order of the bounce rounds recent frames needed.  Only the order changes: the frames rendered
with the schedule in use equal those rendered in row order bit for bit, and the last one equals
the CPU oracle's frame (config (b), the whole 1920x1080 frame)."""
import numpy as np
import pytest

import oracle
from bench import CONFIGS, config_header
from conftest import assert_close
from real_time_ray_tracer_amd import Renderer

pytestmark = pytest.mark.gpu


def render(cfg, frames, schedule, until_active=False):
    W, H, S, spp, mode, _ = CONFIGS[cfg]
    h = config_header(cfg)
    r = Renderer(W, H, S, spp)
    r.set_tile_schedule(schedule)
    f = 0
    k = 0
    active_at = None
    while k < frames or (until_active and active_at is None and k < 400):
        h.moving_light(True)
        h.set_mode(f, h.num_objects)
        r.upload_header(h)
        f = r.dispatch(mode, f)
        k += 1
        if until_active and active_at is None and r.tile_schedule_state() == 2:
            active_at = k
            frames = k + 3  # three more frames with the longest-first order in use
    r.synchronize()
    img = r.image()
    pix = r.download(normals=False, depth=False, image=False).pixels
    state = r.tile_schedule_state()
    r.close()
    return k, h, img, pix, state, active_at


def test_tile_schedule_engages_and_keeps_every_pixel():
    k, h, img, pix, state, active_at = render("b", 2, True, until_active=True)
    assert state == 2 and active_at is not None, "the longest-first order never came into use"
    # the same frames in row order: bit-identical images and ring
    k2, _, img2, pix2, state2, _ = render("b", k, False)
    assert k2 == k and state2 == 0
    assert np.array_equal(img.view(np.uint32), img2.view(np.uint32))
    assert np.array_equal(pix.view(np.uint32), pix2.view(np.uint32))
    # and the last frame equals the oracle's (h holds the header the last frame used)
    W, H, S, spp, mode, _ = CONFIGS["b"]
    d = oracle.dims(W, H, S, spp)
    buf = np.zeros(h.data.size + 3 * 8 * W * H * 4, np.float32)
    buf[:h.data.size] = h.data
    want = np.zeros((H, W, 4), np.float32)
    f_last = (k - 1) % 8
    oracle.run_program(buf, d, oracle.H_COMPUTE, f_last, want, 0, H, nthreads=oracle.nthreads_default())
    assert_close(img, want, "scheduled frame image")


def test_tile_schedule_off_and_on_again():
    W, H, S, spp, mode, _ = CONFIGS["b"]
    h = config_header("b")
    r = Renderer(W, H, S, spp)
    assert r.tile_schedule_state() == 1
    r.set_tile_schedule(False)
    assert r.tile_schedule_state() == 0
    r.set_tile_schedule(True)
    f = 0
    for _ in range(40):
        h.moving_light(True)
        h.set_mode(f, h.num_objects)
        r.upload_header(h)
        f = r.dispatch(mode, f)
    r.synchronize()
    assert r.tile_schedule_state() in (1, 2)
    r.close()



def test_tile_schedule_survives_a_stream_change():
    """rt_set_stream after the order is in use (the context's own stream is released): later
    frames, with the schedule still engaged, equal the same frames rendered in row order."""
    import torch

    W, H, S, spp, mode, _ = CONFIGS["b"]

    def run(schedule):
        h = config_header("b")
        r = Renderer(W, H, S, spp)
        r.set_tile_schedule(schedule)
        f = 0
        for k in range(60):
            if k == 30:
                r.synchronize()
                st = torch.cuda.Stream()
                r.set_stream(st)
            h.moving_light(True)
            h.set_mode(f, h.num_objects)
            r.upload_header(h)
            f = r.dispatch(mode, f)
        r.synchronize()
        img, state = r.image(), r.tile_schedule_state()
        r.close()
        return img, state

    img, state = run(True)
    img2, state2 = run(False)
    assert state == 2 and state2 == 0
    assert np.array_equal(img.view(np.uint32), img2.view(np.uint32))


def _two_poses():
    """config (b) from its own camera and from a camera moved 6 units left and turned: the
    mirror-bouncing tiles move, so the longest-first order changes with the pose"""
    W, H, S, spp, mode, _ = CONFIGS["b"]
    a = config_header("b")
    b = a.copy()
    b.camera_basis((-6.0, 1.0, 14.0), (0.0, 1.0, 0.0), (0.3, 0.0, 1.0), W / H)
    return a, b


def test_tile_schedule_order_swaps_keep_every_pixel():
    """several order swaps in one run (the pose alternates every 32 frames), each
    replacing the table that launches in flight may still read (ev_use / used_on): every 8th
    frame's image and the final ring equal row order's bit for bit."""
    W, H, S, spp, mode, _ = CONFIGS["b"]

    def run(schedule):
        a, b = _two_poses()
        r = Renderer(W, H, S, spp)
        r.set_tile_schedule(schedule)
        f, imgs = 0, []
        for k in range(224):
            h = a if (k // 32) % 2 == 0 else b
            h.moving_light(True)
            h.set_mode(f, h.num_objects)
            r.upload_header(h)
            f = r.dispatch(mode, f)
            if k % 8 == 7:
                imgs.append(r.image())
        pix = r.download(normals=False, depth=False, image=False).pixels
        orders, state = r.tile_schedule_orders(), r.tile_schedule_state()
        r.close()
        return imgs, pix, orders, state

    imgs, pix, orders, state = run(True)
    imgs2, pix2, orders2, state2 = run(False)
    print(f"orders taken up: {orders}")
    assert state == 2 and orders >= 3, (state, orders)
    assert state2 == 0 and orders2 == 0
    for i, (x, y) in enumerate(zip(imgs, imgs2)):
        assert np.array_equal(x.view(np.uint32), y.view(np.uint32)), f"image after frame {8 * i + 7}"
    assert np.array_equal(pix.view(np.uint32), pix2.view(np.uint32))


def test_tile_schedule_with_multi_frame_launches():
    """mode-4 launches of up to 32 frames (rt_set_frame_batch, rt_compute_frames) with
    the schedule on, where every z-block of a launch writes the same cost slots: the ring and the
    image equal row order's bit for bit."""
    W, H, S, spp, mode, _ = CONFIGS["b"]

    def run(schedule):
        a, b = _two_poses()
        r = Renderer(W, H, S, spp)
        r.set_tile_schedule(schedule)
        r.set_frame_batch(32)
        f = 0
        for k in range(12):
            f = r.compute_frames(a if k % 4 < 2 else b, mode, f, 24, 7000, True)
        r.synchronize()
        g = r.download(normals=False, depth=False)
        orders = r.tile_schedule_orders()
        r.close()
        return g, f, orders

    g, f, orders = run(True)
    g2, f2, _ = run(False)
    print(f"orders taken up: {orders}")
    assert f == f2
    assert np.array_equal(g.image.view(np.uint32), g2.image.view(np.uint32))
    assert np.array_equal(g.pixels.view(np.uint32), g2.pixels.view(np.uint32))
