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
