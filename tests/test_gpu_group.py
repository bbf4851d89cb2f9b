"""Row strips through the C ABI (rt_group_*): one process drives G strip contexts and assembles
their image strips into one frame on the first device.  On the one-GPU box all strips share
device 0 (each with its own streams and g-buffer ring); with more devices visible the strips
also spread over them (xGMI peer copies).  Every assembled frame must equal a whole-frame
render (one rt_ctx, the reference's single glDispatchCompute(WIDTH, HEIGHT, 1),
src/main.cpp:604) bit for bit — strips are a partition of independent pixels plus a traced
1-row halo, so nothing may change."""
import subprocess
from pathlib import Path

import numpy as np
import pytest

from bench import CONFIGS, config_header
from conftest import assert_bitwise
from real_time_ray_tracer_amd import Header, Renderer, RtError, StripGroup, aspect_for

pytestmark = pytest.mark.gpu
ROOT = Path(__file__).resolve().parents[1]


def devices(g: int) -> list[int]:
    import torch

    n = max(1, torch.cuda.device_count())
    return [i % n for i in range(g)]


def whole_frames(W, H, h: Header, mode, frames, pipelined=False):
    r = Renderer(W, H, h.S, h.AA)
    if pipelined:
        r.enable_pipelining(True)
    f = r.compute_frames(h.copy(), mode, 0, frames, 7000, False)
    img = r.image()
    r.close()
    return img, f


def synth(W, H, objects, spp, seed=99):
    return Header.synthetic(objects, spp, seed, aspect_for(W, H))


@pytest.mark.parametrize("mode,spp,frames,pipelined", [(1, 4, 10, False), (1, 4, 10, True), (2, 4, 2, False),
                                                        (3, 1, 3, False), (4, 1, 3, False)])
@pytest.mark.parametrize("G", [2, 3])
def test_group_frames_equal_whole_frame(mode, spp, frames, pipelined, G):
    W, H = 200, 150
    h = synth(W, H, 24, spp)
    want, fw = whole_frames(W, H, h, mode, frames, pipelined)
    with StripGroup(W, H, h.S, h.AA, devices(G)) as g:
        if pipelined:
            g.enable_pipelining(True)
        hh = h.copy()
        f = g.compute_frames(hh, mode, 0, frames, 7000, False)
        assert f == fw
        assert_bitwise(g.image(), want, f"G={G} mode {mode}")


@pytest.mark.parametrize("pipelined,root", [(False, 0), (True, 0), (False, 2), (True, 1)])
def test_group_forced_copies_mixed_modes(pipelined, root):
    """The copy path of strips on other devices (rt_group_force_copies: every strip but the root
    strip renders into its own image and copies it into the frame), exercised on one GPU, with
    the root on the bottom strip (0) or another one (rt_group_set_plan's owner permutation).  The copy
    runs on the stream that wrote the strip's image: the output stream after a pipelined mode-1
    frame, the main stream after modes 2-4 (which pipelined contexts still run on their main
    stream), so frames switching modes must still assemble exactly."""
    W, H, spp = 160, 120, 4
    h = synth(W, H, 20, spp, seed=3)
    modes = [1, 2, 1, 3, 4, 1, 1, 2, 4, 3, 1]
    r = Renderer(W, H, h.S, h.AA)
    if pipelined:
        r.enable_pipelining(True)
    with StripGroup(W, H, h.S, h.AA, devices(3)) as g:
        if pipelined:
            g.enable_pipelining(True)
        g.force_copies(True)
        if root:
            g.set_plan([0, 37, 70, 120], root)
        assert g.root_strip() == root
        assert [g.strip_copies(i) for i in range(3)] == [i != root for i in range(3)]
        hr, hg = h.copy(), h.copy()
        fr = fg = 0
        for k, mode in enumerate(modes):
            for hh, f in ((hr, fr), (hg, fg)):
                if mode in (1, 2):
                    hh.fill_rand_buffer(7000 + k)
                else:
                    hh.moving_light(True)
                hh.set_mode(f, hh.num_objects)
            r.upload_header(hr)
            fr = r.dispatch(mode, fr)
            g.upload_header(hg)
            fg = g.dispatch(mode, fg)
            assert fr == fg
            assert_bitwise(g.image(), r.image(), f"frame {k} (mode {mode})")
        # and a burst of frames without a host round trip in between (the copies stay in flight)
        for mode, n in ((1, 9), (2, 3), (4, 3)):
            fr = r.compute_frames(hr, mode, fr, n, 9000, True)
            fg = g.compute_frames(hg, mode, fg, n, 9000, True)
            assert fr == fg
            assert_bitwise(g.image(), r.image(), f"burst of {n} mode-{mode} frames")
        g.force_copies(False)
        assert not g.strip_copies(1)
    r.close()


def test_group_balance_with_a_slow_link_gives_the_root_the_largest_strip():
    """rt_group_balance with the copy path and a stated slow link (rt_group_set_link_model): the
    gather-aware planner gives the root the strip with the most rows; the frames still equal the
    whole frame bit for bit."""
    W, H, spp = 320, 240, 4
    h = synth(W, H, 32, spp, seed=5)
    want, _ = whole_frames(W, H, h, 1, 10, pipelined=True)
    with StripGroup(W, H, h.S, h.AA, devices(4)) as g:
        g.enable_pipelining(True)
        g.force_copies(True)
        g.set_link_model(0.5, 1.0)
        assert g.link_model() == (0.5, 1.0)
        ms = g.balance(h, 1, rounds=3)
        b = g.bounds
        rows = [b[i + 1] - b[i] for i in range(4)]
        root = g.root_strip()
        assert rows[root] == max(rows), (b, root)
        assert [g.strip_copies(i) for i in range(4)] == [i != root for i in range(4)]
        assert len(ms) == 4 and all(t > 0 for t in ms)
        f = g.compute_frames(h.copy(), 1, 0, 10, 7000, False)
        assert f == 10 % 8
        assert_bitwise(g.image(), want, f"balanced strips, root strip {root}")
    # measured link model (no stated rates): the probe fills it in
    with StripGroup(W, H, h.S, h.AA, devices(3)) as g:
        g.force_copies(True)
        g.balance(h, 2, rounds=2)
        link, ingest = g.link_model()
        assert link > 0 and ingest > 0
        f = g.compute_frames(h.copy(), 2, 0, 2, 7000, False)
        want2, _ = whole_frames(W, H, h, 2, 2)
        assert_bitwise(g.image(), want2, "measured link model")


def test_group_dispatch_per_frame_and_uneven_bounds():
    """The per-frame calls (upload_header + dispatch), uneven strips including a 1-row strip,
    and a scene with a plane (the reference's scene1)."""
    W, H, spp = 160, 120, 4
    h = Header.builtin(1, spp, aspect_for(W, H))
    want, _ = whole_frames(W, H, h, 1, 9)
    bounds = [0, 1, 50, 119, 120]
    with StripGroup(W, H, h.S, h.AA, devices(4), bounds=bounds) as g:
        assert g.bounds == bounds
        hh = h.copy()
        f = 0
        for k in range(9):
            hh.fill_rand_buffer(7000 + k)
            hh.set_mode(f, hh.num_objects)
            g.upload_header(hh)
            f = g.dispatch(1, f)
        assert_bitwise(g.image(), want, "per-frame dispatch")


def test_group_balance_keeps_results():
    """rt_group_balance: the plan follows the cost (sky rows cheap), the strips restart with
    fresh rings, and the frames still equal the whole frame."""
    W, H, spp = 320, 240, 4
    h = synth(W, H, 32, spp, seed=5)
    want, _ = whole_frames(W, H, h, 1, 10, pipelined=True)
    with StripGroup(W, H, h.S, h.AA, devices(4)) as g:
        g.enable_pipelining(True)
        ms = g.balance(h, 1, rounds=2)
        b = g.bounds
        assert b[0] == 0 and b[-1] == H and all(b[i] < b[i + 1] for i in range(4))
        assert len(ms) == 4 and all(t > 0 for t in ms)
        f = g.compute_frames(h.copy(), 1, 0, 10, 7000, False)
        assert f == 10 % 8
        assert_bitwise(g.image(), want, "balanced strips")


def test_group_full_size_config_d_strips():
    """Config (d) at full size as 8 strips (the N = 8 partition), pipelined, 10 frames: the
    assembled frame equals the whole-frame render."""
    W, H, S, spp, mode, _ = CONFIGS["d"]
    h = config_header("d")
    want, _ = whole_frames(W, H, h, mode, 10, pipelined=True)
    with StripGroup(W, H, S, spp, devices(8)) as g:
        g.enable_pipelining(True)
        g.compute_frames(h.copy(), mode, 0, 10, 7000, False)
        assert_bitwise(g.image(), want, "config (d), 8 strips")


def test_group_frame_into_caller_buffer():
    import torch

    W, H, spp = 96, 64, 4
    h = synth(W, H, 12, spp)
    want, _ = whole_frames(W, H, h, 2, 2)
    buf = torch.zeros((H, W, 4), dtype=torch.float32, device="cuda:0")
    with StripGroup(W, H, h.S, h.AA, devices(3)) as g:
        g.bind_frame(buf.data_ptr())
        assert g.frame_device_ptr() == buf.data_ptr()
        g.compute_frames(h.copy(), 2, 0, 2, 7000, False)
        g.synchronize()
        assert_bitwise(buf.cpu().numpy(), want, "caller frame buffer")


def test_group_errors():
    W, H = 64, 48
    h = synth(W, H, 8, 4)
    with pytest.raises(RtError):
        StripGroup(W, H, h.S, h.AA, devices(2), bounds=[0, 30, 30])  # empty strip
    with pytest.raises(RtError):
        StripGroup(W, H, h.S, h.AA, [0, 99])  # no such device
    with StripGroup(W, H, h.S, h.AA, devices(2)) as g:
        with pytest.raises(RtError):
            g.dispatch(1, 0)  # no header yet
        g.upload_header(h)
        with pytest.raises(RtError):
            g.dispatch(7, 0)
        with pytest.raises(RtError):
            g.set_bounds([0, 48, 48])


def test_headless_refuses_missing_devices():
    """rt_headless --devices naming a device that is not visible stops with a message."""
    exe = ROOT / "build" / "rt_headless"
    import torch

    n = torch.cuda.device_count()
    p = subprocess.run([str(exe), "--width", "64", "--height", "48", "--strips", "2", "--devices", f"0,{n}"],
                       capture_output=True, text=True, timeout=120)
    assert p.returncode == 1
    assert f"names device {n}" in p.stderr


def test_headless_strips_ppm_equals_whole_frame(tmp_path):
    """build/rt_headless --strips G (the reference's render loop as a C++ program over the
    rt_group_* entry points) writes the same PPM as the whole-frame run."""
    exe = ROOT / "build" / "rt_headless"
    assert exe.exists(), "make headless"
    outs = []
    for extra in ([], ["--strips", "4", "--balance", "1"], ["--strips", "3", "--pipeline", "1"]):
        out = tmp_path / f"f{len(outs)}.ppm"
        p = subprocess.run([str(exe), "--width", "240", "--height", "180", "--frames", "9", "--mode", "1",
                            "--ppm", str(out)] + extra, capture_output=True, text=True, timeout=300)
        assert p.returncode == 0, p.stderr
        outs.append(out.read_bytes())
    assert outs[0] == outs[1] == outs[2]
