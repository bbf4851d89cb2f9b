"""Stream plumbing: a renderer ordered on torch's stream (the default NULL stream, or a
side stream) and rendering into a torch tensor must be visible to torch work enqueued after
it with no extra synchronisation — the contract the pipelined RCCL gather relies on."""
import numpy as np
import pytest

from real_time_ray_tracer_amd import Header, Renderer, aspect_for

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("side_stream", [False, True])
def test_render_into_torch_tensor_on_torch_stream(side_stream):
    import torch

    W, H = 96, 64
    h = Header.synthetic(12, 4, 5, aspect_for(W, H))
    dev = torch.device("cuda", 0)
    s = torch.cuda.Stream(dev) if side_stream else torch.cuda.default_stream(dev)
    with torch.cuda.stream(s):
        r = Renderer(W, H, h.S, h.AA, rows=(16, 48))
        r.set_stream(torch.cuda.current_stream(dev))
        img = torch.full((32, W, 4), -7.0, dtype=torch.float32, device=dev)
        r.bind_image(img.data_ptr())
        f = 0
        for k in range(3):
            h.fill_rand_buffer(7000 + k)
            h.set_mode(f, h.num_objects)
            r.upload_header(h)
            f = r.dispatch(1, f)
            got = img.cpu().numpy()  # ordered after the render on the same stream
            assert (got != -7.0).all(), "torch saw the tensor before the render wrote it"
            img.fill_(-7.0)
        # own-buffer render of the same last frame must equal what torch read
        r2 = Renderer(W, H, h.S, h.AA, rows=(16, 48))
        f2 = 0
        for k in range(3):
            h.fill_rand_buffer(7000 + k)
            h.set_mode(f2, h.num_objects)
            r2.upload_header(h)
            f2 = r2.dispatch(1, f2)
        np.testing.assert_array_equal(got.view(np.uint32), r2.image().view(np.uint32))
        r.close()
        r2.close()


@pytest.mark.parametrize("pipeline", ["0", "1"])
def test_c_headless_driver_renders(tmp_path, pipeline):
    """The C++ frame driver over the C ABI (the reference's render loop without GL): several
    mode-1 frames, then the PPM image in place of the GL blit."""
    import subprocess
    from pathlib import Path

    root = Path(__file__).resolve().parents[1]
    exe = root / "build" / "rt_headless"
    if not exe.exists():
        subprocess.run(["make", "-C", str(root), "headless"], check=True, capture_output=True)
    out = tmp_path / "frame.ppm"
    p = subprocess.run([str(exe), "--width", "160", "--height", "120", "--frames", "10", "--mode", "1",
                        "--pipeline", pipeline, "--ppm", str(out)], capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr
    assert "ms/frame" in p.stdout
    data = out.read_bytes()
    assert data.startswith(b"P6\n160 120\n255\n") and len(data) == len(b"P6\n160 120\n255\n") + 160 * 120 * 3
    assert len(set(data[16:])) > 8  # not a blank frame
