"""Pipelined mode 1 (rt_enable_pipelining): frame k's post-process on a second stream while
frame k+1's AO pass runs.  The ring rotates normals/depth/raw pixels through spare buffers,
so the results must equal the sequential order bit for bit: images, pixels, normals and depth
(including the stale normal/depth of pixels whose sample 0 first hits an emissive sphere),
across ring wraps, mode switches, row strips and a torch output stream."""
import numpy as np
import pytest

from conftest import assert_bitwise
from real_time_ray_tracer_amd import Header, Renderer, aspect_for

pytestmark = pytest.mark.gpu


def _frames(r, h, modes, seed0=7000):
    f = 0
    imgs = []
    for k, mode in enumerate(modes):
        h.fill_rand_buffer(seed0 + k)
        h.set_mode(f, h.num_objects)
        r.upload_header(h)
        f = r.dispatch(mode, f)
        if k in (8, 15):
            imgs.append(r.image())
    imgs.append(r.image())
    return imgs, r.download(True, True, True, False)


@pytest.mark.parametrize("rows", [None, (10, 37)])
@pytest.mark.parametrize("modes", [[1] * 21, [1] * 5 + [2, 2] + [1] * 9 + [3] + [1] * 4])
def test_pipelined_equals_sequential(rows, modes):
    W, H, spp = 96, 64, 4
    h = Header.synthetic(40, spp, 99, aspect_for(W, H))  # 1/16 emissive spheres: stale path
    kw = {} if rows is None else {"rows": rows}
    a = Renderer(W, H, h.S, spp, **kw)
    want_imgs, want = _frames(a, h.copy(), modes)
    b = Renderer(W, H, h.S, spp, **kw)
    b.enable_pipelining(True)
    got_imgs, got = _frames(b, h.copy(), modes)
    for i, (g, w) in enumerate(zip(got_imgs, want_imgs)):
        assert_bitwise(g, w, f"image {i}")
    for name in ("pixels", "normals", "depth"):
        assert_bitwise(getattr(got, name), getattr(want, name), name)
    a.close()
    b.close()


def test_pipelined_full_size_with_torch_output_stream():
    """Config (d) size, 10 frames, output on a torch stream; the image is read on that stream."""
    import torch

    from bench import CONFIG_INDEX, CONFIGS

    W, H, S, spp, mode, _ = CONFIGS["d"]
    h = Header.synthetic(S, spp, 1234 + CONFIG_INDEX["d"], aspect_for(W, H))
    dev = torch.device("cuda", 0)
    main, out = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    a = Renderer(W, H, S, spp)
    b = Renderer(W, H, S, spp)
    b.set_stream(main)
    b.enable_pipelining(True, out)
    img = torch.zeros((H, W, 4), dtype=torch.float32, device=dev)
    b.bind_image(img.data_ptr())
    fa = fb = 0
    for k in range(10):
        h.fill_rand_buffer(7000 + k)
        for r, f in ((a, fa), (b, fb)):
            h.set_mode(f, S)
            r.upload_header(h)
        fa = a.dispatch(1, fa)
        fb = b.dispatch(1, fb)
    with torch.cuda.stream(out):
        got = img.cpu().numpy()
    assert_bitwise(got, a.image(), "image on the output stream")
    ga, gb = a.download(True, True, True, False), b.download(True, True, True, False)
    for name in ("pixels", "normals", "depth"):
        assert_bitwise(getattr(gb, name), getattr(ga, name), name)
    a.close()
    b.close()
