"""Golden fixtures (tests/golden/*.npz, made by tests/golden/make_golden.py): the CPU oracle
and — on a GPU — the HIP path must reproduce them.  Normals/depth bit for bit, pixels and
image within the north-star tolerance."""
from pathlib import Path

import numpy as np
import pytest

import oracle
from conftest import assert_bitwise, assert_close
from real_time_ray_tracer_amd import SSBO, Header

GOLDEN = sorted((Path(__file__).resolve().parent / "golden").glob("*.npz"))


def load(p):
    z = np.load(p)  # allow_pickle=False (default): data only
    return {k: z[k] for k in z.files}


def check(g, pixels, normals, depth, image, what):
    n = int(g["frames"])
    assert_close(image, g["image"], f"{what} image")
    assert_close(pixels[:n], g["pixels"], f"{what} pixels")
    assert_bitwise(normals[:n], g["normals"], f"{what} normals")
    assert_bitwise(depth[:n], g["depth"], f"{what} depth")


def test_fixtures_present():
    assert len(GOLDEN) >= 8


@pytest.mark.parametrize("path", GOLDEN, ids=[p.stem for p in GOLDEN])
def test_oracle_reproduces_golden(path):
    g = load(path)
    W, H = int(g["width"]), int(g["height"])
    h0 = Header(int(g["S"]), int(g["spp"]), g["header"])
    s = SSBO(h0, W, H)
    d = oracle.dims(W, H, h0.S, h0.AA)
    img = np.zeros((H, W, 4), np.float32)
    f = 0
    for k in range(int(g["frames"])):
        h = h0.copy()
        h.fill_rand_buffer(int(g["seed0"]) + k)
        h.set_mode(f, h.num_objects)
        s.set_header(h)
        f = oracle.dispatch(s.data, d, int(g["mode"]), f, img, nthreads=2)
    check(g, s.pixels, s.normals, s.depth, img, path.stem)


@pytest.mark.gpu
@pytest.mark.parametrize("path", GOLDEN, ids=[p.stem for p in GOLDEN])
def test_gpu_reproduces_golden(path):
    from real_time_ray_tracer_amd import Renderer

    g = load(path)
    W, H = int(g["width"]), int(g["height"])
    h0 = Header(int(g["S"]), int(g["spp"]), g["header"])
    r = Renderer(W, H, h0.S, h0.AA)
    f = 0
    for k in range(int(g["frames"])):
        h = h0.copy()
        h.fill_rand_buffer(int(g["seed0"]) + k)
        h.set_mode(f, h.num_objects)
        r.upload_header(h)
        f = r.dispatch(int(g["mode"]), f)
    gb = r.download()
    r.close()
    check(g, gb.pixels, gb.normals, gb.depth, gb.image, path.stem)
