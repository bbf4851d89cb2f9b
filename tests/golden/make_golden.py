#!/usr/bin/env python
"""Generate the golden fixtures tests/golden/*.npz.  TEST INFRASTRUCTURE.

Each fixture is one small frame sequence: the SSBO header (scene, camera, light, background)
and per-frame rand_buffer seeds are the inputs; the outputs are the final image and the
touched g-buffer ring slots (reference [F][W][H] layout).  Produced by the C oracle
(oracle/rt_oracle.c) and, before being written, cross-checked against the independent numpy
restatement (oracle/numpy_ref.py).  The reference itself cannot run here (OpenGL compute;
SURVEY.md §8c), so these are self-generated vectors: parity unpinned by reference artifacts.

    python tests/golden/make_golden.py
"""
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))

import oracle  # noqa: E402
from oracle import numpy_ref  # noqa: E402
from real_time_ray_tracer_amd import SSBO, Header, aspect_for  # noqa: E402

W, H = 48, 32
CASES = [
    # name, scene, spp, mode, frames
    ("scene1_mode1", "s1", 4, 1, 3),
    ("scene1_mode2", "s1", 4, 2, 2),
    ("scene1_mode3", "s1", 4, 3, 1),
    ("scene1_mode4", "s1", 4, 4, 1),
    ("scene6_mode1", "s6", 4, 1, 3),
    ("syn16_mode1", "syn16", 16, 1, 3),
    ("syn16_mode4", "syn16", 1, 4, 1),
    ("planes_mode2", "planes", 4, 2, 2),
]


def scene(name, spp):
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


def run(h0, mode, frames, impl):
    s = SSBO(h0, W, H)
    img = np.zeros((H, W, 4), np.float32)
    d = oracle.dims(W, H, h0.S, h0.AA)
    f = 0
    for k in range(frames):
        h = h0.copy()
        h.fill_rand_buffer(7000 + k)
        h.set_mode(f, h.num_objects)
        s.set_header(h)
        if impl == "c":
            f = oracle.dispatch(s.data, d, mode, f, img, nthreads=4)
        else:
            f = numpy_ref.dispatch(s.data, W, H, h.S, h.AA, mode, f, img)
    return s, img


def main():
    out = Path(__file__).resolve().parent
    for name, sc, spp, mode, frames in CASES:
        h0 = scene(sc, spp)
        s, img = run(h0, mode, frames, "c")
        sn, imgn = run(h0, mode, frames, "numpy")
        ok = np.abs(img - imgn) <= 1e-4 * np.maximum(np.abs(img), np.abs(imgn)) + 1e-6
        assert ok.all(), f"{name}: C oracle and numpy restatement disagree"
        assert np.array_equal(s.depth.view(np.uint32), sn.depth.view(np.uint32)), name
        np.savez_compressed(out / f"{name}.npz", header=h0.data, S=h0.S, spp=spp, mode=mode, frames=frames,
                            width=W, height=H, seed0=7000, image=img,
                            pixels=s.pixels[:frames], normals=s.normals[:frames], depth=s.depth[:frames])
        print(f"{name}: image mean {img[..., :3].mean():.4f}")


if __name__ == "__main__":
    main()
