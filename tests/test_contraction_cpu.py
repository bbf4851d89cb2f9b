"""The hash's contraction contract, on the CPU.

random() (ao_compute.glsl:63-73) multiplies sin(dot(st, (12.9898, 78.233))) by 43758.5 before
fract(), so every rounding of its argument is amplified into a different sample.  Three places
are the compiler's choice in the GLSL: the dot() inside random() (fused here), the hemisphere
seed sums (ao_compute.glsl:152-157, unfused here) and the anti-aliasing jitter seed sums
(ao_compute.glsl:317-319, unfused here).  A re-execution reproduces this build's frames only if it
makes the same three choices (and computes the correctly rounded sin, tests/test_sin_cpu.py).
These tests pin that: the goldens are reproduced by the build's variant and by no other, and the
numpy restatement, in each variant, agrees with the C oracle in the same variant (its literal,
unfused dot() is written independently of the oracle's)."""
import numpy as np
import pytest

import oracle
from conftest import assert_bitwise, assert_close
from oracle import numpy_ref
from real_time_ray_tracer_amd import SSBO, Header, aspect_for

from test_golden import GOLDEN, load

AO_GOLDEN = [p for p in GOLDEN if "mode1" in p.stem or "mode2" in p.stem]


def _close(a, b):
    return np.abs(a - b) <= 1e-4 * np.maximum(np.abs(a), np.abs(b)) + 1e-6


def _oracle_frames(g, flags):
    W, H = int(g["width"]), int(g["height"])
    h0 = Header(int(g["S"]), int(g["spp"]), g["header"])
    s = SSBO(h0, W, H)
    d = oracle.dims(W, H, h0.S, h0.AA)
    img = np.zeros((H, W, 4), np.float32)
    f = 0
    oracle.set_contraction(flags)
    try:
        for k in range(int(g["frames"])):
            h = h0.copy()
            h.fill_rand_buffer(int(g["seed0"]) + k)
            h.set_mode(f, h.num_objects)
            s.set_header(h)
            f = oracle.dispatch(s.data, d, int(g["mode"]), f, img, nthreads=2)
    finally:
        oracle.set_contraction(0)
    return img, s


@pytest.mark.parametrize("path", AO_GOLDEN, ids=[p.stem for p in AO_GOLDEN])
def test_only_the_build_variant_reproduces_the_goldens(path):
    g = load(path)
    n = int(g["frames"])
    fractions = {}
    for flags in (0, oracle.C_UNFUSED_DOT, oracle.C_FUSED_SEEDS, oracle.C_FUSED_JITTER):
        img, s = _oracle_frames(g, flags)
        fractions[flags] = float(_close(img[..., :3], g["image"][..., :3]).mean())
        same = np.array_equal(s.depth[:n].view(np.uint32), g["depth"].view(np.uint32))
        if flags == 0:
            assert fractions[0] == 1.0 and same
    print(f"\n{path.stem}: image channels within 1e-4 of the golden per variant {fractions}")
    # the unfused dot and the fused hemisphere seeds move many samples; the fused jitter seeds
    # move the anti-aliased primary rays (spp > 1), fewer but still visible
    assert fractions[oracle.C_UNFUSED_DOT] < 0.95 and fractions[oracle.C_FUSED_SEEDS] < 0.95
    if int(g["spp"]) > 1:
        assert fractions[oracle.C_FUSED_JITTER] < 1.0
    assert oracle.get_contraction() == 0


@pytest.mark.parametrize("flags", [0, 1, 2, 4, 7])
@pytest.mark.parametrize("mode", [1, 2])
def test_numpy_restatement_matches_oracle_per_variant(flags, mode):
    """numpy_ref.CONTRACTION = flags against oracle.set_contraction(flags) on a small AO frame
    sequence: the same variant gives the same frames (image within tolerance, normals and depth
    bit for bit), so the cross-check is independent on this axis too."""
    W, H, spp, frames = 20, 14, 4, 2
    h0 = Header.synthetic(10, spp, 321, aspect_for(W, H))
    outs = []
    for which in ("oracle", "numpy"):
        s = SSBO(h0.copy(), W, H)
        d = oracle.dims(W, H, h0.S, h0.AA)
        img = np.zeros((H, W, 4), np.float32)
        f = 0
        old = numpy_ref.CONTRACTION
        oracle.set_contraction(flags)
        numpy_ref.CONTRACTION = flags
        try:
            for k in range(frames):
                h = h0.copy()
                h.fill_rand_buffer(7000 + k)
                h.set_mode(f, h.num_objects)
                s.set_header(h)
                if which == "oracle":
                    f = oracle.dispatch(s.data, d, mode, f, img, nthreads=2)
                else:
                    f = numpy_ref.dispatch(s.data, W, H, h.S, h.AA, mode, f, img)
        finally:
            oracle.set_contraction(0)
            numpy_ref.CONTRACTION = old
        outs.append((img, s.normals[:frames].copy(), s.depth[:frames].copy()))
    (ia, na, da), (ib, nb, db) = outs
    assert_close(ib, ia, f"variant {flags} mode {mode} image")
    assert_bitwise(nb, na, f"variant {flags} mode {mode} normals")
    assert_bitwise(db, da, f"variant {flags} mode {mode} depth")
