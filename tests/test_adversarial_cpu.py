"""The adversarial scenes (tests/adversarial_scenes.py) really contain the geometry they claim,
checked in the oracle's float semantics on the CPU; the GPU parity on them is
tests/test_gpu_adversarial.py."""
import numpy as np
import pytest

import oracle
from adversarial_scenes import CAM, NAMES, _ray, scene


def spheres(h):
    sh = h.shapes[:h.num_objects]
    return [(i, sh[i, 0, :3], float(sh[i, 0, 3])) for i in range(h.num_objects) if int(sh[i, 4, 3]) == 1]


@pytest.mark.parametrize("W,H", [(64, 48), (3840, 2160)])
def test_tangent_rays_have_zero_discriminant(W, H):
    h, pix = scene("tangent", W, H, 4)
    for k, (x, y) in enumerate(pix):
        d = _ray(h, W, H, x, y)
        c = h.shapes[12 + k, 0]
        assert oracle.sphere_del(CAM, d, c[:3], c[3]) == 0.0
        # the reference's del == 0 branch: t = -b, a positive hit in front of the camera
        assert oracle.sphere_eval(CAM, d, c[:3], c[3]) > 1.0


def test_camera_and_light_inside():
    h, _ = scene("cam_inside", 64, 48, 4)
    inside = [i for i, c, r in spheres(h) if np.linalg.norm(CAM - c) < r]
    assert inside == [2]
    h, _ = scene("huge", 64, 48, 4)
    assert [i for i, c, r in spheres(h) if np.linalg.norm(CAM - c) < r] == [17]
    h, _ = scene("light_inside", 64, 48, 4)
    L = h.vec4(5)[:3]
    for frames in range(4):  # moving_light(+0.1 per frame) keeps it inside for the tests' frames
        Lk = L + 0.1 * frames
        assert [i for i, c, r in spheres(h) if np.linalg.norm(Lk - c) < r] == [16]


def test_straddle_geometry():
    h, _ = scene("straddle", 64, 48, 4)
    s = {i: (c, r) for i, c, r in spheres(h)}
    for i in (16, 18):  # the camera plane z = 14 cuts these spheres
        c, r = s[i]
        assert abs(c[2] - CAM[2]) < r and np.linalg.norm(c - CAM) > r
    for i in (17, 19):  # entirely behind the camera (it looks down -z)
        c, r = s[i]
        assert c[2] - r > CAM[2]


@pytest.mark.parametrize("name", NAMES)
def test_oracle_renders_every_scene(name):
    """Every scene renders in every mode on the oracle (small frame) with the features visible
    where claimed: finite pixels apart from the reference's own NaN cases."""
    W, H = 32, 24
    for mode in (1, 2, 3, 4):
        h, _ = scene(name, W, H, 4)
        from real_time_ray_tracer_amd import SSBO
        s = SSBO(h, W, H)
        d = oracle.dims(W, H, h.S, h.AA)
        img = np.zeros((H, W, 4), np.float32)
        oracle.dispatch(s.data, d, mode, 0, img)
        assert np.isfinite(img).mean() > 0.99, f"{name} mode {mode}"
