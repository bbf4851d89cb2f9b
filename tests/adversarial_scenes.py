"""Adversarial scenes for the cone-culled kernels (test infrastructure).

The production kernels skip ray-sphere tests on conservative cone/ball proofs (DESIGN.md §5:
the pool cone of the camera rays, the first-bounce cone, the per-ray pre-test, the shadow
cone).  The synthetic BASELINE scenes keep every sphere outside and in front of the camera,
so these scenes put geometry exactly where those proofs have their margins:

  cam_inside      the camera inside a sphere (p_compute.glsl:99-106, the t1 branch), with
                  spheres inside it too: every first-bounce origin lies inside a sphere
  straddle        spheres straddling the camera plane, entirely behind the camera, and
                  behind it on the line of sight (reached by mirror / AO bounces only)
  tangent         primary rays exactly tangent to spheres: the computed discriminant is
                  0.0f (p_compute.glsl:92-95), constructed by an ulp search on the centre
  huge            radius-1e4 spheres: config q's ground and an emissive sky dome that
                  contains the camera and the whole scene
  tiny_far        radius-1e-3 spheres at distance ~1e3, centred on chosen pixels' rays
  overlap         duplicate spheres (the lower index must win every tie), overlapping and
                  concentric spheres, a touching pair
  light_inside    the light inside a sphere (the shadow cone's apex is enclosed)
  adv256          256 spheres (past the 128-object LDS tables) carrying these features

scene(name, W, H, spp) -> (Header, [(x, y) pixels of interest]).  The pixels of interest are
where a constructed feature shows (tangent pixels, tiny spheres); the full-size tests check
tiles around them.
"""
from __future__ import annotations

import numpy as np

import oracle
from real_time_ray_tracer_amd import Header, aspect_for

NAMES = ["cam_inside", "straddle", "tangent", "huge", "tiny_far", "overlap", "light_inside", "adv256"]

CAM = np.array([0.0, 0.0, 14.0], np.float32)  # src/main.cpp:98


def _syn(n: int, spp: int, W: int, H: int, S: int) -> Header:
    return Header.synthetic(n, spp, 1234, aspect_for(W, H), num_shapes=S)


def _ray(h: Header, W: int, H: int, x: int, y: int) -> np.ndarray:
    """The unjittered camera ray of pixel (x, y): sample 0 of the AO modes, every Phong ray."""
    hp = np.float32(x) / np.float32(W)
    vp = np.float32(y) / np.float32(H)
    return oracle.primary_dir(h.data, hp, vp)


def tangent_center(d: np.ndarray, dist: float, r: float, seed: int, origin=CAM) -> np.ndarray:
    """A sphere centre for which the ray (origin, d) has discriminant exactly 0.0f: start with
    the line at distance r from the centre and walk the centre's float bits at random until
    fmaf(r, r, fmaf(b, b, -dot(pmc, pmc))) == 0 (r*r must be exact: r with few bits)."""
    up = np.array([0.0, 1.0, 0.0])
    perp = np.cross(d.astype(np.float64), up)
    perp /= np.linalg.norm(perp)
    c0 = (origin.astype(np.float64) + dist * d.astype(np.float64) + r * perp).astype(np.float32)
    rng = np.random.default_rng(seed)
    for _ in range(200000):
        c = (c0.view(np.int32) + rng.integers(-64, 65, 3).astype(np.int32)).view(np.float32)
        if oracle.sphere_del(origin, d, c, r) == 0.0:
            return c
    raise RuntimeError("no exactly tangent centre found")


def _cam_inside(W, H, spp):
    h = _syn(1, spp, W, H, 8)
    h.pack_sphere(1, (0.0, 0.0, 11.0), 0.8, (0.8, 0.3, 0.3))
    h.pack_sphere(2, (0.4, -0.3, 12.5), 4.0, (0.7, 0.7, 0.9))              # encloses the camera
    h.pack_sphere(3, (-1.2, 0.6, 11.2), 0.35, (3.0, 3.0, 3.0), emissive=True)
    h.pack_sphere(4, (1.3, -0.7, 10.5), 0.7, (0.9, 0.9, 0.9), reflectivity=0.0)  # mirror
    h.pack_sphere(5, (0.2, 1.2, 10.0), 0.5, (0.2, 0.8, 0.4), reflectivity=0.3)   # glossy
    h.pack_sphere(6, (-0.9, -1.1, 12.0), 0.6, (0.5, 0.5, 0.1), reflectivity=0.6)
    h.pack_sphere(7, (0.0, 0.0, 11.0), 0.8, (0.1, 0.1, 0.9))               # duplicate of 1
    h.set_mode(0, 8)
    return h, [(W // 2, H // 2)]


def _straddle(W, H, spp):
    h = _syn(16, spp, W, H, 21)
    h.pack_sphere(16, (-2.0, 0.0, 14.0), 1.5, (0.9, 0.5, 0.2))              # straddles the camera plane
    h.pack_sphere(17, (0.0, 0.0, 20.0), 3.0, (0.9, 0.9, 0.2))               # entirely behind
    h.pack_sphere(18, (2.6, 1.2, 15.0), 2.0, (0.9, 0.9, 0.9), reflectivity=0.0)  # straddling mirror
    h.pack_sphere(19, (0.0, -1.0, 16.0), 0.8, (4.0, 2.0, 1.0), emissive=True)    # behind, on the axis
    h.pack_sphere(20, (0.0, 2.0, 5.0), 1.5, (0.95, 0.95, 0.95), reflectivity=0.0)  # mirror facing the camera
    h.set_mode(0, 21)
    return h, [(0, H // 2), (W - 1, H - 1), (W // 2, (H * 2) // 3)]


def _tangent(W, H, spp):
    h = _syn(12, spp, W, H, 17)
    pix = [(W // 4, H // 3), (W // 2, H // 2), ((3 * W) // 4, (2 * H) // 3), (W // 3, (3 * H) // 4),
           ((2 * W) // 3, H // 5)]
    radii = [1.5, 0.75, 1.25, 1.0, 0.5]
    for k, ((x, y), r) in enumerate(zip(pix, radii)):
        d = _ray(h, W, H, x, y)
        c = tangent_center(d, 6.0 + k, r, seed=100 + k)
        h.pack_sphere(12 + k, c, r, (0.3 + 0.1 * k, 0.8 - 0.1 * k, 0.5), reflectivity=[1.0, 0.0, 0.4, 1.0, 0.7][k])
    h.set_mode(0, 17)
    return h, pix


def _huge(W, H, spp):
    h = _syn(16, spp, W, H, 18)
    h.pack_sphere(16, (0.0, -10002.5, 0.0), 1e4, (0.45, 0.4, 0.35))                  # config q's ground
    h.pack_sphere(17, (0.0, 0.0, 0.0), 1e4, (0.6, 0.7, 0.9), emissive=True)          # sky dome around everything
    h.set_mode(0, 18)
    return h, [(W // 2, H // 8)]


def _tiny_far(W, H, spp):
    h = _syn(16, spp, W, H, 28)
    pix = [(W // 5, (4 * H) // 5), (W // 2, (7 * H) // 8), ((4 * W) // 5, (3 * H) // 4), (W // 8, H - 2),
           ((7 * W) // 8, (5 * H) // 6), (W // 3, (2 * H) // 3), ((3 * W) // 5, (9 * H) // 10), (W - 2, H - 2)]
    for k, (x, y) in enumerate(pix):
        d = _ray(h, W, H, x, y)
        c = (CAM.astype(np.float64) + (900.0 + 25.0 * k) * d.astype(np.float64)).astype(np.float32)
        h.pack_sphere(16 + k, c, 1e-3, (4.0, 4.0, 0.5) if k % 2 else (0.9, 0.2, 0.9), emissive=bool(k % 2))
    rng = np.random.default_rng(5)
    for k in range(4):  # tiny and far, off every pixel centre
        c = rng.uniform([-400, 50, -1100], [400, 500, -900]).astype(np.float32)
        h.pack_sphere(24 + k, c, 1e-3, (0.9, 0.9, 0.9))
    h.set_mode(0, 28)
    return h, pix


def _overlap(W, H, spp):
    h = _syn(16, spp, W, H, 26)
    h.pack_sphere(16, (1.0, 0.5, 2.0), 1.0, (0.9, 0.2, 0.2), reflectivity=0.5)
    h.pack_sphere(17, (1.0, 0.5, 2.0), 1.0, (0.2, 0.9, 0.2))                 # duplicate: 16 wins every tie
    h.pack_sphere(18, (1.6, 0.5, 2.2), 0.9, (0.2, 0.2, 0.9), reflectivity=0.0)
    h.pack_sphere(19, (1.0, 0.5, 2.0), 0.5, (3.0, 3.0, 3.0), emissive=True)  # concentric inside 16
    h.pack_sphere(20, (0.0, -35.0, 0.0), 33.0, (0.1, 0.1, 0.1))              # duplicate of the ground (0)
    h.pack_sphere(21, (-2.0, 1.0, 1.0), 1.2, (2.0, 1.0, 3.0), emissive=True)
    h.pack_sphere(22, (-1.2, 1.3, 1.4), 0.8, (0.9, 0.9, 0.9), reflectivity=0.0)
    h.pack_sphere(23, (3.0, -0.5, 0.0), 1.0, (0.7, 0.7, 0.2))                # touching pair
    h.pack_sphere(24, (5.0, -0.5, 0.0), 1.0, (0.2, 0.7, 0.7), reflectivity=0.2)
    h.pack_sphere(25, (3.0, -0.5, 0.0), 1.0, (0.7, 0.7, 0.2))                # duplicate of 23
    h.set_mode(0, 26)
    return h, [(W // 2 + W // 20, H // 2 + H // 20)]


def _light_inside(W, H, spp):
    h = _syn(16, spp, W, H, 18)
    h.pack_sphere(16, (-3.0, 3.0, -2.0), 1.0, (0.9, 0.9, 0.9), reflectivity=0.5)
    h.pack_sphere(17, (4.0, 1.0, 0.0), 1.5, (0.3, 0.6, 0.9), reflectivity=0.0)
    L = h.vec4(5)  # light_pos: inside sphere 16 (it moves by +0.1 per frame in the Phong tests)
    L[:] = (-3.05, 2.95, -2.05, 0.0)
    h.set_mode(0, 18)
    return h, [(W // 3, (2 * H) // 3)]


def _adv256(W, H, spp):
    h = _syn(256, spp, W, H, 256)
    h.pack_sphere(240, (-2.0, 0.0, 14.0), 1.5, (0.9, 0.5, 0.2))            # straddles the camera plane
    h.pack_sphere(241, (0.0, 0.0, 20.0), 3.0, (0.9, 0.9, 0.2))             # behind
    h.pack_sphere(242, (2.6, 1.2, 15.0), 2.0, (0.9, 0.9, 0.9), reflectivity=0.0)
    g5 = h.shapes[5, 0].copy()
    h.pack_sphere(243, tuple(g5[:3]), float(g5[3]), (0.1, 0.9, 0.1))       # duplicate of 5
    g7 = h.shapes[7, 0].copy()
    h.pack_sphere(244, tuple(g7[:3]), float(g7[3]) * 0.5, (3.0, 3.0, 3.0), emissive=True)  # concentric in 7
    h.pack_sphere(245, (0.0, 0.0, 0.0), 1e4, (0.6, 0.7, 0.9), emissive=True)  # sky dome: camera inside
    h.pack_sphere(246, (0.0, -10002.5, 0.0), 1e4, (0.45, 0.4, 0.35))
    pix = [(W // 2, (2 * H) // 3), ((2 * W) // 3, (5 * H) // 6)]
    d = _ray(h, W, H, *pix[0])
    h.pack_sphere(247, tangent_center(d, 5.0, 1.0, seed=7), 1.0, (0.9, 0.4, 0.1))
    d = _ray(h, W, H, *pix[1])
    c = (CAM.astype(np.float64) + 950.0 * d.astype(np.float64)).astype(np.float32)
    h.pack_sphere(248, c, 1e-3, (4.0, 4.0, 4.0), emissive=True)
    h.set_mode(0, 256)
    return h, pix


_BUILDERS = {"cam_inside": _cam_inside, "straddle": _straddle, "tangent": _tangent, "huge": _huge,
             "tiny_far": _tiny_far, "overlap": _overlap, "light_inside": _light_inside, "adv256": _adv256}


def scene(name: str, W: int, H: int, spp: int):
    return _BUILDERS[name](W, H, spp)
