#!/usr/bin/env python
"""How much random()'s argument rounding choices move the frames.
MEASUREMENT TOOL (CPU only; runs the oracle, test infrastructure).

The GLSL (ao_compute.glsl:63-73, 152-157, 317-319) leaves it to the compiler whether each a*b+c
in the hash's argument is one fused multiply-add or two roundings.  random() multiplies sin by
43758.5 before fract(), so a one-ulp change of its argument picks another sample.  This renders
configs (c) and (d) (the bench's scenes and rand_buffer seeds, 3 frames) with the C oracle in
each contraction variant (oracle.set_contraction) and compares every variant with the build's
own semantics (variant 0, which the kernels and the goldens use):
  1 = unfused dot() inside random() (the GLSL read literally: both products rounded);
  2 = fused hemisphere seeds (seed1 + xy*seed4 -> fma(xy, seed4, seed1), ...);
  4 = fused anti-aliasing jitter seeds (seed1 + xy*seed2 - xy + seed3 -> (fma(xy, seed2, seed1) - xy) + seed3, ...);
  7 = all three.
Reported per config and variant: the fraction of image channels within the north-star tolerance
(|a - b| <= 1e-4 max(|a|, |b|) + 1e-6), of pixels with all three channels within it, and of depth /
normal vec4s that are bit-identical (frame 3's ring slot).

    python tools/contraction_effect.py [--configs c,d] [--frames 3] [--threads 8] [--out FILE]
"""
from __future__ import annotations

import argparse
import json
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

VARIANTS = {0: "build (fused dot in random(), seed / jitter sums as written)",
            1: "unfused dot() inside random()",
            2: "fused hemisphere seed arithmetic",
            4: "fused jitter seed arithmetic",
            7: "all three"}


def render(cfg: str, frames: int, threads: int, flags: int) -> dict:
    import oracle
    from bench import CONFIGS, config_header
    from real_time_ray_tracer_amd import SSBO

    oracle.set_contraction(flags)
    try:
        W, H, S, spp, mode, _ = CONFIGS[cfg]
        h = config_header(cfg)
        s = SSBO(h, W, H)
        d = oracle.dims(W, H, h.S, h.AA)
        img = np.zeros((H, W, 4), np.float32)
        f = 0
        for k in range(frames):
            h.fill_rand_buffer(7000 + k)
            h.set_mode(f, h.num_objects)
            s.set_header(h)
            f = oracle.dispatch(s.data, d, mode, f, img, nthreads=threads)
        slot = (f - 1) % 8
        return {"image": img, "depth": s.depth[slot].copy(), "normals": s.normals[slot].copy()}
    finally:
        oracle.set_contraction(0)


def compare(a: dict, b: dict) -> dict:
    x, y = a["image"][..., :3], b["image"][..., :3]
    close = np.abs(x - y) <= 1e-4 * np.maximum(np.abs(x), np.abs(y)) + 1e-6
    same_d = np.all(a["depth"].view(np.uint32) == b["depth"].view(np.uint32), axis=-1)
    same_n = np.all(a["normals"].view(np.uint32) == b["normals"].view(np.uint32), axis=-1)
    return {"image_channels_within_1e-4": round(float(close.mean()), 6),
            "pixels_all_channels_within_1e-4": round(float(close.all(axis=-1).mean()), 6),
            "max_abs_diff": round(float(np.abs(x - y).max()), 6),
            "depth_bit_identical": round(float(same_d.mean()), 6),
            "normals_bit_identical": round(float(same_n.mean()), 6)}


def main() -> None:
    import oracle

    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="c,d")
    ap.add_argument("--frames", type=int, default=3)
    ap.add_argument("--threads", type=int, default=8)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    res = {"what": __doc__.split("\n\n")[1].replace("\n", " "), "variants": VARIANTS, "frames": a.frames,
           "oracle": oracle.lib_name(), "configs": {}}
    for cfg in a.configs.split(","):
        t0 = time.time()
        base = render(cfg, a.frames, a.threads, 0)
        res["configs"][cfg] = {}
        for flags in (1, 2, 4, 7):
            res["configs"][cfg][str(flags)] = compare(render(cfg, a.frames, a.threads, flags), base)
            print(cfg, flags, VARIANTS[flags], json.dumps(res["configs"][cfg][str(flags)]), flush=True)
        print(f"{cfg}: {time.time() - t0:.0f} s", flush=True)
    txt = json.dumps(res, indent=1)
    if a.out:
        Path(a.out).write_text(txt + "\n")
    print(txt)


if __name__ == "__main__":
    main()
