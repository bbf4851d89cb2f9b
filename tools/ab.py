#!/usr/bin/env python
"""Interleaved A/B timing of kernel variants in one process (cdna_hip_programming.md §5.4
rule 24).  Each round renders the same frames once per variant (env RTRT_AO_VARIANT, read by
the shim at launch) and records the per-launch HIP-event time of the trace kernel; images
must be bit-identical across variants.

    python tools/ab.py --config d --variants 0,1,2 --rounds 3 --frames 4
    python tools/ab.py --config d --libs build/old/librtrt.so,real_time_ray_tracer_amd/librtrt.so

With --libs the variants are two (or more) builds of the library, each loaded as its own copy
in the same process, so builds are compared on the same GPU clock state (and bit for bit).
"""
import argparse
import json
import os
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

from bench import CONFIGS, config_header  # noqa: E402
from real_time_ray_tracer_amd import Header, Renderer, aspect_for  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="d")
    ap.add_argument("--variants", default="0,1,2")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--frames", type=int, default=4)
    ap.add_argument("--env", default="RTRT_AO_VARIANT")
    ap.add_argument("--libs", default="", help="comma-separated librtrt.so builds to compare instead of variants")
    ap.add_argument("--prog", type=int, default=0, help="program to time (default: the trace pass)")
    ap.add_argument("--time-from", type=int, default=1, help="first frame timed (history fills over 8 frames)")
    ap.add_argument("--allow-diff", action="store_true", help="timing ablations: images may differ")
    args = ap.parse_args()
    W, H, S, spp, mode, desc = CONFIGS[args.config]
    variants = [v for v in args.variants.split(",")]
    libs = {}
    if args.libs:
        import ctypes as C
        from real_time_ray_tracer_amd import _lib
        _lib.load()  # torch first, then the default build (the Header helpers use it)
        variants = args.libs.split(",")
        for path in variants:
            lib = C.CDLL(str(Path(path).resolve()), mode=C.RTLD_LOCAL)
            for name, (res, argt) in _lib.SIGNATURES.items():
                if not hasattr(lib, name):  # an older build: entry points added since are unused here
                    continue
                fn = getattr(lib, name)
                fn.restype = res
                fn.argtypes = argt
            libs[path] = lib
    h = config_header(args.config)
    prog = args.prog or {1: 1, 2: 3, 3: 4, 4: 5}[mode]
    times = {v: [] for v in variants}
    ref_img = None
    counts = None
    for rnd in range(args.rounds):
        for v in variants:
            if libs:
                from real_time_ray_tracer_amd import _lib
                _lib._LIB = libs[v]
            else:
                os.environ[args.env] = v
            r = Renderer(W, H, S, spp)
            if rnd == 0 and v == variants[0]:
                r.enable_counters(True)
            f = 0
            for k in range(args.frames):
                if mode in (1, 2):
                    h.fill_rand_buffer(7000 + k)
                else:
                    h.moving_light(False)
                h.set_mode(f, h.num_objects)
                r.upload_header(h)
                if k == args.time_from:
                    r.enable_timing(True)
                f = r.dispatch(mode, f)
            n, ms = r.kernel_stats(prog)
            times[v].append(ms / n)
            if rnd == 0 and v == variants[0]:
                counts = r.read_counters()
            img = r.image()
            if ref_img is None:
                ref_img = img
            same = np.array_equal(img.view(np.uint32), ref_img.view(np.uint32))
            print(f"round {rnd} variant {v}: {ms / n:.3f} ms/launch identical={same}", flush=True)
            if not same and not args.allow_diff:
                raise SystemExit(f"variant {v} changed the image")
            r.close()
    out = {"config": desc, "counters": counts,
           "ms": {v: {"median": float(np.median(t)), "min": float(np.min(t))} for v, t in times.items()}}
    if counts:
        out["lane_utilisation"] = counts["tests"] / max(counts["executed_lane_tests"], 1)
        out["segments_per_sample"] = counts["segments"] / max(counts["samples"], 1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
