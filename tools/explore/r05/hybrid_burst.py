#!/usr/bin/env python
"""Config (b) hybrid_kernel per-launch time as a burst (200 back-to-back launches between two
events, after 64 frames so the tile schedule is in use), for A/B-library variants selected by an
environment variable (RTRT_HY_ABL timing ablations) or library builds (--libs).

    RTRT_LIB=build/librtrt_ab.so python tools/explore/r05/hybrid_burst.py --env RTRT_HY_ABL --variants 0,1,2,3,5
    python tools/explore/r05/hybrid_burst.py --libs a.so,b.so
"""
import argparse
import ctypes as C
import json
import os
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[3]
sys.path.insert(0, str(ROOT))

import torch  # noqa: E402

from bench import CONFIGS, config_header  # noqa: E402
from real_time_ray_tracer_amd import Renderer, _lib  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="b")
    ap.add_argument("--env", default="RTRT_HY_ABL")
    ap.add_argument("--variants", default="0")
    ap.add_argument("--libs", default="")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--reps", type=int, default=200)
    ap.add_argument("--no-schedule", action="store_true", help="tile schedule off (row order) for every variant")
    a = ap.parse_args()
    W, H, S, spp, mode, _ = CONFIGS[a.config]
    prog = {3: 4, 4: 5}[mode]
    libs = {}
    variants = a.variants.split(",")
    if a.libs:
        _lib.load()
        variants = a.libs.split(",")
        for path in variants:
            lib = C.CDLL(str(Path(path).resolve()), mode=C.RTLD_LOCAL)
            for name, (res, argt) in _lib.SIGNATURES.items():
                if hasattr(lib, name):
                    getattr(lib, name).restype = res
                    getattr(lib, name).argtypes = argt
            libs[path] = lib
    times = {v: [] for v in variants}
    for rnd in range(a.rounds):
        for v in variants:
            if libs:
                _lib._LIB = libs[v]
            else:
                os.environ[a.env] = v
            h = config_header(a.config)
            r = Renderer(W, H, S, spp)
            if a.no_schedule:
                r.set_tile_schedule(False)
            f = 0
            for k in range(64):
                h.moving_light(True)
                h.set_mode(f, h.num_objects)
                r.upload_header(h)
                f = r.dispatch(mode, f)
            r.synchronize()
            slot = (f - 1) % 8
            st = torch.cuda.current_stream()
            r.set_stream(st)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            r.run_program(prog, slot)
            torch.cuda.synchronize()
            e0.record(st)
            for _ in range(a.reps):
                r.run_program(prog, slot)
            e1.record(st)
            e1.synchronize()
            us = e0.elapsed_time(e1) / a.reps * 1e3
            times[v].append(us)
            print(f"round {rnd} variant {v}: {us:.2f} us/launch (schedule state {r.tile_schedule_state()})", flush=True)
            r.close()
    print(json.dumps({"config": a.config, "us_per_launch": {v: {"median": float(np.median(t)), "min": float(np.min(t))}
                                                             for v, t in times.items()}}))


if __name__ == "__main__":
    main()
