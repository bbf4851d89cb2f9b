#!/usr/bin/env python
"""Single-process check that row-strip contexts reproduce the whole frame bit for bit at a
bench config (the distributed path minus the collective).

    python tools/strip_check.py --config d --bounds 0,971,2160 --frames 4 --mode 1
"""
import argparse
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

from bench import CONFIG_INDEX, CONFIGS  # noqa: E402
from real_time_ray_tracer_amd import Header, Renderer, aspect_for  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="d")
    ap.add_argument("--bounds", default="0,971,2160")
    ap.add_argument("--frames", type=int, default=4)
    ap.add_argument("--mode", type=int, default=0)
    a = ap.parse_args()
    W, H, S, spp, mode, _ = CONFIGS[a.config]
    mode = a.mode or mode
    b = [int(v) for v in a.bounds.split(",")]
    h = Header.synthetic(S, spp, 1234 + CONFIG_INDEX[a.config], aspect_for(W, H))
    full = Renderer(W, H, S, spp)
    strips = [Renderer(W, H, S, spp, rows=(b[i], b[i + 1])) for i in range(len(b) - 1)]
    f = 0
    for k in range(a.frames):
        h.fill_rand_buffer(7000 + k)
        h.set_mode(f, S)
        for r in [full] + strips:
            r.upload_header(h)
            fn = r.dispatch(mode, f)
        f = fn
        want = full.image()
        got = np.concatenate([s.image() for s in strips], 0)
        bad = np.any(got.view(np.uint32) != want.view(np.uint32), axis=2)
        ys = np.nonzero(bad.any(axis=1))[0]
        print(f"frame {k}: mismatched pixels {int(bad.sum())}" + (f" rows {ys.min()}..{ys.max()} ({len(ys)})" if len(ys) else ""),
              flush=True)
        if k == a.frames - 1:
            gf = full.download(True, True, True, False)
            parts = [s.download(True, True, True, False) for s in strips]
            for name in ("pixels", "normals", "depth"):
                g = np.concatenate([getattr(p, name) for p in parts], 2)
                w = getattr(gf, name)
                print(name, "mismatch", int(np.any(g.view(np.uint32) != w.view(np.uint32), axis=3).sum()))


if __name__ == "__main__":
    main()
