#!/usr/bin/env python
"""Wall ms per pipelined mode-1 frame (rt_compute_frames, 40 frames, 3 rounds) of a bench config.
With RTRT_LIB=build/librtrt_ab.so RTRT_POST_SKIP=1 the post-process launches are skipped: the
AO-only floor of the same two-stream pipeline.

    python tools/explore/pipeline_floor.py --config d
"""
import argparse
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
from bench import CONFIGS, config_header  # noqa: E402
from real_time_ray_tracer_amd import Renderer  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="d")
    ap.add_argument("--frames", type=int, default=40)
    ap.add_argument("--no-pipeline", action="store_true")
    a = ap.parse_args()
    W, H, S, spp, mode, _ = CONFIGS[a.config]
    h = config_header(a.config)
    r = Renderer(W, H, S, spp)
    if not a.no_pipeline:
        r.enable_pipelining(True)
    f = r.compute_frames(h, mode, 0, 12, 7000, False)
    r.synchronize()
    out = []
    for _ in range(3):
        t0 = time.perf_counter()
        f = r.compute_frames(h, mode, f, a.frames, 7000, False)
        r.synchronize()
        out.append((time.perf_counter() - t0) / a.frames * 1e3)
    print(a.config, "pipelined" if not a.no_pipeline else "sequential", " ".join(f"{x:.4f}" for x in out))


if __name__ == "__main__":
    main()
