#!/usr/bin/env python
"""Per-frame vs batched launches of a mode-2/3/4 config: HIP-event kernel time per frame and wall
time per frame for rt_compute_frames with rt_set_frame_batch(1) and (8), on the same frames.

    python tools/explore/per_frame_launch.py --config c --frames 40
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
    ap.add_argument("--config", default="c")
    ap.add_argument("--frames", type=int, default=40)
    a = ap.parse_args()
    W, H, S, spp, mode, _ = CONFIGS[a.config]
    h = config_header(a.config)
    r = Renderer(W, H, S, spp)
    prog = {2: 3, 3: 4, 4: 5}[mode]
    f = r.compute_frames(h, mode, 0, 16, 7000, False)
    for batch in (1, 8, 1, 8):
        r.set_frame_batch(batch)
        r.synchronize()
        r.enable_timing(True)
        r.reset_stats()
        t0 = time.perf_counter()
        f = r.compute_frames(h, mode, f, a.frames, 7000, False)
        r.synchronize()
        wall = (time.perf_counter() - t0) / a.frames * 1e3
        n, ms = r.kernel_stats(prog)
        r.enable_timing(False)
        print(f"batch {batch}: wall {wall:.4f} ms/frame, kernel {ms / max(n, 1):.4f} ms/frame over {n} frames")


if __name__ == "__main__":
    main()
