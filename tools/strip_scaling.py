#!/usr/bin/env python
"""Single-GPU estimate of strong-scaling efficiency before the driver's multi-GPU run: time
each rank's strip of an N-way split on its own (pipelined mode 1, as bench.py runs it) and
compare the slowest strip with the whole frame / N.  The gather is not included.

    python tools/strip_scaling.py --config d --n 8 --frames 20
"""
import argparse
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

from bench import CONFIGS, config_header  # noqa: E402
from real_time_ray_tracer_amd import Header, Renderer, aspect_for  # noqa: E402
from real_time_ray_tracer_amd.dist import balanced_bounds, equal_bounds  # noqa: E402


def frame_ms(W, H, S, spp, mode, h, rows, frames, warm=8, kernels=False, multi=False):
    r = Renderer(W, H, S, spp, rows=rows)
    if mode == 1 and not kernels:
        r.enable_pipelining(True)
    if kernels:
        r.enable_timing(True)
    f = 0
    if frame_ms.warm_ms > 0:  # steady-state clocks: render for warm_ms of wall time first (DVFS ramp)
        tw = time.perf_counter()
        k = 0
        while (time.perf_counter() - tw) * 1e3 < frame_ms.warm_ms:
            h.fill_rand_buffer(7000 + k)
            h.set_mode(f, h.num_objects)
            r.upload_header(h)
            f = r.dispatch(mode, f)
            k += 1
            if k % 8 == 0:
                r.synchronize()
    if multi:  # the render loop in C++ (rt_compute_frames): multi-frame launches for modes 2-4
        f = r.compute_frames(h, mode, f, warm, 7000, False)
        r.synchronize()
        t0 = time.perf_counter()
        f = r.compute_frames(h, mode, f, frames, 7000 + warm, False)
        t_enq = time.perf_counter() - t0
        r.synchronize()
        ms = (time.perf_counter() - t0) / frames * 1e3
        r.close()
        frame_ms.host_ms = t_enq / frames * 1e3
        return ms
    for k in range(warm + frames):
        if k == warm:
            r.synchronize()
            t0 = time.perf_counter()
        h.fill_rand_buffer(7000 + k)
        h.set_mode(f, h.num_objects)
        r.upload_header(h)
        f = r.dispatch(mode, f)
    t_enq = time.perf_counter() - t0
    r.synchronize()
    ms = (time.perf_counter() - t0) / frames * 1e3
    if kernels:  # sum of the mode's kernel averages (HIP events, not overlapped)
        ms = 0.0
        for p in {1: [1, 2], 2: [3], 3: [4], 4: [5]}[mode]:
            n, tot = r.kernel_stats(p)
            ms += tot / max(n, 1)
    r.close()
    frame_ms.host_ms = t_enq / frames * 1e3  # host enqueue time per frame (GPU-bound if < ms)
    return ms


frame_ms.warm_ms = 0.0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="d")
    ap.add_argument("--n", type=int, default=8)
    ap.add_argument("--frames", type=int, default=20)
    ap.add_argument("--equal", action="store_true")
    ap.add_argument("--kernels", action="store_true", help="sum of kernel times (sequential) instead of frame wall time")
    ap.add_argument("--mode", type=int, default=0, help="override the config's mode (e.g. 2: the AO pass alone)")
    ap.add_argument("--warm-ms", type=float, default=0.0,
                    help="render this long before timing each case, so the GPU clock has settled (DVFS ramp)")
    ap.add_argument("--multi", action="store_true", help="frames through rt_compute_frames (multi-frame launches)")
    ap.add_argument("--only", type=int, default=-1, help="time only this strip (e.g. under rocprofv3)")
    ap.add_argument("--calibrate", action="store_true",
                    help="bench.py's calibration: time the plan's strips (pipelined frames for mode 1), rescale the profile, "
                         "re-balance; best of three measured plans")
    a = ap.parse_args()
    W, H, S, spp, mode, _ = CONFIGS[a.config]
    mode = a.mode or mode
    frame_ms.warm_ms = a.warm_ms
    h = config_header(a.config)
    full = frame_ms(W, H, S, spp, mode, h, None, a.frames, kernels=a.kernels, multi=a.multi) if a.only < 0 else float("nan")
    if a.equal:
        b = equal_bounds(H, a.n)
    else:  # cost profile from the row counters of one whole-frame probe
        r = Renderer(W, H, S, spp)
        r.enable_counters(totals=False, rows=True)
        h.fill_rand_buffer(7000)
        h.set_mode(0, S)
        r.upload_header(h)
        r.dispatch(mode, 0)
        cost = r.read_row_counters().astype(np.float64)
        r.close()
        b = balanced_bounds(cost, a.n)
        if a.calibrate:
            from real_time_ray_tracer_amd.dist import calibrate_row_cost
            measured = []
            for it in range(3):
                t = [frame_ms(W, H, S, spp, mode, h, (b[i], b[i + 1]), 16, warm=8, kernels=mode != 1) for i in range(a.n)]
                measured.append((max(t), list(b)))
                print(f"calibration plan {it}: {b} strip ms {[round(x, 3) for x in t]}")
                if it < 2:
                    cost = calibrate_row_cost(b, cost, t)
                    b = balanced_bounds(cost, a.n)
            b = min(measured, key=lambda m: m[0])[1]
    strips, host = [], []
    for i in range(a.n):
        if a.only >= 0 and i != a.only:
            continue
        strips.append(frame_ms(W, H, S, spp, mode, h, (b[i], b[i + 1]), a.frames, kernels=a.kernels, multi=a.multi))
        host.append(frame_ms.host_ms)
    print(f"whole frame {full:.3f} ms; {a.n} strips {b}")
    print("strip ms", [round(t, 3) for t in strips])
    print("host enqueue ms/frame", [round(t, 3) for t in host])
    if a.only >= 0:
        return
    print(f"ideal {full / a.n:.3f} ms, slowest strip {max(strips):.3f} ms -> efficiency "
          f"{full / a.n / max(strips):.3f} (balance {np.mean(strips) / max(strips):.3f}, "
          f"sum of strips / whole {sum(strips) / full:.3f})")


if __name__ == "__main__":
    main()
