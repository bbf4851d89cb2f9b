#!/usr/bin/env python
"""Single-GPU estimate of strong-scaling efficiency before the driver's multi-GPU run: time
each rank's strip of an N-way split on its own (pipelined mode 1, as bench.py runs it) and
compare the slowest strip with the whole frame / N.  With --calibrate the plans after the
first are gather-aware (rt_plan_strips_gather, as bench.py plans them): the root strip (rank 0's,
never sent) and the bounds minimise max(render, per-link copy, root ingest) at a STATED link rate
(--link-gbps, default 76.8 GB/s = one direction of one 153.6 GB/s xGMI link, MI355X), and the
estimate is reported with and without that link bound (the copies themselves cannot run on a
one-GPU box).

    python tools/strip_scaling.py --config d --n 8 --frames 20 --calibrate --warm-ms 300
"""
import json
import argparse
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

from bench import CONFIGS, config_header  # noqa: E402
from real_time_ray_tracer_amd import Header, Renderer, aspect_for  # noqa: E402
from real_time_ray_tracer_amd.dist import (balanced_bounds, equal_bounds, gather_bound,  # noqa: E402
                                           gather_bounds)


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
    ap.add_argument("--link-gbps", type=float, default=76.8,
                    help="stated one-way rate of one xGMI link into the root (GB/s) for the gather-aware plans")
    ap.add_argument("--ingest-gbps", type=float, default=0.0, help="root ingest rate (default min(n-1, 7) x link)")
    ap.add_argument("--save-profile", default="", help="write the calibrated per-row ms profile and plan (JSON)")
    a = ap.parse_args()
    W, H, S, spp, mode, _ = CONFIGS[a.config]
    link = a.link_gbps
    ingest = a.ingest_gbps or min(a.n - 1, 7) * link
    root = 0
    row_ms = None
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
                per_row = np.concatenate([np.full(b[i + 1] - b[i], t[i] / (b[i + 1] - b[i])) for i in range(a.n)])
                pred = gather_bound(per_row, b, root, W, link, ingest)
                measured.append((pred["bound_ms"], list(b), root, t, per_row))
                print(f"calibration plan {it}: {b} root strip {root} strip ms {[round(x, 3) for x in t]} predicted "
                      f"{ {k: round(v, 4) for k, v in pred.items()} }")
                if it < 2:
                    cost = calibrate_row_cost(b, cost, t)
                    b, root, _ = gather_bounds(cost, a.n, W, link, ingest)
            _, b, root, _, row_ms = min(measured, key=lambda m: m[0])
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
    per_row = np.concatenate([np.full(b[i + 1] - b[i], strips[i] / (b[i + 1] - b[i])) for i in range(a.n)])
    g = gather_bound(per_row, b, root, W, link, ingest)
    sent = [(b[i + 1] - b[i]) * W * 16 for i in range(a.n) if i != root]
    print(f"gather (stated link {link} GB/s, ingest {ingest} GB/s): root strip {root} ({b[root + 1] - b[root]} rows), "
          f"largest sent strip {max(sent) / 1e6 if sent else 0:.1f} MB, link bound {g['link_ms']:.3f} ms, ingest bound "
          f"{g['ingest_ms']:.3f} ms -> frame bound {g['bound_ms']:.3f} ms, efficiency with the gather "
          f"{full / a.n / g['bound_ms']:.3f}")
    if a.save_profile:
        Path(a.save_profile).write_text(json.dumps({
            "config": a.config, "n": a.n, "bounds": b, "root_strip": root, "strip_ms": strips, "whole_frame_ms": full,
            "link_gbps": link, "ingest_gbps": ingest, "predicted": g,
            "row_ms_calibrated": [round(float(x), 9) for x in (row_ms if row_ms is not None else per_row)]}) + "\n")


if __name__ == "__main__":
    main()
