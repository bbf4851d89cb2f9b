#!/usr/bin/env python
"""Exploration: AO launches of the whole frame and of single strips (multi-frame launches,
rt_compute_frames, mode 2), for a rocprofv3 --pmc GRBM_GUI_ACTIVE run: the effective clock per
dispatch = GRBM_GUI_ACTIVE / 8 XCDs / duration.  Strips are labelled by their launch order.

    rocprofv3 --pmc GRBM_GUI_ACTIVE --kernel-trace -d out -o run -- python3 tools/explore/clock_probe.py
"""
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))

from bench import CONFIGS, config_header  # noqa: E402
from real_time_ray_tracer_amd import Renderer  # noqa: E402

W, H, S, spp, _, _ = CONFIGS["d"]
h = config_header("d")
bounds = [0, 172, 333, 488, 664, 976, 1246, 1562, 2160]
for name, rows in [("whole", None), ("strip0", (0, 172)), ("strip7", (1562, 2160)), ("whole", None)]:
    r = Renderer(W, H, S, spp, rows=rows)
    f = r.compute_frames(h, 2, 0, 8, 7000, False)
    r.synchronize()
    t0 = time.perf_counter()
    f = r.compute_frames(h, 2, f, 16, 7008, False)
    r.synchronize()
    print(name, rows, f"{(time.perf_counter() - t0) / 16 * 1e3:.3f} ms/frame", flush=True)
    r.close()
