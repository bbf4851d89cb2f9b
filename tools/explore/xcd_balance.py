#!/usr/bin/env python
"""Exploration: per-XCD finish times of AO launches (A/B build, RTRT_AO_VARIANT=100 writes each
XCD's first wave start, last wave end, wave count and summed wave time into the row counters).
Whole frame and the 8 strips of config (d), mode 2, one launch per frame.

    RTRT_LIB=build/librtrt_ab.so python tools/explore/xcd_balance.py [--rot 0|1]
"""
import os
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
os.environ["RTRT_AO_VARIANT"] = "100"

from bench import CONFIGS, config_header  # noqa: E402
from real_time_ray_tracer_amd import Renderer  # noqa: E402

W, H, S, spp, _, _ = CONFIGS["d"]
h = config_header("d")
bounds = [0, 172, 333, 488, 664, 976, 1246, 1562, 2160]
cases = [("whole", None), ("strip0", (0, 172))] if len(sys.argv) < 2 else [("whole", None)]
for name, rows in cases:
    r = Renderer(W, H, S, spp, rows=rows)
    r.enable_counters(totals=False, rows=True)
    f = 0
    res = []
    for k in range(4):
        h.fill_rand_buffer(7000 + k)
        h.set_mode(f, h.num_objects)
        r.upload_header(h)
        r.read_row_counters(reset=True)
        f = r.dispatch(2, f)
        r.synchronize()
        call = r.read_row_counters(reset=True)
        c = call[:32].astype(np.uint64)
        if name == "whole" and k == 0:
            m = call[32:32 + 1024].astype(np.int64) - 1
            print("block -> XCD, blocks 0..127:", m[:128].tolist())
            print("blocks per XCD among the first 1024:", np.bincount(m[m >= 0], minlength=8).tolist())
        end = c[0:16:2].astype(np.float64)
        start = (~c[1:16:2]).astype(np.float64)
        waves, busy = c[16:24], c[24:32].astype(np.float64)
        t0 = start.min()
        dur = (end.max() - t0) * 1e-2  # 100 MHz -> us
        rel_end = (end - t0) * 1e-2
        res.append((dur, rel_end, waves, busy * 1e-2))
    dur, rel_end, waves, busy = res[-1]
    print(f"{name:7s} launch {dur:8.1f} us; XCD ends (us) {np.round(rel_end, 1).tolist()}; "
          f"spread {rel_end.max() - rel_end.min():.1f} us ({100 * (rel_end.max() - rel_end.min()) / dur:.1f}%); "
          f"busy per XCD (ms) {np.round(busy / 1e3, 2).tolist()}; waves {waves.tolist()}", flush=True)
    r.close()
