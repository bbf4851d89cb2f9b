#!/usr/bin/env python
"""Where the pooled AO kernel's wave time goes: runs the ABL=3 build of ao_batch_kernel
(RTRT_AO_VARIANT=93, s_memtime laps per section summed over waves) on a bench config.

    python tools/sections.py --config d --frames 3
    python tools/sections.py --config d --variant 96   # the first bounce split into cull / survivors / shade
    python tools/sections.py --config d --variant 97   # event counts: first-bounce survivors, bounce-round tails
    python tools/sections.py --config d --variant 98   # full bounce rounds and split tail rounds apart
    python tools/sections.py --config e --variant 193  # (e)'s instantiation (196, 198 as 96, 98)
"""
import argparse
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

from bench import CONFIGS, config_header  # noqa: E402
from real_time_ray_tracer_amd import Header, Renderer, aspect_for  # noqa: E402

NAMES = ["cull setup", "prepare (primary + first shade)", "hand-out / regeneration", "bounce test + shade",
         "first bounce (batched) + combine + stores"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="d")
    ap.add_argument("--frames", type=int, default=3)
    ap.add_argument("--variant", default="93")
    a = ap.parse_args()
    W, H, S, spp, mode, _ = CONFIGS[a.config]
    os.environ["RTRT_AO_VARIANT"] = a.variant
    h = config_header(a.config)
    r = Renderer(W, H, S, spp)
    f = 0
    for k in range(a.frames):
        if k == a.frames - 1:
            r.enable_counters(True)
            r.read_counters(reset=True)
        h.fill_rand_buffer(7000 + k)
        h.set_mode(f, h.num_objects)
        r.upload_header(h)
        f = r.dispatch(2 if mode == 1 else mode, f)  # AO pass only: counters 5..7 are the kernel's
    c = r.read_counters()
    keys = ["samples", "segments", "shadow_rays", "tests", "executed_lane_tests", "filtered_pixels", "history_read",
            "history_accepted"]
    if a.variant == "97":
        v = [c[k] for k in keys]
        print(f"first bounce: {v[4]} batches, {v[5] / max(v[4], 1):.1f} live lanes per batch, "
              f"{v[0] / max(v[4], 1):.2f} survivor iterations per batch")
        print(f"  survivor iterations with any pre-test pass {v[1] / max(v[0], 1):.3f}, with any del >= 0 among "
              f"the passing lanes {v[2] / max(v[0], 1):.3f}; lanes passing per iteration {v[3] / max(v[0], 1):.2f}")
        print(f"bounce rounds: {v[6]} sphere iterations, any live lane del >= 0 in {v[7] / max(v[6], 1):.3f}")
        return
    if a.variant in ("98", "198"):
        names = ["cull setup", "prepare (primary + first shade)", "hand-out / regeneration", "full bounce rounds",
                 "first bounce (batched) + combine + stores", "split tail rounds"]
        v = [c[k] for k in keys]
        tot = sum(v[:6])
        for n, x in zip(names, v[:6]):
            print(f"{n:42s} {x / 1e9:9.3f} Gclk  {100 * x / tot:5.1f}%")
        print(f"full rounds {v[6]}, split tail rounds {v[7]}")
        return
    if a.variant in ("96", "196"):
        names = ["cull setup", "prepare (primary + first shade)", "hand-out / regeneration", "bounce test + shade",
                 "combine + stores", "first bounce: cone + cull", "first bounce: survivor tests",
                 "first bounce: shade"]
        v = [c[k] for k in keys]
        for n, x in zip(names, v):
            print(f"{n:34s} {x / 1e9:9.3f} Gclk  {100 * x / sum(v):5.1f}%")
        return
    vals = [c["samples"], c["segments"], c["shadow_rays"], c["tests"], c["executed_lane_tests"]]
    tot = sum(vals)
    for n, v in zip(NAMES, vals):
        print(f"{n:34s} {v / 1e9:9.3f} Gclk  {100 * v / tot:5.1f}%")
    rounds, sum_ncull, prepares = c["filtered_pixels"], c["history_read"], c["history_accepted"]
    b1_surv, sum_ncull = sum_ncull >> 24, sum_ncull & ((1 << 24) - 1)
    print(f"batched first bounce: {b1_surv / max(prepares, 1):.2f} spheres tested per prepared batch (of {S})")
    print(f"bounce rounds {rounds}  prepares {prepares}  mean culled primary set {sum_ncull / max(prepares, 1):.2f}")
    print(f"bounce sphere-iterations per frame {rounds * S / 1e6:.1f} M; per 64-sample prepare batch "
          f"{rounds / max(prepares, 1):.2f} rounds")
    r.close()
    # the default kernel's work counters on the same frames: useful bounce segments
    os.environ["RTRT_AO_VARIANT"] = "7"
    r = Renderer(W, H, S, spp)
    f = 0
    for k in range(a.frames):
        if k == a.frames - 1:
            r.enable_counters(True)
            r.read_counters(reset=True)
        h.fill_rand_buffer(7000 + k)
        h.set_mode(f, h.num_objects)
        r.upload_header(h)
        f = r.dispatch(2 if mode == 1 else mode, f)
    c2 = r.read_counters()
    r.close()
    bounce = c2["segments"] - c2["samples"]
    print(f"useful bounce segments {bounce / 1e6:.1f} M = {bounce / max(rounds * 64, 1):.3f} of bounce lane slots; "
          f"samples {c2['samples'] / 1e6:.1f} M; executed lane-tests {c2['executed_lane_tests'] / 1e9:.2f} G")


if __name__ == "__main__":
    main()
