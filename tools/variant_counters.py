#!/usr/bin/env python
"""Work counters of AO kernel variants on a bench config (lane utilisation of the bounce
rounds = algorithmic tests / executed lane-tests).

    python tools/variant_counters.py --config d --variants 7,20
"""
import argparse
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

from bench import CONFIG_INDEX, CONFIGS  # noqa: E402
from real_time_ray_tracer_amd import Header, Renderer, aspect_for  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="d")
    ap.add_argument("--variants", default="7")
    ap.add_argument("--frames", type=int, default=2)
    a = ap.parse_args()
    W, H, S, spp, mode, _ = CONFIGS[a.config]
    h = Header.synthetic(S, spp, 1234 + CONFIG_INDEX[a.config], aspect_for(W, H))
    for v in a.variants.split(","):
        os.environ["RTRT_AO_VARIANT"] = v
        r = Renderer(W, H, S, spp)
        f = 0
        for k in range(a.frames):
            if k == a.frames - 1:
                r.enable_counters(True)
                r.read_counters(reset=True)
                r.enable_timing(True)
            h.fill_rand_buffer(7000 + k)
            h.set_mode(f, S)
            r.upload_header(h)
            f = r.dispatch(2 if mode == 1 else mode, f)
        c = r.read_counters()
        n, ms = r.kernel_stats(3 if mode in (1, 2) else {3: 4, 4: 5}[mode])
        print(f"variant {v}: {ms / max(n, 1):.3f} ms  samples {c['samples'] / 1e6:.1f}M segments {c['segments'] / 1e6:.1f}M "
              f"tests {c['tests'] / 1e9:.2f}G executed {c['executed_lane_tests'] / 1e9:.2f}G "
              f"ratio {c['tests'] / max(c['executed_lane_tests'], 1):.3f}", flush=True)
        r.close()


if __name__ == "__main__":
    main()
