#!/usr/bin/env python
"""Host cost of one frame's enqueue (header fill + upload + dispatch), measured on frames too
small to keep the GPU busy, so the loop is host-bound: wall time per frame = host time.  For
the N-GPU strips of bench.py, whose GPU time per frame shrinks as 1/N, this is the floor.

    python tools/host_cost.py [--mode 1] [--frames 400]
"""
import argparse
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

from real_time_ray_tracer_amd import Header, Renderer, aspect_for  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mode", type=int, default=1)
    ap.add_argument("--frames", type=int, default=400)
    ap.add_argument("--W", type=int, default=3840)
    ap.add_argument("--rows", type=int, default=2, help="strip height (tiny: the GPU idles)")
    a = ap.parse_args()
    W, H, S, spp = a.W, 2160, 64, 16
    h = Header.synthetic(S, spp, 1237, aspect_for(W, H))
    for pipelined in ([False, True] if a.mode == 1 else [False]):
        for timing in (False, True):
            r = Renderer(W, H, S, spp, rows=(1000, 1000 + a.rows))
            if pipelined:
                r.enable_pipelining(True)
            r.enable_timing(timing)
            f = 0
            for k in range(a.frames + 20):
                if k == 20:
                    r.synchronize()
                    t0 = time.perf_counter()
                h.fill_rand_buffer(7000 + k)
                h.set_mode(f, S)
                r.upload_header(h)
                f = r.dispatch(a.mode, f)
            t_enq = time.perf_counter() - t0
            r.synchronize()
            t_all = time.perf_counter() - t0
            print(f"mode {a.mode} pipelined={pipelined} timing={timing}: enqueue {t_enq / a.frames * 1e3:.4f} ms/frame, "
                  f"wall {t_all / a.frames * 1e3:.4f} ms/frame", flush=True)
            r.close()


if __name__ == "__main__":
    main()
