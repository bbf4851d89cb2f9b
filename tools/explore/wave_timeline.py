"""Per-wave timeline of hybrid_kernel at config (b) (A/B build, RTRT_HY_ABL=7: each wave's
s_memtime start/end and longest path land in its lane-0 pixel of the frame slot)."""
import os
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
os.environ["RTRT_HY_ABL"] = os.environ.get("RTRT_HY_ABL", "7")
from bench import CONFIGS, config_header  # noqa: E402
from real_time_ray_tracer_amd import Renderer  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "b"
W, H, S, spp, mode, _ = CONFIGS[cfg]
h = config_header(cfg)
r = Renderer(W, H, S, spp)
f = 0
for k in range(3):
    h.moving_light(False)
    h.set_mode(f, h.num_objects)
    r.upload_header(h)
    last = f
    f = r.dispatch(mode, f)
g = r.download(pixels=True, normals=False, depth=False, image=False)
px = g.pixels[last].view(np.uint32)  # [W][H][4]
xs = np.arange(0, W, 8)
ys = np.arange(0, H, 8)
rec = px[xs][:, ys]  # [nx][ny][4]
st = rec[..., 0].astype(np.int64)
en = rec[..., 1].astype(np.int64)
mx = rec[..., 2]
gx = (W + 15) // 16
bx = (xs // 16)[:, None] + 0 * ys[None, :]
by = 0 * xs[:, None] + (ys // 16)[None, :]
xcd = (by * gx + bx) % 8
hi = rec[..., 3].astype(np.int64)
spans = []
for k in [-1] + list(range(8)):
    sel = xcd == k if k >= 0 else xcd >= 0
    s0 = (hi[sel] << 32) | st[sel]
    e0 = (hi[sel] << 32) | en[sel]
    e0 = np.where(e0 < s0, e0 + (1 << 32), e0)
    t0 = s0.min()
    S, E = s0 - t0, e0 - t0
    dur = E - S
    spans.append(E.max())
    T = np.linspace(0, E.max(), 11)
    res = [int(((S <= t) & (E > t)).sum()) for t in T]
    print(f"xcd {k} (ticks of 10 ns): waves {sel.sum()} span {E.max()} clk, dur mean {dur.mean():.0f} max {dur.max()}, "
          f"start p50 {np.percentile(S, 50):.0f} p90 {np.percentile(S, 90):.0f} max {S.max()}, resident over time {res}")
    if k == -1:
        late = E >= np.percentile(E, 99)
        print("   last 1% of ends: max segs hist", np.bincount(mx[sel][late]).tolist(), "their start mean", S[late].mean(),
              "dur mean", dur[late].mean())
        order = np.argsort(S)
        print("   durations by start decile", [int(dur[order[i * len(order) // 10:(i + 1) * len(order) // 10]].mean()) for i in range(10)])
