"""Per-pixel segment counts of h_compute at config (b) (numpy restatement of the oracle), and
their distribution per 8x8 wave tile: how much of a wave's bounce loop its lanes use."""
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
from bench import CONFIGS, config_header  # noqa: E402
from oracle import numpy_ref as nr  # noqa: E402

W, H, S, spp, mode, _ = CONFIGS["b"]
h = config_header("b")
h.moving_light(False)
ssbo = np.zeros(h.data.size + 3 * 8 * W * H * 4, np.float32)
ssbo[:h.data.size] = h.data
R = nr.Ref(ssbo, W, H, S, spp) if hasattr(nr, "Ref") else None
cls = [v for v in vars(nr).values() if isinstance(v, type) and hasattr(v, "h_compute")][0]
R = cls(ssbo, W, H, S, spp)
F = np.float32
ys, xs = np.mgrid[0:H, 0:W]
x = xs.ravel().astype(np.int64); y = ys.ravel().astype(np.int64)
dirs = R.primary(x, y)
pos = np.broadcast_to(R.hdr[4, :3], dirs.shape).astype(F).copy()
live = np.ones(len(x), bool)
segs = np.zeros(len(x), np.int32)
for seg in range(R.D):
    idx = np.nonzero(live)[0]
    if idx.size == 0:
        break
    segs[idx] += 1
    t, ind = R.closest(pos[idx], dirs[idx], 0.001)
    stop = np.ones(idx.size, bool)
    hit = ind >= 0
    hi = idx[hit]
    curr = pos[hi] + t[hit, None] * dirs[hi]
    nn = R.normal(ind[hit], curr)
    refl = (F(1.0) - R.shapes[ind[hit], 3, 3]).astype(F)
    go = ~(refl < F(0.001))
    stop[hit] = ~go
    g = hi[go]
    dn = nr.dot3(dirs[g], nn[go])
    dirs[g] = nr.normalize3(dirs[g] - F(2.0) * (dn[:, None] * nn[go]))
    pos[g] = curr[go]
    live[idx[stop]] = False
s = segs.reshape(H, W)
print("pixels", s.size, "mean segs", s.mean(), "hist", np.bincount(s.ravel())[:22].tolist())
Ht, Wt = H // 8 * 8, W // 8 * 8
tiles = s[:Ht, :Wt].reshape(Ht // 8, 8, Wt // 8, 8).transpose(0, 2, 1, 3).reshape(-1, 64)
mx = tiles.max(1); sm = tiles.sum(1)
print("tiles", len(mx), "lane use of seg loop", sm.sum() / (64 * mx.sum()))
print("tile max hist", np.bincount(mx)[:22].tolist())
print("share of wave-seg-iterations in tiles with max>=3:", (mx * (mx >= 3)).sum() / mx.sum())
