#!/usr/bin/env python
"""Exploration (float64, statistics only — not parity): how many sphere tests would a
conservative per-round cone cull leave for the FIRST-bounce rays of config (d), with the
64 rays of a round taken (a) in sample order, (b) grouped by direction inside the pool?

    python tools/explore/bounce_coherence.py [npools]
"""
import sys

import numpy as np

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from real_time_ray_tracer_amd.host import Header, aspect_for  # noqa: E402

W, H, S, SPP = 3840, 2160, 64, 16
TP = 256 // SPP


def main():
    npools = int(sys.argv[1]) if len(sys.argv) > 1 else 3000
    h = Header.synthetic(S, SPP, 1234 + 3, aspect_for(W, H))
    d = h.data.astype(np.float64)
    hor, ver, llc, cam = d[4:7], d[8:11], d[12:15], d[16:19]
    sh = h.shapes.astype(np.float64)
    C, R = sh[:, 0, :3], sh[:, 0, 3]
    emis, refl = sh[:, 1, 3] > 0.9, sh[:, 3, 3]
    rng = np.random.default_rng(1)
    pools = rng.integers(0, W * H // TP, npools)
    tot = {"base": 0, "order": 0, "sorted4": 0, "sorted_oct": 0, "batch_g1": 0, "batch_g2": 0, "batch_g4": 0,
           "batch_g8": 0, "batch_g1_2s": 0}
    nb = 0
    for p in pools:
        pix = p * TP + np.arange(TP)
        x, y = (pix % W).astype(np.float64), (pix // W).astype(np.float64)
        x = np.repeat(x, SPP) + rng.uniform(-0.083, 0.083, TP * SPP)
        y = np.repeat(y, SPP) + rng.uniform(-0.083, 0.083, TP * SPP)
        dirs = llc + (x / W)[:, None] * hor + (y / H)[:, None] * ver
        dirs /= np.linalg.norm(dirs, axis=1)[:, None]
        pmc = cam - C  # [S,3]
        b = dirs @ pmc.T  # [N,S]
        dl = b * b - (pmc * pmc).sum(1) + R * R
        s = np.sqrt(np.maximum(dl, 0))
        t2, t1 = -b - s, -b + s
        t = np.where(t2 > 1e-4, t2, np.where(t1 > 1e-4, t1, np.inf))
        t[dl < 0] = np.inf
        ind = t.argmin(1)
        tm = t[np.arange(len(t)), ind]
        live = np.isfinite(tm) & ~emis[ind]
        if not live.any():
            continue
        ind, tm, dr = ind[live], tm[live], dirs[live]
        o = cam + tm[:, None] * dr
        n = o - C[ind]
        n /= np.linalg.norm(n, axis=1)[:, None]
        u = rng.normal(size=(len(o), 3))
        u /= np.linalg.norm(u, axis=1)[:, None]
        rf = refl[ind][:, None]
        Rv = dr - 2 * (dr * n).sum(1)[:, None] * n
        Rv /= np.linalg.norm(Rv, axis=1)[:, None]
        nd = np.where(rf > 0.999, n + u, Rv + rf * u)
        nd /= np.linalg.norm(nd, axis=1)[:, None]
        nb += len(o)
        tot["base"] += len(o) * S

        def cull_count(idx, per_ray=True, two_sided=False):
            oo, dd = o[idx], nd[idx]
            oc = oo.mean(0)
            rho = np.linalg.norm(oo - oc, axis=1).max()
            a = dd.sum(0)
            a /= max(np.linalg.norm(a), 1e-30)
            cth = (dd @ a).min()
            th = np.arccos(np.clip(cth, -1, 1))
            v = C - oc
            L = np.linalg.norm(v, axis=1)
            Rp = R + rho + 1e-3
            inside = L <= Rp
            al = np.arcsin(np.clip(Rp / np.maximum(L, 1e-30), 0, 1))
            be = np.arccos(np.clip((v @ a) / np.maximum(L, 1e-30), -1, 1))
            keep = inside | (be <= th + al)
            if two_sided:
                keep |= (np.pi - be) <= th + al
            return keep.sum() * len(idx) if per_ray else keep.sum()

        N = len(o)
        # the prepare batches: 64 consecutive samples (4 pixels x 16 spp); their live lanes run
        # the first bounce together (lanes that ended at the primary hit idle)
        item = np.nonzero(live)[0]
        for bstart in range(0, TP * SPP, 64):
            sel = np.nonzero((item >= bstart) & (item < bstart + 64))[0]
            if len(sel) == 0:
                continue
            az_b = np.arctan2(nd[sel] @ np.cross(nd[sel].mean(0), [0.3, 1, 0.1]),
                              nd[sel] @ np.cross(np.cross(nd[sel].mean(0), [0.3, 1, 0.1]), nd[sel].mean(0)))
            ordb = sel[np.argsort(az_b)]
            for G, key in ((1, "batch_g1"), (2, "batch_g2"), (4, "batch_g4"), (8, "batch_g8")):
                gs = np.array_split(ordb, G)
                tot[key] += 64 * max(cull_count(g, False) for g in gs if len(g))
            tot["batch_g1_2s"] += 64 * cull_count(sel, False, True)
        for k in range(0, N, 64):
            tot["order"] += cull_count(np.arange(k, min(N, k + 64)))
        # group by direction: sort by (octant around the mean axis) — simple: by azimuth
        a = nd.mean(0)
        a /= np.linalg.norm(a)
        e1 = np.cross(a, [0.3, 1.0, 0.1]); e1 /= np.linalg.norm(e1)
        e2 = np.cross(a, e1)
        az = np.arctan2(nd @ e2, nd @ e1)
        el = nd @ a
        order = np.lexsort((el, az))
        for k in range(0, N, 64):
            tot["sorted4"] += cull_count(order[k:k + 64])
        # k-means-ish: sort by elevation bands then azimuth inside
        key = np.floor((el + 1) * 1.0) * 10 + az
        order = np.argsort(key)
        for k in range(0, N, 64):
            tot["sorted_oct"] += cull_count(order[k:k + 64])
    print(f"first-bounce rays sampled: {nb}")
    for k, v in tot.items():
        print(f"{k:10s}: {v / max(nb, 1):6.2f} lane-tests per ray")


if __name__ == "__main__":
    main()
