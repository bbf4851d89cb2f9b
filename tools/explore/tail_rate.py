#!/usr/bin/env python
"""Exploration (float64, statistics only — not parity): for the first-bounce batches of
config (d) (64 consecutive samples = 4 pixels x 16 spp, live lanes only), how often does a
sphere that survives the batch's bounce cone get its hit tail run (some lane with del >= 0),
how many lanes meet it, and how often would a per-batch angular pre-test (each sphere's
cone of directions seen from the batch origin ball) pass on some lane?  Also the same
tail rate for incoherent rays against the whole table (the later bounce rounds).

    python tools/explore/tail_rate.py [npools]
"""
import sys

import numpy as np

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from real_time_ray_tracer_amd.host import Header, aspect_for  # noqa: E402

W, H, S, SPP = 3840, 2160, 64, 16
TP = 256 // SPP


def main():
    npools = int(sys.argv[1]) if len(sys.argv) > 1 else 1500
    h = Header.synthetic(S, SPP, 1234 + 3, aspect_for(W, H))
    d = h.data.astype(np.float64)
    hor, ver, llc, cam = d[4:7], d[8:11], d[12:15], d[16:19]
    sh = h.shapes.astype(np.float64)
    C, R = sh[:, 0, :3], sh[:, 0, 3]
    emis, refl = sh[:, 1, 3] > 0.9, sh[:, 3, 3]
    rng = np.random.default_rng(1)
    pools = rng.integers(0, W * H // TP, npools)
    st = dict(batches=0, cand=0, tail=0, lanes_hit=0, pre=0, pre_lanes=0, live=0)
    later = dict(iters=0, tail=0, lanes=0)
    later_o, later_d = [], []
    for p in pools:
        pix = p * TP + np.arange(TP)
        x, y = (pix % W).astype(np.float64), (pix // W).astype(np.float64)
        x = np.repeat(x, SPP) + rng.uniform(-0.083, 0.083, TP * SPP)
        y = np.repeat(y, SPP) + rng.uniform(-0.083, 0.083, TP * SPP)
        dirs = llc + (x / W)[:, None] * hor + (y / H)[:, None] * ver
        dirs /= np.linalg.norm(dirs, axis=1)[:, None]
        pmc = cam - C
        b = dirs @ pmc.T
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
        item = np.nonzero(live)[0]
        ind, tm, dr = ind[live], tm[live], dirs[live]
        o = cam + tm[:, None] * dr
        n = o - C[ind]
        n /= np.linalg.norm(n, axis=1)[:, None]
        u = rng.uniform(-1, 1, size=(len(o), 3))
        u /= np.linalg.norm(u, axis=1)[:, None]
        rf = refl[ind][:, None]
        Rv = dr - 2 * (dr * n).sum(1)[:, None] * n
        Rv /= np.linalg.norm(Rv, axis=1)[:, None]
        nd = np.where(rf > 0.999, n + u, Rv + rf * u)
        nd /= np.linalg.norm(nd, axis=1)[:, None]
        for bstart in range(0, TP * SPP, 64):
            sel = np.nonzero((item >= bstart) & (item < bstart + 64))[0]
            if len(sel) == 0:
                continue
            oo, dd = o[sel], nd[sel]
            oc = oo[0]
            rho = np.linalg.norm(oo - oc, axis=1).max()
            a = dd.sum(0)
            a /= max(np.linalg.norm(a), 1e-30)
            th = np.arccos(np.clip((dd @ a).min(), -1, 1))
            v = C - oc
            L = np.linalg.norm(v, axis=1)
            Rp = R + rho
            inside = L - rho - R <= 1e-2 * (L + rho)
            al = np.arcsin(np.clip(Rp / np.maximum(L, 1e-30), 0, 1))
            be = np.arccos(np.clip((v @ a) / np.maximum(L, 1e-30), -1, 1))
            keep = inside | (be <= th + al)
            st["batches"] += 1
            st["live"] += len(sel)
            st["cand"] += keep.sum()
            # exact discriminant per (ray, candidate)
            pm = oo[:, None, :] - C[None, keep, :]
            bb = (dd[:, None, :] * pm).sum(2)
            de = bb * bb - (pm * pm).sum(2) + R[keep] ** 2
            hit = de >= 0
            st["tail"] += hit.any(0).sum()
            st["lanes_hit"] += hit.sum()
            # angular pre-test: direction within the sphere's angular radius (+ rho) from oc
            va = v[keep] / L[keep, None]
            cal = np.cos(np.minimum(al[keep] * 1.0 + 1e-3, np.pi))
            pre = ((dd @ va.T) >= cal[None, :]) | inside[keep][None, :]
            st["pre"] += pre.any(0).sum()
            st["pre_lanes"] += pre.sum()
            # continue the paths that hit something non-emissive: later-bounce rays
            tt = np.where(hit, -bb - np.sqrt(np.maximum(de, 0)), np.inf)
            tt = np.where(tt > 1e-4, tt, np.where(hit & (-bb + np.sqrt(np.maximum(de, 0)) > 1e-4),
                                                  -bb + np.sqrt(np.maximum(de, 0)), np.inf))
            j = tt.argmin(1)
            tj = tt[np.arange(len(j)), j]
            ok = np.isfinite(tj)
            kidx = np.nonzero(keep)[0][j]
            ok &= ~emis[kidx]
            if ok.any():
                o2 = cam + tj[ok, None] * dd[ok]  # sic: camera origin (ao_compute.glsl:210)
                n2 = o2 - C[kidx[ok]]
                n2 /= np.linalg.norm(n2, axis=1)[:, None]
                u2 = u[sel][ok]
                rf2 = refl[kidx[ok]][:, None]
                R2 = dd[ok] - 2 * (dd[ok] * n2).sum(1)[:, None] * n2
                R2 /= np.linalg.norm(R2, axis=1)[:, None]
                d2 = np.where(rf2 > 0.999, n2 + u2, R2 + rf2 * u2)
                d2 /= np.linalg.norm(d2, axis=1)[:, None]
                later_o.append(o2)
                later_d.append(d2)
    print(f"batches {st['batches']}, live lanes/batch {st['live'] / st['batches']:.1f}")
    print(f"B1 candidates/batch {st['cand'] / st['batches']:.2f}; tail runs on {st['tail'] / st['cand']:.3f} of them; "
          f"lanes with del>=0 per candidate {st['lanes_hit'] / st['cand']:.2f}")
    print(f"angular pre-test passes on some lane for {st['pre'] / st['cand']:.3f} of candidates; "
          f"lanes passing per candidate {st['pre_lanes'] / st['cand']:.2f}")
    O, Dd = np.concatenate(later_o), np.concatenate(later_d)
    perm = rng.permutation(len(O))
    O, Dd = O[perm], Dd[perm]
    n64 = len(O) // 64
    tails = 0
    lanes = 0
    for k in range(n64):
        oo, dd = O[64 * k:64 * k + 64], Dd[64 * k:64 * k + 64]
        pm = oo[:, None, :] - C[None]
        bb = (dd[:, None, :] * pm).sum(2)
        de = bb * bb - (pm * pm).sum(2) + R ** 2
        tails += (de >= 0).any(0).sum()
        lanes += (de >= 0).sum()
    print(f"later bounces (random 64-ray waves, all {S} spheres): tail runs on {tails / (n64 * S):.3f} of sphere "
          f"iterations; lanes with del>=0 per iteration {lanes / (n64 * S):.2f}")


if __name__ == "__main__":
    main()
