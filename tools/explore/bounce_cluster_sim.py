#!/usr/bin/env python
"""CPU estimate (numpy, float64, no GPU) of what hierarchical culling could skip in the AO
kernel's later bounce rounds at config (d): for waves of 64 later-bounce rays (segments >= 3,
as the kernel's full rounds hold them: the paths of one pool), the fraction of spheres some
lane's LINE meets (del >= 0: the hit tail runs; DESIGN §5 measures 5.3%), and the fraction of
spatial clusters (k-means groups of ~C spheres, bounding sphere inflated by nothing) that some
lane's ray may hit — the spheres a cluster cull would still have to test.

    python tools/explore/bounce_cluster_sim.py [--pools 300] [--cluster 8]
"""
import argparse
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
from bench import CONFIGS, config_header  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pools", type=int, default=300)
    ap.add_argument("--cluster", type=int, default=8)
    ap.add_argument("--config", default="d")
    a = ap.parse_args()
    W, H, S, spp, mode, _ = CONFIGS[a.config]
    h = config_header(a.config)
    n = h.num_objects
    sh = h.shapes[:n].astype(np.float64)
    C, R = sh[:, 0, :3], sh[:, 0, 3]
    col_emis = sh[:, 1, 3] > 0.9
    refl = sh[:, 3, 3]
    hv = lambda i: h.vec4(i)[:3].astype(np.float64)  # noqa: E731
    hor, ver, llc, cam = hv(1), hv(2), hv(3), hv(4)
    rng = np.random.default_rng(1)
    rays = []  # (pool, seg, pos, dir) of segments >= 3
    for p in range(a.pools):
        y = rng.integers(0, H)
        x0 = rng.integers(0, W // 16) * 16
        px = np.repeat(np.arange(x0, x0 + 16), spp) + rng.uniform(-0.08, 0.08, 16 * spp)
        py = y + rng.uniform(-0.08, 0.08, 16 * spp)
        d = llc + np.outer(px / W, hor) + np.outer(py / H, ver)
        d /= np.linalg.norm(d, axis=1, keepdims=True)
        hemi = rng.normal(size=(16 * spp, 3))
        hemi /= np.linalg.norm(hemi, axis=1, keepdims=True)
        pos = np.repeat(cam[None], 16 * spp, 0)
        live = np.ones(16 * spp, bool)
        for seg in range(20):
            pmc = pos[:, None, :] - C[None]
            b = np.einsum("kj,kij->ki", d, pmc)
            dl = R[None] ** 2 + b * b - np.einsum("kij,kij->ki", pmc, pmc)
            s = np.sqrt(np.maximum(dl, 0))
            t2, t1 = -b - s, -b + s
            t = np.where(t2 > 1e-4, t2, np.where(t1 > 1e-4, t1, np.inf))
            t[dl < 0] = np.inf
            ind = np.argmin(t, 1)
            tt = t[np.arange(len(t)), ind]
            if seg >= 2:
                for k in np.nonzero(live)[0]:
                    rays.append((p, seg, pos[k].copy(), d[k].copy()))
            hit = live & np.isfinite(tt)
            live = hit & ~col_emis[ind]
            curr = cam + tt[:, None] * d  # camera origin (ao_compute.glsl:210)
            nn = curr - C[ind]
            nn /= np.linalg.norm(nn, axis=1, keepdims=True)
            rf = refl[ind]
            Rr = d - 2 * np.einsum("kj,kj->k", d, nn)[:, None] * nn
            X = np.where((rf > 0.999)[:, None], hemi + nn, Rr + rf[:, None] * hemi)
            X /= np.linalg.norm(X, axis=1, keepdims=True)
            d = np.where(live[:, None], X, d)
            pos = np.where(live[:, None], curr, pos)
            if not live.any():
                break
    # waves: consecutive rays of one pool, 64 at a time
    by_pool = {}
    for p, seg, o, d in rays:
        by_pool.setdefault(p, []).append((o, d))
    # clusters: k-means on the small spheres; the huge ground sphere alone
    small = np.nonzero(R < 10)[0]
    k = max(1, len(small) // a.cluster)
    cen = C[small][rng.choice(len(small), k, replace=False)]
    for _ in range(50):
        lab = np.argmin(((C[small][:, None] - cen[None]) ** 2).sum(-1), 1)
        cen = np.array([C[small][lab == j].mean(0) if (lab == j).any() else cen[j] for j in range(k)])
    crad = np.array([max(np.linalg.norm(C[small][lab == j] - cen[j], axis=1) + R[small][lab == j]) if (lab == j).any() else 0
                     for j in range(k)])
    csize = np.bincount(lab, minlength=k)
    sph_frac, clu_frac, tested = [], [], []
    for p, lst in by_pool.items():
        for i in range(0, len(lst) - 63, 64):
            o = np.array([x[0] for x in lst[i:i + 64]])
            d = np.array([x[1] for x in lst[i:i + 64]])
            pmc = o[:, None] - C[None]
            b = np.einsum("kj,kij->ki", d, pmc)
            dl = R[None] ** 2 + b * b - np.einsum("kij,kij->ki", pmc, pmc)
            sph_frac.append((dl >= 0).any(0).mean())
            pmc = o[:, None] - cen[None]
            b = np.einsum("kj,kij->ki", d, pmc)
            dl = crad[None] ** 2 + b * b - np.einsum("kij,kij->ki", pmc, pmc)
            # forward-only: a cluster entirely behind an origin outside it cannot be hit
            inside = np.einsum("kij,kij->ki", pmc, pmc) < crad[None] ** 2
            ahead = (-b + np.sqrt(np.maximum(dl, 0))) > 0
            hitc = (dl >= 0) & (inside | ahead)
            anyc = hitc.any(0)
            clu_frac.append(anyc.mean())
            tested.append((csize[anyc].sum() + (n - len(small))) / n)
    print(f"config {a.config}: {len(rays)} later-bounce rays, {len(sph_frac)} full waves")
    print(f"spheres some lane's line meets (del >= 0): {np.mean(sph_frac):.3f}")
    print(f"clusters of ~{a.cluster} (k = {k}, mean bounding radius {crad.mean():.2f}) some lane may hit: "
          f"{np.mean(clu_frac):.3f}; spheres left to test: {np.mean(tested):.3f} of {n}")


if __name__ == "__main__":
    main()
