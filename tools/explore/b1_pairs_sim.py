#!/usr/bin/env python
"""How many exact-test passes does the batched first bounce of ao_batch_kernel run per prepared
batch (64 samples: 4 pixels x 16 spp), as built (RT_B1_DEFER: survivors with disjoint pre-test
masks merged, each lane holding one pending sphere) and if every (ray, sphere) pair that passes
the pre-test were packed into full-wave passes of 64 pairs (a pair list, flushed when the next
survivor's pairs would not fit)?  A float64 numpy model of the kernel's batch cone
(bounce_cone), its per-sphere cull and pre-test rows (bounce_cone_keep_pt) and the pre-test
itself, on sampled rows of a config's first frame; counts only, no parity claim.

    python tools/explore/b1_pairs_sim.py --config d --rows 24
"""
from __future__ import annotations

import argparse
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))

from bench import CONFIGS, config_header  # noqa: E402
from oracle import numpy_ref as nr  # noqa: E402
from real_time_ray_tracer_amd import SSBO  # noqa: E402

F = np.float32


def first_bounce_states(fr: nr.Frame, y: int):
    """Per sample of row y (x-major, then aa): origin and direction of the first bounce, live."""
    W, AA = fr.W, fr.AA
    x = np.arange(W)
    px, py = x.astype(F), np.full(W, y, F)
    cam = fr.hdr[4, :3]
    P = np.zeros((W, AA, 3)); Dn = np.zeros((W, AA, 3)); L = np.zeros((W, AA), bool)
    for aa in range(AA):
        fst, snd = fr.rb[2 * aa], fr.rb[2 * aa + 1]
        if aa == 0:
            dirs = fr.primary(x, np.full(W, y))
        else:
            s1, s2, s3, s4 = (snd[0], fst[1]), (fst[2], snd[3]), (fst[0], snd[1]), (snd[2], fst[3])
            u = nr.grandom(((s1[0] + px * s2[0]) - px) + s3[0], ((s1[1] + py * s2[1]) - py) + s3[1])
            w = nr.grandom(s4[0] * px - (s3[0] * px) * s2[0], s4[1] * py - (s3[1] * py) * s2[1])
            il = F(1.0) / np.sqrt(nr.fma(w, w, u * u))
            dirs = fr.primary(x, np.full(W, y), (u * il) / F(6.0) - F(0.08333), (w * il) / F(6.0) - F(0.08333))
        a = nr.grandom(fst[0] + px * snd[2], fst[1] + py * snd[3])
        b = nr.grandom(fst[2] - px * snd[2], fst[3] - py * snd[3])
        e = nr.grandom(snd[0] * px + snd[2], snd[1] * py + snd[3])
        hemi = nr.normalize3(np.stack([a * F(2) - F(1), b * F(2) - F(1), e * F(2) - F(1)], 1))
        pos = np.broadcast_to(cam, (W, 3)).astype(F)
        t, ind = fr.closest(pos, dirs, 0.0001)
        hit = ind >= 0
        emis = np.zeros(W, bool)
        emis[hit] = fr.shapes[ind[hit], 1, 3] > F(0.9)
        cont = hit & ~emis
        ci = np.nonzero(cont)[0]
        if ci.size:
            curr = cam + t[ci, None] * dirs[ci]
            nn = fr.normal(ind[ci], curr)
            refl = fr.shapes[ind[ci], 3, 3]
            diffuse = refl > F(0.999)
            nd = np.empty_like(nn)
            nd[diffuse] = nr.normalize3(hemi[ci[diffuse]] + nn[diffuse])
            gl = ~diffuse
            if gl.any():
                dg = dirs[ci[gl]]
                dn = nr.dot3(dg, nn[gl])
                R = nr.normalize3(dg - F(2.0) * (dn[:, None] * nn[gl]))
                nd[gl] = nr.normalize3(R + refl[gl, None] * hemi[ci[gl]])
            P[ci, aa] = curr
            Dn[ci, aa] = nd
            L[ci, aa] = True
    return P.reshape(-1, 3), Dn.reshape(-1, 3), L.reshape(-1)


def batch_masks(P, Dn, L, geo):
    """[B, S] uint64 pre-test pass masks of the survivors (0 for culled spheres), B batches of 64."""
    B = P.shape[0] // 64
    P, Dn, L = P[:B * 64].reshape(B, 64, 3), Dn[:B * 64].reshape(B, 64, 3), L[:B * 64].reshape(B, 64)
    keepb = L.sum(1) >= 1
    first = np.argmax(L, 1)
    o = P[np.arange(B), first]
    e2 = np.where(L, ((P - o[:, None]) ** 2).sum(2), 0).max(1)
    s = np.where(L[..., None], Dn, 0).sum(1)
    rho = np.sqrt(e2) * 1.0001 + 1e-6 * np.abs(o).sum(1)
    s2 = (s ** 2).sum(1)
    ax = s / np.sqrt(np.maximum(s2, 1e-30))[:, None]
    ct = np.where(L, (Dn * ax[:, None]).sum(2), 1.0).min(1) - 2e-5
    ct = np.where(s2 > 1e-6, ct, -1.0)
    ct = np.clip(ct, -1.0, 1.0)
    st = np.sqrt(np.maximum(0.0, 1 - ct * ct))
    S = geo.shape[0]
    masks = np.zeros((B, S), np.uint64)
    nkeep = np.zeros(B, np.int64)
    keepm = np.zeros((B, S), bool)
    bits = (np.uint64(1) << np.arange(64, dtype=np.uint64))
    for j in range(S):
        c, r = geo[j, :3].astype(np.float64), abs(float(geo[j, 3]))
        v = c - o
        Ln = np.sqrt((v ** 2).sum(1))
        Lmax = Ln + rho
        near = ~((Ln - rho - r) > 1e-2 * Lmax)
        R = np.sqrt(r * r + 1e-5 * (Lmax ** 2 + r * r)) * 1.00001 + rho
        sa = R / Ln
        ca = np.sqrt(np.maximum(0.0, 1 - sa * sa))
        u = v / Ln[:, None]
        K = np.where(sa < 1.0, ca - 2e-5, -2.0)
        cover = ~(st * ca + ct * sa > 1e-5)
        Kc = ct * ca - st * sa - 2e-5
        keep = near | cover | ~((ax * u).sum(1) < Kc)
        K = np.where(near, -2.0, K)
        u = np.where(near[:, None], 0.0, u)
        pas = ((Dn * u[:, None]).sum(2) >= K[:, None]) & L
        m = (pas * bits).sum(1, dtype=np.uint64)
        masks[:, j] = np.where(keep & keepb, m, 0)
        nkeep += keep & keepb
        keepm[:, j] = keep & keepb
    return masks, keepb, L.sum(1), nkeep, keepm


def build_clusters(geo, size):
    """rt_shim.hip build_clusters: recursive median splits of the centres along the widest axis
    into groups of <= size; (centre, R) with every member inside (float64 here)."""
    idx = list(range(geo.shape[0]))
    work, groups = [(0, len(idx))], []
    while work:
        a, b = work.pop()
        if b - a <= size:
            groups.append(idx[a:b])
            continue
        c = geo[idx[a:b], :3].astype(np.float64)
        ax = int(np.argmax(c.max(0) - c.min(0)))
        mid = (a + b) // 2
        part = sorted(idx[a:b], key=lambda i: (float(geo[i, ax]), i))
        idx[a:b] = part
        work.append((mid, b))
        work.append((a, mid))
    out = []
    for g in groups:
        c = geo[g, :3].astype(np.float64).mean(0)
        R = max(np.linalg.norm(geo[i, :3] - c) + abs(float(geo[i, 3])) for i in g)
        out.append((np.array(g), c, R))
    return out


def cluster_pretest(P, Dn, L, geo, clusters):
    """Per batch: the clusters whose ball some live lane's pre-test passes (the same pre-test as a
    sphere's, on the ball inflated to R sqrt(1+1e-5) + sqrt(1e-5) Lmax + rho), and the cone-kept
    spheres that lie in such clusters."""
    B = P.shape[0] // 64
    P, Dn, L = P[:B * 64].reshape(B, 64, 3), Dn[:B * 64].reshape(B, 64, 3), L[:B * 64].reshape(B, 64)
    first = np.argmax(L, 1)
    o = P[np.arange(B), first]
    e2 = np.where(L, ((P - o[:, None]) ** 2).sum(2), 0).max(1)
    rho = np.sqrt(e2) * 1.0001 + 1e-6 * np.abs(o).sum(1)
    member_pass = np.zeros((B, geo.shape[0]), bool)
    npass = np.zeros(B, np.int64)
    for g, c, R in clusters:
        v = c - o
        Ln = np.sqrt((v ** 2).sum(1))
        Lmax = Ln + R + rho
        Re = R * np.sqrt(1 + 1e-5) * 1.0001 + np.sqrt(1e-5) * Lmax * 1.0001 + rho
        sa = Re / Ln
        near = ~(sa < 1.0)
        ca = np.sqrt(np.maximum(0.0, 1 - sa * sa))
        u = v / Ln[:, None]
        K = np.where(near, -2.0, ca - 2e-5)
        pas = (((Dn * u[:, None]).sum(2) >= K[:, None]) & L).any(1)
        npass += pas
        member_pass[:, g] = pas[:, None]
    return member_pass, npass


def count(masks, cap=64):
    B, S = masks.shape
    ru = np.zeros(B, np.uint64)
    defer = np.zeros(B, np.int64)
    npair = np.zeros(B, np.int64)
    packed = np.zeros(B, np.int64)
    pairs = np.zeros(B, np.int64)
    passing = np.zeros(B, np.int64)
    for j in range(S):
        pm = masks[:, j]
        on = pm != 0
        ov = on & ((pm & ru) != 0)
        defer += ov
        ru = np.where(ov, np.uint64(0), ru) | pm
        c = np.bitwise_count(pm).astype(np.int64)
        full = on & (npair + c > cap)
        packed += full
        npair = np.where(full, 0, npair) + c
        pairs += c
        passing += on
    defer += ru != 0
    packed += npair > 0
    return defer, packed, pairs, passing


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="d")
    ap.add_argument("--rows", type=int, default=24)
    ap.add_argument("--seed", type=int, default=5)
    a = ap.parse_args()
    W, H, S, spp, mode, _ = CONFIGS[a.config]
    h = config_header(a.config)
    h.fill_rand_buffer(7000)
    h.set_mode(0, h.num_objects)
    s = SSBO(h, 4, 4, num_frames=1)
    fr = nr.Frame(s.data, 4, 4, h.S, h.AA, F_=1)  # (no g-buffer: the primary rays use W, H only)
    fr.W, fr.H = W, H
    geo = fr.shapes[:fr.nobj, 0]
    rows = np.random.default_rng(a.seed).choice(H, a.rows, replace=False)
    tot = dict(batches=0, b1=0, defer=0, packed=0, pairs=0, passing=0, live=0, kept=0, ckept=0, cpass=0, nclus=0)
    csize = max(8, int(np.ceil(np.sqrt(geo.shape[0]))))
    clusters = build_clusters(geo, csize)
    for y in rows:
        P, Dn, L = first_bounce_states(fr, int(y))
        masks, keepb, nl, nk, km = batch_masks(P, Dn, L, geo)
        tot["kept"] += int(nk.sum())
        mp, npc = cluster_pretest(P, Dn, L, geo, clusters)
        kept_sph = (masks != 0)  # (survivors some lane passes are a subset of the cone-kept ones)
        # cone-kept spheres in passing clusters: recount the cone keep per sphere from batch_masks' nk
        tot["cpass"] += int(npc[keepb].sum())
        tot["nclus"] += len(clusters) * int(keepb.sum())
        tot["ckept"] += int((mp[keepb] & km[keepb]).sum())
        tot["miss"] = tot.get("miss", 0) + int((kept_sph[keepb] & ~mp[keepb]).sum())
        d, p, q, ps = count(masks[keepb])
        tot["batches"] += masks.shape[0]
        tot["b1"] += int(keepb.sum())
        tot["defer"] += int(d.sum()); tot["packed"] += int(p.sum())
        tot["pairs"] += int(q.sum()); tot["passing"] += int(ps.sum()); tot["live"] += int(nl.sum())
    b = max(tot["b1"], 1)
    print(f"config {a.config}, {a.rows} rows: {tot['batches']} batches, {tot['b1']} with a first bounce, "
          f"{tot['live'] / b:.1f} live lanes each")
    print(f"per first-bounce batch: cone-cull survivors {tot['kept'] / b:.2f} of {geo.shape[0]}, "
          f"survivors passed by some lane {tot['passing'] / b:.2f}, "
          f"(ray, sphere) pairs {tot['pairs'] / b:.1f}")
    print(f"clusters of <= {csize}: {len(clusters)}, of which some lane's ball pre-test passes {tot['cpass'] / b:.2f} "
          f"per batch; cone survivors inside them {tot['ckept'] / b:.2f} (loop iterations after the cluster pre-test); "
          f"passing survivors outside them (must be 0): {tot.get('miss', 0)}")
    print(f"exact-test passes per batch: merged as built (RT_B1_DEFER) {tot['defer'] / b:.2f}, "
          f"packed 64-pair passes {tot['packed'] / b:.2f}")


if __name__ == "__main__":
    main()
