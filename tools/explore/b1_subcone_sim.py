#!/usr/bin/env python
"""Sector sub-cones for the first bounce (model): the batch's rays split into k sectors around the cone
axis, one cone each; prints the one-cone survivors per batch and the sum over the k sector cones.

    python tools/explore/b1_subcone_sim.py <config> <rows> <k>
"""
import sys, numpy as np
from pathlib import Path
ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT)); sys.path.insert(0, str(ROOT / 'tools/explore'))
import b1_pairs_sim as S
from bench import CONFIGS, config_header
from oracle import numpy_ref as nr
from real_time_ray_tracer_amd import SSBO
cfg = sys.argv[1]; rows = int(sys.argv[2]); k = int(sys.argv[3])
W, H, Sn, spp, mode, _ = CONFIGS[cfg]
h = config_header(cfg); h.fill_rand_buffer(7000); h.set_mode(0, h.num_objects)
s = SSBO(h, 4, 4, num_frames=1); fr = nr.Frame(s.data, 4, 4, h.S, h.AA, F_=1); fr.W, fr.H = W, H
geo = fr.shapes[:fr.nobj, 0]
def keep_count(P, Dn, L):
    # cone-kept spheres for one group: P, Dn [B,64,3], L [B,64]
    B = P.shape[0]
    ok = L.sum(1) >= 1
    first = np.argmax(L, 1); o = P[np.arange(B), first]
    e2 = np.where(L, ((P - o[:, None]) ** 2).sum(2), 0).max(1)
    sm = np.where(L[..., None], Dn, 0).sum(1)
    rho = np.sqrt(e2) * 1.0001 + 1e-6 * np.abs(o).sum(1)
    s2 = (sm ** 2).sum(1); ax = sm / np.sqrt(np.maximum(s2, 1e-30))[:, None]
    ct = np.where(L, (Dn * ax[:, None]).sum(2), 1.0).min(1) - 2e-5
    ct = np.clip(np.where(s2 > 1e-6, ct, -1.0), -1, 1); st = np.sqrt(np.maximum(0, 1 - ct * ct))
    n = np.zeros(B)
    for j in range(geo.shape[0]):
        c, r = geo[j, :3].astype(np.float64), abs(float(geo[j, 3]))
        v = c - o; Ln = np.sqrt((v ** 2).sum(1)); Lmax = Ln + rho
        near = ~((Ln - rho - r) > 1e-2 * Lmax)
        R = np.sqrt(r * r + 1e-5 * (Lmax ** 2 + r * r)) * 1.00001 + rho
        sa = R / Ln; ca = np.sqrt(np.maximum(0, 1 - sa * sa)); u = v / Ln[:, None]
        cover = ~(st * ca + ct * sa > 1e-5); Kc = ct * ca - st * sa - 2e-5
        keep = near | cover | ~((ax * u).sum(1) < Kc)
        n += keep & ok
    return n
rng = np.random.default_rng(5)
tot1 = totk = nb = 0
for y in rng.choice(H, rows, replace=False):
    P, Dn, L = S.first_bounce_states(fr, int(y))
    B = P.shape[0] // 64
    P, Dn, L = P[:B*64].reshape(B, 64, 3), Dn[:B*64].reshape(B, 64, 3), L[:B*64].reshape(B, 64)
    okb = L.sum(1) >= 1
    n1 = keep_count(P, Dn, L)
    # k groups: by angle around the batch axis (sectors of the tangent plane)
    sm = np.where(L[..., None], Dn, 0).sum(1); ax = sm / np.maximum(np.linalg.norm(sm, axis=1), 1e-30)[:, None]
    e1 = np.cross(ax, np.array([0.3, 0.9, 0.1])); e1 /= np.maximum(np.linalg.norm(e1, axis=1), 1e-30)[:, None]
    e2v = np.cross(ax, e1)
    ang = np.arctan2((Dn * e2v[:, None]).sum(2), (Dn * e1[:, None]).sum(2))
    grp = np.floor((ang + np.pi) / (2 * np.pi) * k).astype(int) % k
    nk = np.zeros(B)
    for g in range(k):
        nk += keep_count(P, Dn, L & (grp == g))
    tot1 += n1[okb].sum(); totk += nk[okb].sum(); nb += okb.sum()
print(f"{cfg}: one cone {tot1/nb:.1f} survivors per batch; {k} sector cones, sum of their survivors {totk/nb:.1f}")
