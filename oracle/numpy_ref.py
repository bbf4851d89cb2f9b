"""Independent numpy restatement of the five compute shaders.  TEST INFRASTRUCTURE ONLY.

Written from the GLSL (not from rt_oracle.c) to cross-check the C oracle on small frames:
vectorised over pixels (and over pixels for each AO sample, samples in order), binary32
arithmetic with fmaf emulated through binary64 (a*b is exact in binary64; the single
rounding of the sum to binary64 then binary32 can differ from a true fmaf only on a
double-rounding tie, ~2^-29 per operation).  shadow_ray's binary64 length uses plain binary64
operations (numpy has no binary64 fma), so it may differ from the oracle's fused form in the
last ulp.  The float semantics follow oracle/rt_oracle.h.  Parity unpinned by reference
artifacts (the reference has none).

Citations: resources/p_compute.glsl:65-245, h_compute.glsl:168-321, ao_compute.glsl:143-339,
aop_compute.glsl:141-336, aop_postprocessing.glsl:57-208; dispatch src/main.cpp:553-671.
"""
from __future__ import annotations

import numpy as np

F = np.float32
D64 = np.float64

AOP_COMPUTE, AOP_POSTPROCESSING, AO_COMPUTE, P_COMPUTE, H_COMPUTE = 1, 2, 3, 4, 5
GAMMA = F(1.0) / F(2.2)  # p_compute.glsl:240


def fma(a, b, c):
    a, b, c = np.broadcast_arrays(np.asarray(a, F), np.asarray(b, F), np.asarray(c, F))
    return (a.astype(D64) * b.astype(D64) + c.astype(D64)).astype(F)


def dot3(a, b):
    return fma(a[..., 2], b[..., 2], fma(a[..., 1], b[..., 1], a[..., 0] * b[..., 0]))


def normalize3(v):
    il = F(1.0) / np.sqrt(dot3(v, v))
    return v * il[..., None]


def clamp(x, lo, hi):  # GLSL min(max(x, lo), hi) with GLSL's NaN-agnostic definitions
    m = np.where(x < lo, F(lo), x)
    return np.where(F(hi) < m, F(hi), m).astype(F)


def det_sin(x):
    """sin() inside random(): the plain binary64 re-execution, (float)sin((double)x) with numpy's
    (glibc's) sin.  The C oracle and the kernels compute the correctly rounded binary32 sin,
    which this equals except at the rare double-rounding inputs (tests/test_oracle_cpu.py lists
    and arbitrates them with mpmath)."""
    x = np.asarray(x, F)
    with np.errstate(invalid="ignore"):
        return np.sin(x.astype(np.float64)).astype(F)


# Contraction of random()'s argument arithmetic (the GLSL leaves a*b+c to the compiler): the
# same flags as the C oracle's rto_set_contraction.  0 = the kernels' semantics (dot() inside
# random() fused, the seed / jitter sums as written).  C_UNFUSED_DOT = ao_compute.glsl:63-73
# read literally (both products rounded, then the sum): this restatement's own, independent
# form on this axis.  C_FUSED_SEEDS / C_FUSED_JITTER: the seed sums of ao_compute.glsl:152-157 /
# 317-319 contracted as a GLSL compiler does by default.
C_UNFUSED_DOT, C_FUSED_SEEDS, C_FUSED_JITTER = 1, 2, 4
CONTRACTION = 0


def grandom(sx, sy):
    if CONTRACTION & C_UNFUSED_DOT:
        d = (np.asarray(sx, F) * F(12.9898) + np.asarray(sy, F) * F(78.233)).astype(F)
    else:
        d = fma(sy, F(78.233), np.asarray(sx, F) * F(12.9898))
    m = det_sin(d) * F(43758.5453123)
    return (m - np.floor(m)).astype(F)


class Frame:
    """Views of a reference-layout SSBO (header, shapes, rand_buffer, g-buffer [F][W][H])."""

    def __init__(self, ssbo: np.ndarray, W: int, H: int, S: int, AA: int, F_: int = 8, D: int = 20):
        self.ssbo, self.W, self.H, self.S, self.AA, self.F, self.D = ssbo, W, H, S, AA, F_, D
        self.hdr = ssbo[:28].reshape(7, 4)
        self.shapes = ssbo[28:28 + 20 * S].reshape(S, 5, 4)
        o = 28 + 20 * S
        self.rb = ssbo[o:o + 8 * AA].reshape(2 * AA, 4)
        o += 8 * AA
        n = F_ * W * H * 4
        self.pix = ssbo[o:o + n].reshape(F_, W, H, 4)
        self.nrm = ssbo[o + n:o + 2 * n].reshape(F_, W, H, 4)
        self.dep = ssbo[o + 2 * n:o + 3 * n].reshape(F_, W, H, 4)
        self.nobj = int(self.hdr[0, 2])
        self.frame = int(self.hdr[0, 1])

    # ---- intersection, p_compute.glsl:77-138 ----
    def eval_ray(self, pos, dirs, i):
        sh = self.shapes[i]
        sid = int(sh[4, 3])
        n = pos.shape[0]
        if sid == 1:
            c, r = sh[0, :3], sh[0, 3]
            pmc = pos - c
            b = dot3(dirs, pmc)
            dl = fma(np.full(n, r, F), np.full(n, r, F), fma(b, b, -dot3(pmc, pmc)))
            res = np.full(n, F(-1.0))
            zero = dl == 0
            res[zero] = -b[zero]
            g = ~(dl < 0) & ~zero
            s = np.sqrt(dl[g])
            t1 = -b[g] + s
            t2 = -b[g] - s
            res[g] = np.where(t2 < 0, np.where(t1 < 0, F(-1.0), t1), t2)
            return res
        if sid == 5:
            nv = sh[0, :3]
            den = dot3(np.broadcast_to(nv, dirs.shape), dirs)
            with np.errstate(divide="ignore", invalid="ignore"):
                res = (dot3(np.broadcast_to(nv, pos.shape), sh[3, :3] - pos) / den).astype(F)
            return np.where((den < F(0.001)) & (den > F(-0.001)), F(-1.0), res)
        return np.full(n, F(-1.0))

    def closest(self, pos, dirs, thr):
        t = np.full(pos.shape[0], F(-1.0))
        ind = np.full(pos.shape[0], -1)
        for i in range(self.nobj):
            res = self.eval_ray(pos, dirs, i)
            upd = (res > F(thr)) & ((res < t) | (t < 0))
            t = np.where(upd, res, t)
            ind = np.where(upd, i, ind)
        return t, ind

    def normal(self, ind, p):
        sid = self.shapes[ind, 4, 3].astype(np.int64)
        c = self.shapes[ind, 0, :3]
        return np.where((sid == 1)[:, None], normalize3(p - c), c)

    def shadow_lit(self, pos):  # p_compute.glsl:145-166
        light = self.hdr[5, :3]
        lv = light - pos
        l = normalize3(lv)
        ln = np.sqrt(dot3(lv, lv))
        npos = pos + F(0.01) * l
        lit = np.ones(pos.shape[0], bool)
        for i in range(self.nobj):
            t = self.eval_ray(npos, l, i).astype(D64)
            dist = np.sqrt((t[:, None] * l.astype(D64)) ** 2 @ np.ones(3))
            lit &= ~((t > D64(F(0.0001))) & (dist < ln.astype(D64)))
        return lit

    def primary(self, x, y, jx=None, jy=None):
        px, py = x.astype(F), y.astype(F)
        if jx is not None:
            px, py = px + jx, py + jy
        hp = (px / F(self.W)).astype(F)
        vp = (py / F(self.H)).astype(F)
        llc, h, v = self.hdr[3, :3], self.hdr[1, :3], self.hdr[2, :3]
        d = (llc + hp[:, None] * h) + vp[:, None] * v
        return normalize3(d.astype(F))

    def phong_terms(self, ind, curr, dirs, col4, lit):
        light = self.hdr[5, :3]
        nn = self.normal(ind, curr)
        l = normalize3(light - curr)
        spec = np.power(clamp(dot3(normalize3(l - dirs), nn), 0.0, 1.0), F(500.0)).astype(F)
        k = clamp(dot3(nn, l), 0.06, 1.0)
        out = np.where(lit[:, None], col4 * k[:, None] + spec[:, None], col4 * F(0.06))
        return out.astype(F), nn

    # ---- programs ----
    def pixels_xy(self, y0, y1):
        ys, xs = np.meshgrid(np.arange(y0, y1), np.arange(self.W), indexing="ij")
        return xs.ravel(), ys.ravel()

    def store(self, x, y, col, image, gy0):
        self.pix[self.frame, x, y - gy0] = col
        if image is not None:
            image[y - gy0, x] = col

    def p_compute(self, x, y, image, gy0):
        dirs = self.primary(x, y)
        cam = np.broadcast_to(self.hdr[4, :3], dirs.shape)
        t, ind = self.closest(cam, dirs, 0.0)
        res = np.broadcast_to(self.hdr[6], (len(x), 4)).astype(F).copy()
        hit = ind >= 0
        if hit.any():
            curr = cam[hit] + t[hit, None] * dirs[hit]
            lit = self.shadow_lit(curr)
            col4 = self.shapes[ind[hit], 4].copy()
            col4[:, 3] = 0
            out, _ = self.phong_terms(ind[hit], curr, dirs[hit], col4, lit)
            out[:, 3] = np.where(lit, F(0.0) + out[:, 3], F(0.0))
            res[hit] = out
        col = np.concatenate([np.power(F(0.0) + res[:, :3], GAMMA), np.zeros((len(x), 1), F)], 1).astype(F)
        self.store(x, y, col, image, gy0)

    def h_compute(self, x, y, image, gy0):
        n = len(x)
        dirs = self.primary(x, y)
        pos = np.broadcast_to(self.hdr[4, :3], dirs.shape).astype(F).copy()
        res = np.zeros((n, 4), F)
        c = np.zeros(n, F)
        arefl = np.zeros(n, F)
        live = np.ones(n, bool)
        for seg in range(self.D):
            idx = np.nonzero(live)[0]
            if idx.size == 0:
                break
            t, ind = self.closest(pos[idx], dirs[idx], 0.001)
            att = np.broadcast_to(self.hdr[6], (idx.size, 4)).astype(F).copy()
            stop = np.ones(idx.size, bool)
            hit = ind >= 0
            if hit.any():
                hi = idx[hit]
                curr = pos[hi] + t[hit, None] * dirs[hi]
                lit = self.shadow_lit(curr)
                out, nn = self.phong_terms(ind[hit], curr, dirs[hi], self.shapes[ind[hit], 4], lit)
                att[hit] = out
                refl = (F(1.0) - self.shapes[ind[hit], 3, 3]).astype(F)
                go = ~(refl < F(0.001))
                stop[hit] = ~go
                g = hi[go]
                dn = dot3(dirs[g], nn[go])
                dirs[g] = normalize3(dirs[g] - F(2.0) * (dn[:, None] * nn[go]))
                pos[g] = curr[go]
                arefl[g] = refl[go]
            if seg == 0:
                c[idx] = arefl[idx]
                res[idx] = att
            else:
                den = F(1.0) + c[idx]
                res[idx] = ((res[idx] + c[idx, None] * att) / den[:, None]).astype(F)
                c[idx] = c[idx] * arefl[idx]
            live[idx[stop]] = False
        col = np.concatenate([np.power(F(0.0) + res[:, :3], GAMMA), np.zeros((n, 1), F)], 1).astype(F)
        self.store(x, y, col, image, gy0)

    def ao_compute(self, x, y, image, gy0, write_image):
        n, D, f = len(x), self.D, self.frame
        gy = y - gy0
        px, py = x.astype(F), y.astype(F)
        cam = self.hdr[4, :3]
        acc = np.zeros((n, 4), F)
        for aa in range(self.AA):
            fst, snd = self.rb[2 * aa], self.rb[2 * aa + 1]
            if aa == 0:
                dirs = self.primary(x, y)
            else:  # ao_compute.glsl:310-323
                s1, s2, s3, s4 = (snd[0], fst[1]), (fst[2], snd[3]), (fst[0], snd[1]), (snd[2], fst[3])
                if CONTRACTION & C_FUSED_JITTER:
                    u = grandom((fma(px, s2[0], s1[0]) - px) + s3[0], (fma(py, s2[1], s1[1]) - py) + s3[1])
                    w = grandom(fma(s4[0], px, -((s3[0] * px) * s2[0])), fma(s4[1], py, -((s3[1] * py) * s2[1])))
                else:
                    u = grandom(((s1[0] + px * s2[0]) - px) + s3[0], ((s1[1] + py * s2[1]) - py) + s3[1])
                    w = grandom(s4[0] * px - (s3[0] * px) * s2[0], s4[1] * py - (s3[1] * py) * s2[1])
                il = F(1.0) / np.sqrt(fma(w, w, u * u))
                jx = (u * il) / F(6.0) - F(0.08333)
                jy = (w * il) / F(6.0) - F(0.08333)
                dirs = self.primary(x, y, jx, jy)
            # get_pt_within_unit_sphere(aa), ao_compute.glsl:143-158
            if CONTRACTION & C_FUSED_SEEDS:
                a = grandom(fma(px, snd[2], fst[0]), fma(py, snd[3], fst[1]))
                b = grandom(fma(-px, snd[2], fst[2]), fma(-py, snd[3], fst[3]))
                e = grandom(fma(snd[0], px, snd[2]), fma(snd[1], py, snd[3]))
            else:
                a = grandom(fst[0] + px * snd[2], fst[1] + py * snd[3])
                b = grandom(fst[2] - px * snd[2], fst[3] - py * snd[3])
                e = grandom(snd[0] * px + snd[2], snd[1] * py + snd[3])
            hemi = normalize3(np.stack([a * F(2) - F(1), b * F(2) - F(1), e * F(2) - F(1)], 1))
            res = np.ones((n, 4), F)
            pos = np.broadcast_to(cam, (n, 3)).astype(F).copy()
            live = np.ones(n, bool)
            for depth in range(D, 0, -1):
                idx = np.nonzero(live)[0]
                if idx.size == 0:
                    break
                t, ind = self.closest(pos[idx], dirs[idx], 0.0001)
                miss = ind < 0
                att = np.empty((idx.size, 4), F)
                att[miss] = self.hdr[6]
                hit = ~miss
                emis = np.zeros(idx.size, bool)
                emis[hit] = self.shapes[ind[hit], 1, 3] > F(0.9)
                att[hit] = self.shapes[ind[hit], 4]
                first = aa == 0 and depth == D
                mi = idx[miss]
                if first:
                    self.nrm[f, x[mi], gy[mi]] = 0
                    self.dep[f, x[mi], gy[mi]] = 0
                stopped = idx[miss | emis]
                self.dep[f, x[stopped], gy[stopped], 1] = F(D - depth)
                cont = hit & ~emis
                ci = idx[cont]
                if ci.size:
                    curr = cam + t[cont, None] * dirs[ci]  # sic: camera origin (ao_compute.glsl:210)
                    nn = self.normal(ind[cont], curr)
                    if first:
                        self.nrm[f, x[ci], gy[ci]] = np.concatenate([nn, np.ones((ci.size, 1), F)], 1)
                        self.dep[f, x[ci], gy[ci]] = np.stack([t[cont], np.zeros(ci.size, F), np.zeros(ci.size, F),
                                                               np.ones(ci.size, F)], 1)
                    pos[ci] = curr
                    refl = self.shapes[ind[cont], 3, 3]
                    diffuse = refl > F(0.999)
                    nd = np.empty_like(nn)
                    nd[diffuse] = normalize3(hemi[ci[diffuse]] + nn[diffuse])
                    gl = ~diffuse
                    if gl.any():
                        dg = dirs[ci[gl]]
                        dn = dot3(dg, nn[gl])
                        R = normalize3(dg - F(2.0) * (dn[:, None] * nn[gl]))
                        nd[gl] = normalize3(R + refl[gl, None] * hemi[ci[gl]])
                    dirs[ci] = nd
                res[idx] = res[idx] * att
                live[stopped] = False
            acc = (acc + res).astype(F)
        fa = F(self.AA)
        acc = (acc / fa).astype(F)
        self.dep[f, x, gy] = (self.dep[f, x, gy] / fa).astype(F)
        col = np.concatenate([np.power(acc[:, :3], GAMMA), np.zeros((n, 1), F)], 1).astype(F)
        self.store(x, y, col, image if write_image else None, gy0)

    def aop_postprocessing(self, x, y, image, gy0, gh):
        f, Fn, W, H = self.frame, self.F, self.W, self.H
        snap = self.pix[f].copy()
        gy = y - gy0
        color = snap[x, gy].copy()
        nn = self.nrm[f, x, gy]
        active = nn[:, 3] > F(0.99)
        nv = nn[:, :3]
        nd, nb = self.dep[f, x, gy, 0], self.dep[f, x, gy, 1]

        def weight(xx, yy, present):
            pr = present & (yy >= gy0) & (yy < gy0 + gh)
            xc = np.clip(xx, 0, W - 1)
            yc = np.clip(yy - gy0, 0, gh - 1)
            kn, kd, kv = self.nrm[f, xc, yc], self.dep[f, xc, yc], snap[xc, yc]
            dd = F(1.0) - clamp(np.abs(nd - kd[:, 0]), 0.0, 1.0)
            bd = F(1.0) - clamp(np.abs(nb - kd[:, 1]) / F(1.7), 0.0, 1.0)
            wv = (dot3(nv, kn[:, :3]) * dd * bd + F(0.2)).astype(F)
            wv = np.where(kn[:, 3] < F(0.001), F(1.0), wv)
            wv = np.where(pr, wv, F(0.0))
            return wv, np.where(pr[:, None], kv, F(0.0))

        nbrs = [(x, y + 1, y + 1 < H), (x, y - 1, y >= 2), (x - 1, y, x > 0), (x + 1, y, x + 1 < W)]
        acc = color.copy()
        den = np.ones(len(x), F)
        for xx, yy, pr in nbrs:
            wv, kv = weight(xx, yy, pr)
            acc = (acc + wv[:, None] * kv).astype(F)
            den = (den + wv).astype(F)
        sp = (acc / den[:, None]).astype(F)
        cs = np.zeros((len(x), 4), F)
        denom = np.full(len(x), F(0.9))
        go = np.ones(len(x), bool)
        for i in range(1, Fn):
            cf = (f + Fn - i) % Fn
            hn, hd = self.nrm[cf, x, gy], self.dep[cf, x, gy]
            dd = F(1.0) - clamp(np.abs(nd - hd[:, 0]), 0.0, 1.0)
            bd = F(1.0) - clamp(np.abs(nb - hd[:, 1]) / F(1.7), 0.0, 1.0)
            coeff = (dot3(nv, hn[:, :3]) * dd * bd).astype(F)
            go &= coeff > F(0.85)
            cs = np.where(go[:, None], cs + coeff[:, None] * self.pix[cf, x, gy], cs).astype(F)
            denom = np.where(go, denom + coeff, denom).astype(F)
        filt = ((sp * F(0.9) + cs) / denom[:, None]).astype(F)
        out = np.where(active[:, None], filt, color)
        self.store(x, y, out, image, gy0)


def run_program(ssbo, W, H, S, AA, program, frame, image=None, F_=8, D=20, gy0=0, gh=None, y0=None, y1=None):
    gh = H if gh is None else gh
    ssbo[1] = F(frame)
    fr = Frame(ssbo, W, gh, S, AA, F_, D)
    fr.H = H  # full-frame height for ray generation / bounds
    y0 = gy0 if y0 is None else y0
    y1 = gy0 + gh if y1 is None else y1
    ys, xs = np.meshgrid(np.arange(y0, y1), np.arange(W), indexing="ij")
    x, y = xs.ravel(), ys.ravel()
    if program == P_COMPUTE:
        fr.p_compute(x, y, image, gy0)
    elif program == H_COMPUTE:
        fr.h_compute(x, y, image, gy0)
    elif program in (AO_COMPUTE, AOP_COMPUTE):
        fr.ao_compute(x, y, image, gy0, program == AO_COMPUTE)
    elif program == AOP_POSTPROCESSING:
        fr.aop_postprocessing(x, y, image, gy0, gh)
    else:
        raise ValueError(program)


def dispatch(ssbo, W, H, S, AA, mode, frame, image=None, F_=8, D=20):
    progs = {1: [AOP_COMPUTE, AOP_POSTPROCESSING], 2: [AO_COMPUTE], 3: [P_COMPUTE], 4: [H_COMPUTE]}[mode]
    for p in progs:
        run_program(ssbo, W, H, S, AA, p, frame, image, F_, D)
    return (frame + 1) % F_
