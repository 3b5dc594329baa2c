"""Independent numpy restatement of the MIS integrator — TEST INFRASTRUCTURE ONLY.

Second CPU restatement of ``kernel drawTriangle`` of the SwiftPM build
(``Sources/gpuRaytracer/shaders.metal:635-707``) and its helpers, vectorised
over pixels with the exact-fma emulation of ``pt_oracle_np`` (DESIGN.md §3,
§3.11).  It cross-checks ``pto_render_mis`` of ``pt_oracle.c`` bit for bit on
tiny images (tests/test_oracle.py); only tests/ import it.
"""
from __future__ import annotations

import ctypes
import ctypes.util

import numpy as np

from pt_oracle_np import V, _closest, cross, dot, f32, fma32, halton, normalize, sincos
from pt_oracle_np import Scene as _BaseScene

_libm = ctypes.CDLL(ctypes.util.find_library("m"))
_libm.powf.restype = ctypes.c_float
_libm.powf.argtypes = [ctypes.c_float, ctypes.c_float]

PI = f32(3.14159274)        # M_PI_F
INV_PI = f32(0.318309873)   # 1.0 / M_PI_F
TWO_PI = f32(6.28318548)


class Scene(_BaseScene):
    def __init__(self, camera, materials, light, vertices):
        super().__init__(camera, materials, light, vertices)
        mt = np.frombuffer(bytes(materials), dtype=np.float32).reshape(-1, 12)
        for k, T in enumerate(self.tris):
            T["metallic"] = f32(mt[k, 4])
            T["roughness"] = f32(mt[k, 5])
        lt = np.frombuffer(bytes(light), dtype=np.float32)
        self.Le = V(*lt[8:11])                 # emittedRadiance
        self.lw, self.ld = f32(lt[12]), f32(lt[13])
        self.ev100 = f32(np.frombuffer(bytes(camera), dtype=np.float32)[15])


def _u32_hash(x):
    x = np.asarray(x, np.uint32)
    x = x ^ (x >> np.uint32(16))
    x = (x.astype(np.uint64) * np.uint64(0x7feb352d)).astype(np.uint32)
    x = x ^ (x >> np.uint32(15))
    x = (x.astype(np.uint64) * np.uint64(0x846ca68b)).astype(np.uint32)
    return x ^ (x >> np.uint32(16))


def _unit(h):
    return h.astype(f32) * f32(2.3283064365386963e-10)


def _vfull(v, shape):
    return V(np.full(shape, v.x, f32), np.full(shape, v.y, f32), np.full(shape, v.z, f32))


def _field(sc, ids, key, shape):
    out = np.zeros(shape, f32)
    for k in np.unique(ids[ids >= 0]):
        out = np.where(ids == k, sc.tris[k][key], out)
    return out


def _vfield(sc, ids, key, shape):
    x, y, z = (np.zeros(shape, f32) for _ in range(3))
    for k in np.unique(ids[ids >= 0]):
        m = ids == k
        v = sc.tris[k][key]
        x, y, z = np.where(m, v.x, x), np.where(m, v.y, y), np.where(m, v.z, z)
    return V(x, y, z)


def _onb(n):  # buildOrthonormalBasis (:159-172)
    big = np.abs(n.x) > f32(0.9)
    a = V(np.where(big, f32(0), f32(1)), np.where(big, f32(1), f32(0)), np.zeros_like(n.x))
    t = normalize(a - n.scale(dot(a, n)))
    return t, cross(n, t)


def _c01(x):
    return np.minimum(f32(1.0), np.maximum(f32(0.0), x))


def _d_ggx(NoH, a):
    a2 = a * a
    f = (NoH * a2 - NoH) * NoH + f32(1.0)
    return a2 / ((PI * f) * f)


def _brdf(din, n, m, l):  # calculateBRDFContribution (:259-289)
    v = -normalize(din)
    h = normalize(v + l)
    NoV = np.abs(dot(n, v)) + f32(1e-5)
    NoL, NoH, LoH = _c01(dot(n, l)), _c01(dot(n, h)), _c01(dot(l, h))
    dif, met, rough = m
    f0 = V(*(f32(0.04) + (c - f32(0.04)) * met for c in (dif.x, dif.y, dif.z)))
    D = _d_ggx(NoH, rough)
    x = f32(1.0) - LoH
    x2 = x * x
    p5 = (x2 * x2) * x
    F = V(*(c + (f32(1.0) - c) * p5 for c in (f0.x, f0.y, f0.z)))
    a2 = rough * rough
    GGXL = NoV * np.sqrt(((-NoL) * a2 + NoL) * NoL + a2)
    GGXV = NoL * np.sqrt(((-NoV) * a2 + NoV) * NoV + a2)
    G = f32(0.5) / (GGXV + GGXL)
    den = (f32(4.0) * NoV) * NoL + f32(1e-7)
    DG = D * G
    Fr = V(*((DG * c) / den for c in (F.x, F.y, F.z)))
    Fd = dif.scale(INV_PI)
    km = f32(1.0) - met
    kD = V(*((f32(1.0) - c) * km for c in (F.x, F.y, F.z)))
    return kD.mul(Fd + Fr).scale(NoL)


def _vndf_pdf(Vv, n, L, rough):  # calculateVNDFPdf (:437-445)
    h = normalize(Vv + L)
    NoH, VoH, NoV = np.abs(dot(n, h)), np.abs(dot(Vv, h)), np.abs(dot(n, Vv))
    a = rough * rough
    a2 = a * a
    NoV2 = NoV * NoV
    G1 = f32(2.0) / (f32(1.0) + np.sqrt(f32(1.0) + (a2 * (f32(1.0) - NoV2)) / NoV2))
    return ((_d_ggx(NoH, rough) * G1) * VoH) / (f32(4.0) * NoV)


def _cos_pdf(n, d):
    return np.maximum(f32(0.0), dot(n, d)) / PI


def _light_pdf(sc, p, d):
    toL = sc.lc - p
    dist = np.sqrt(dot(toL, toL))
    cosT = np.maximum(f32(0.0), dot(-d, V(f32(0), f32(-1), f32(0))))
    return (dist * dist) / ((sc.lw * sc.ld) * cosT + f32(1e-6))


def _power(p1, p2, p3, n):
    a = n * p1
    return a / (((a + n * p2) + n * p3) + f32(1e-6))


def _direct(sc, lt, p, n, din, m, ux, uy, nS, power, mask):
    """calculateDirectLightSamplingContribution (:519-541) on the lanes in mask."""
    shape = p.x.shape
    origin = p + n.scale(f32(1e-4))
    sx = (ux - f32(0.5)) * sc.lw
    sy = (uy - f32(0.5)) * sc.ld
    sp = (sc.lc + lt[0].scale(sx)) + lt[1].scale(sy)
    tl = sp - origin
    dist = np.sqrt(dot(tl, tl))
    with np.errstate(divide="ignore", invalid="ignore"):
        L = V(tl.x / dist, tl.y / dist, tl.z / dist)
    ids, _ = _closest(sc, origin, L, f32(0.001), dist)
    is_light = np.array([T["light"] for T in sc.tris] + [False])
    lit = mask & (ids >= 0) & is_light[ids]
    zero = V(np.zeros(shape, f32), np.zeros(shape, f32), np.zeros(shape, f32))
    if not lit.any():
        return zero
    with np.errstate(divide="ignore", invalid="ignore"):
        dl_pdf = _light_pdf(sc, p, L)
        c = _brdf(din, n, m, L)
        if power:
            w = _power(dl_pdf, _cos_pdf(n, L), _vndf_pdf(-din, n, L, m[2]), nS)
            a = c.scale(w).mul(_vfull(sc.Le, shape))
        else:
            a = c.mul(_vfull(sc.Le, shape))
        r = V(a.x / dl_pdf, a.y / dl_pdf, a.z / dl_pdf)
    return r.where(lit, zero)


def _continue(sc, lt, x, origin, d, pdf, w, u2x, u2y, mask):
    shape = origin.x.shape
    ids, t = _closest(sc, origin, d, f32(0.001), f32(1000.0))
    is_light = np.array([T["light"] for T in sc.tris] + [False])
    hit = mask & (ids >= 0)
    lit = hit & is_light[ids]
    surf = hit & ~lit
    zero = V(np.zeros(shape, f32), np.zeros(shape, f32), np.zeros(shape, f32))
    with np.errstate(divide="ignore", invalid="ignore"):
        c = _brdf(x["din"], x["n"], x["m"], d)
        a = c.scale(w).mul(_vfull(sc.Le, shape))
        em = V(a.x / pdf, a.y / pdf, a.z / pdf)
        q = V(c.x / pdf, c.y / pdf, c.z / pdf)
    r = em.where(lit, zero)
    if surf.any():
        sid = np.where(surf, ids, -1)
        y_p = origin + d.scale(t)
        y_n = _vfield(sc, sid, "N", shape)
        y_m = (_vfield(sc, sid, "diffuse", shape), _field(sc, sid, "metallic", shape),
               _field(sc, sid, "roughness", shape))
        nee = _direct(sc, lt, y_p, y_n, d, y_m, u2x, u2y, f32(1.0), False, surf)
        r = q.mul(nee).where(surf, r)
    return r


def _mis(sc, lt, x, S, mask):
    """recursiveMultiImportanceSampling (:543-625) for the hit lanes in mask."""
    shape = x["p"].x.shape
    nS = f32(S)
    z = np.zeros(shape, f32)
    dl, cs, vn = V(z, z, z), V(z, z, z), V(z, z, z)
    n, m = x["n"], x["m"]
    for i in range(S):
        dl = dl + _direct(sc, lt, x["p"], n, x["din"], m, halton(np.uint32(i), 0),
                          halton(np.uint32(i), 1), nS, True, mask)
    t, b = _onb(n)
    origin = x["p"] + n.scale(f32(1e-4))
    Vv = -x["din"]
    for i in range(S):
        ux, uy = halton(np.uint32(i + S), 2), halton(np.uint32(i + S), 3)
        sp, cp = sincos(TWO_PI * ux)
        cosT, sinT = np.sqrt(uy), np.sqrt(f32(1.0) - uy)
        d = normalize((t.scale(cp * sinT) + b.scale(sp * sinT)) + n.scale(cosT))
        cpdf = _cos_pdf(n, d)
        with np.errstate(divide="ignore", invalid="ignore"):
            w = _power(cpdf, _light_pdf(sc, x["p"], d), _vndf_pdf(Vv, n, d, m[2]), nS)
        cs = cs + _continue(sc, lt, x, origin, d, cpdf, w, halton(np.uint32(i), 6),
                            halton(np.uint32(i), 7), mask)
    for i in range(S):
        ux, uy = halton(np.uint32(i + 2 * S), 4), halton(np.uint32(i + 2 * S), 5)
        alpha = m[2] * m[2]
        Ve = normalize(V(alpha * dot(Vv, t), alpha * dot(Vv, b), dot(Vv, n)))
        T1 = normalize(V(Ve.z, np.zeros(shape, f32), -Ve.x))
        T2 = cross(Ve, T1)
        lenVe = np.sqrt(dot(Ve, Ve))
        ctm = lenVe / np.sqrt(f32(1.0) + lenVe * lenVe)
        ct = ctm + (f32(1.0) - ctm) * uy
        st = np.sqrt(f32(1.0) - ct * ct)
        sp, cp = sincos(TWO_PI * ux)
        h = normalize((T1.scale(cp * st) + T2.scale(sp * st)) + Ve.scale(ct))
        Nh = normalize(V(alpha * h.x, alpha * h.y, np.maximum(f32(0.0), h.z)))
        wH = normalize((t.scale(Nh.x) + b.scale(Nh.y)) + n.scale(Nh.z))
        I = -Vv
        d = I - wH.scale(f32(2.0) * dot(wH, I))
        with np.errstate(divide="ignore", invalid="ignore"):
            vpdf = _vndf_pdf(Vv, n, d, m[2])
            w = _power(vpdf, _light_pdf(sc, x["p"], d), _cos_pdf(n, d), nS)
        vn = vn + _continue(sc, lt, x, origin, d, vpdf, w, halton(np.uint32(i + S), 6),
                            halton(np.uint32(i + S), 7), mask)
    s = (dl + cs) + vn
    return V(s.x / nS, s.y / nS, s.z / nS)


def _log(x):  # DESIGN.md §3.11 (cephes logf)
    bx = x.view(np.uint32)
    e = (bx >> np.uint32(23)).astype(np.int32) - 126
    m = ((bx & np.uint32(0x007FFFFF)) | np.uint32(0x3F000000)).view(f32)
    lo = m < f32(0.707106781)
    e = np.where(lo, e - 1, e)
    m = np.where(lo, (m + m) - f32(1.0), m - f32(1.0))
    z = m * m
    y = np.full(m.shape, f32(7.0376836292e-2))
    for c in (-1.1514610310e-1, 1.1676998740e-1, -1.2420140846e-1, 1.4249322787e-1,
              -1.6668057665e-1, 2.0000714765e-1, -2.4999993993e-1, 3.3333331174e-1):
        y = fma32(y, m, f32(c))
    y = (y * m) * z
    fe = e.astype(f32)
    y = fma32(fe, f32(-2.12194440e-4), y)
    y = fma32(f32(-0.5), z, y)
    return fma32(fe, f32(0.693359375), m + y)


def _exp(x):
    z = np.floor(x * f32(1.44269504088896341) + f32(0.5)).astype(f32)
    r = fma32(-z, f32(0.693359375), x)
    r = fma32(-z, f32(-2.12194440e-4), r)
    p = np.full(x.shape, f32(1.9875691500e-4))
    for c in (1.3981999507e-3, 8.3334519073e-3, 4.1665795894e-2, 1.6666665459e-1,
              5.0000001201e-1):
        p = fma32(p, r, f32(c))
    y = fma32(p, r * r, r) + f32(1.0)
    return y * ((z.astype(np.int32) + 127).astype(np.uint32) << np.uint32(23)).view(f32)


def pow_pt(x, y):
    x = np.atleast_1d(np.asarray(x, f32))
    ok = x > f32(7.88860905e-31)
    xs = np.where(ok, x, f32(1.0))
    return np.where(ok, _exp(f32(y) * _log(xs)), f32(0.0)).astype(f32)


def render_mis(sc, camera_rays, mis_samples):
    """Full frame; returns ((H, W, 4) float32 (sum, camera_rays), (H, W, 4) uint8)."""
    H, W = sc.H, sc.W
    ys, xs = np.mgrid[0:H, 0:W]
    xs, ys = xs.ravel().astype(np.uint32), ys.ravel().astype(np.uint32)
    shape = xs.shape
    S = mis_samples // 3
    lt = _onb(V(np.array([0], f32), np.array([-1], f32), np.array([0], f32)))
    lt = (V(lt[0].x[0], lt[0].y[0], lt[0].z[0]), V(lt[1].x[0], lt[1].y[0], lt[1].z[0]))
    is_light = np.array([T["light"] for T in sc.tris] + [False])
    z = np.zeros(shape, f32)
    acc = V(z, z, z)
    for i in range(camera_rays):
        with np.errstate(over="ignore"):
            sid = (ys * np.uint32(800) + xs) * np.uint32(i)
            jx = _unit(_u32_hash(xs + ys * np.uint32(800) + sid))
            jy = _unit(_u32_hash(ys + xs * np.uint32(600) + sid + np.uint32(12345)))
        s = ((xs.astype(f32) + jx) / f32(W)) * f32(2.0) - f32(1.0)
        t = -(((ys.astype(f32) + jy) / f32(H)) * f32(2.0) - f32(1.0))
        d = normalize((sc.u.scale(s * sc.halfW) + sc.v.scale(t * sc.halfH)) - sc.w)
        o = _vfull(sc.pos, shape)
        ids, th = _closest(sc, o, d, f32(0.001), f32(1000.0))
        hit = ids >= 0
        lit = hit & is_light[ids]
        surf = hit & ~lit
        acc = (acc + _vfull(sc.Le, shape)).where(lit, acc)
        if surf.any():
            sidx = np.where(surf, ids, -1)
            x = dict(p=o + d.scale(th), n=_vfield(sc, sidx, "N", shape), din=d,
                     m=(_vfield(sc, sidx, "diffuse", shape), _field(sc, sidx, "metallic", shape),
                        _field(sc, sidx, "roughness", shape)))
            acc = (acc + _mis(sc, lt, x, S, surf)).where(surf, acc)
    nc = f32(camera_rays)
    out = np.empty((H * W, 4), f32)
    out[:, 0], out[:, 1], out[:, 2], out[:, 3] = acc.x, acc.y, acc.z, nc
    ev = sc.ev100
    exposure = f32(1.0) / (f32(1.2) * f32(_libm.powf(2.0, float(ev))))
    out8 = np.full((H * W, 4), 255, np.uint8)
    for k, c in enumerate((acc.x, acc.y, acc.z)):
        e = (c / nc) * exposure
        tm = _c01(e / (e + f32(1.0)))
        g = pow_pt(tm, f32(1.0) / f32(2.2))
        out8[:, k] = (g * f32(255.0)).astype(np.uint8)
    return out.reshape(H, W, 4), out8.reshape(H, W, 4)
