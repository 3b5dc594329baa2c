"""Independent numpy restatement of ``pathTrace`` — TEST INFRASTRUCTURE ONLY.

Second, independently written CPU restatement of the reference kernel
(``RTrace/raytrace.metal:11-111`` + ``RTrace/sampling.metal``) under the
arithmetic contract of DESIGN.md §3.  It is vectorised over rays (SoA numpy
float32 arrays) instead of the scalar per-pixel loop of ``pt_oracle.c``, so a
shared-code bug cannot hide in both.  It is slow (pure numpy) and used only to
cross-check the C oracle on tiny images (tests/test_oracle.py).

Contract details reproduced here:
  * fp32 everywhere, round-to-nearest; fmaf emulated exactly with a
    round-to-odd float64 sum (``fma32``), so results are bit-comparable.
  * ``dot``/``cross`` use fma as in DESIGN.md §3.2; ``tanf``/``cosf``/``sinf``
    on the host come from the C library (ctypes), as in the oracle.
Only tests/ import this module.
"""
from __future__ import annotations

import ctypes
import ctypes.util

import numpy as np

f32 = np.float32
_libm = ctypes.CDLL(ctypes.util.find_library("m"))
_libm.tanf.restype = ctypes.c_float
_libm.tanf.argtypes = [ctypes.c_float]

PRIMES = np.array([2, 3, 5, 7, 11, 13, 17, 19, 23, 29, 31, 37, 41, 43, 47, 53,
                   59, 61, 67, 71, 73, 79, 83, 89], dtype=np.uint32)


def fma32(a, b, c):
    """Exactly rounded fp32 fma(a, b, c) via float64 round-to-odd."""
    a = np.asarray(a, f32).astype(np.float64)
    b = np.asarray(b, f32).astype(np.float64)
    c = np.asarray(c, f32).astype(np.float64)
    p = a * b                      # exact: 24+24 bit product fits in 53 bits
    s = p + c
    bb = s - p
    err = (p - (s - bb)) + (c - bb)  # TwoSum: exact error of s
    s = np.atleast_1d(s)
    err = np.atleast_1d(err)
    bits = s.view(np.uint64)
    fix = (err != 0) & ((bits & np.uint64(1)) == 0) & np.isfinite(s)
    toward = np.where(err > 0, np.inf, -np.inf)
    s = np.where(fix, np.nextafter(s, toward), s)
    return s.astype(f32)


class V:
    """SoA float32 3-vector."""

    __slots__ = ("x", "y", "z")

    def __init__(self, x, y, z):
        self.x = np.asarray(x, f32)
        self.y = np.asarray(y, f32)
        self.z = np.asarray(z, f32)

    def __add__(self, o):
        return V(self.x + o.x, self.y + o.y, self.z + o.z)

    def __sub__(self, o):
        return V(self.x - o.x, self.y - o.y, self.z - o.z)

    def __neg__(self):
        return V(-self.x, -self.y, -self.z)

    def mul(self, o):
        return V(self.x * o.x, self.y * o.y, self.z * o.z)

    def scale(self, s):
        s = np.asarray(s, f32)
        return V(self.x * s, self.y * s, self.z * s)

    def where(self, m, o):
        return V(np.where(m, self.x, o.x), np.where(m, self.y, o.y), np.where(m, self.z, o.z))


def dot(a, b):
    return fma32(a.z, b.z, fma32(a.y, b.y, a.x * b.x))


def cross(a, b):
    return V(fma32(a.y, b.z, -(a.z * b.y)), fma32(a.z, b.x, -(a.x * b.z)),
             fma32(a.x, b.y, -(a.y * b.x)))


def normalize(a):
    return a.scale(f32(1.0) / np.sqrt(dot(a, a)))


def saturate(x):
    return np.minimum(np.maximum(x, f32(0.0)), f32(1.0))


def halton(i, d):
    """sampling.metal:107-122, vectorised over i (uint32)."""
    b = np.uint32(PRIMES[d])
    inv_b = f32(1.0) / f32(b)
    i = np.array(i, dtype=np.uint32, copy=True)
    f = np.ones(i.shape, f32)
    r = np.zeros(i.shape, f32)
    live = i > 0
    while live.any():
        f = np.where(live, f * inv_b, f)
        r = np.where(live, r + f * (i % b).astype(f32), r)
        i = np.where(live, i // b, i)
        live = i > 0
    return r


def sincos(x):
    x = np.asarray(x, f32)
    k = np.rint(x * f32(0.636619772))
    r = fma32(-k, f32(1.57079637e+00), x)
    r = fma32(-k, f32(-4.37113883e-08), r)
    q = k.astype(np.int32) & 3
    r2 = r * r
    s = fma32(r * r2, fma32(r2, fma32(r2, f32(-1.9515295891e-4), f32(8.3321608736e-3)),
                            f32(-1.6666654611e-1)), r)
    c = fma32(r2 * r2, fma32(r2, fma32(r2, f32(2.443315711809948e-5),
                                       f32(-1.388731625493765e-3)), f32(4.166664568298827e-2)),
              fma32(f32(-0.5), r2, f32(1.0)))
    sin = np.select([q == 0, q == 1, q == 2], [s, c, -s], -c)
    cos = np.select([q == 0, q == 1, q == 2], [c, -s, -c], s)
    return sin.astype(f32), cos.astype(f32)


class Scene:
    """Precomputed primitive records from the ABI arrays (numpy views)."""

    def __init__(self, camera, materials, light, vertices, spheres=None):
        cam = np.frombuffer(bytes(camera), dtype=np.float32)
        res = np.frombuffer(bytes(camera), dtype=np.int32)[12:14]
        self.W, self.H = int(res[0]), int(res[1])
        self.pos = V(*cam[0:3])
        direction = V(*cam[4:7])
        up = V(*cam[8:11])
        fov = f32(cam[14])
        aspect = f32(self.W // self.H)
        self.halfW = f32(_libm.tanf(float(fov / f32(2.0))))
        self.halfH = self.halfW / aspect
        self.w = -normalize(direction)
        self.u = normalize(cross(up, self.w))
        self.v = normalize(cross(self.w, self.u))
        lt = np.frombuffer(bytes(light), dtype=np.float32)
        self.lc = V(*lt[0:3])
        self.lcol = V(*lt[4:7])
        vt = np.frombuffer(bytes(vertices), dtype=np.float32).reshape(-1, 4)
        mt = np.frombuffer(bytes(materials), dtype=np.float32).reshape(-1, 12) if len(vt) else np.zeros((0, 12), f32)
        self.tris = []
        for k in range(len(vt) // 3):
            a, b, c = (V(*vt[3 * k + j, :3]) for j in range(3))
            e1, e2 = b - a, c - a
            n = cross(e1, e2)
            N = normalize(n)
            right = normalize(cross(N, V(f32(0.0072), f32(1.0), f32(0.0034))))
            fwd = cross(right, N)
            em = V(*mt[k, 8:11])
            self.tris.append(dict(v0=a, e1=e1, e2=e2, n=n, N=N, right=right, fwd=fwd,
                                  diffuse=V(*mt[k, 0:3]), emissive=em,
                                  light=bool(np.sqrt(dot(em, em)) > 0)))
        self.sph = []
        if spheres is not None and len(bytes(spheres)):
            st = np.frombuffer(bytes(spheres), dtype=np.float32).reshape(-1, 20)
            for row in st:
                em = V(*row[12:15])
                self.sph.append(dict(c=V(*row[0:3]), r2=f32(row[16]) * f32(row[16]),
                                     diffuse=V(*row[4:7]), emissive=em,
                                     light=bool(np.sqrt(dot(em, em)) > 0)))


def _tri_test(T, o, d, tmin, tmax):
    tv = o - T["v0"]
    c = cross(tv, d)
    den = dot(T["n"], d)
    bu = -dot(T["e2"], c)
    bv = dot(T["e1"], c)
    tn = -dot(T["n"], tv)
    neg = den < 0
    den = np.where(neg, -den, den)
    bu = np.where(neg, -bu, bu)
    bv = np.where(neg, -bv, bv)
    tn = np.where(neg, -tn, tn)
    ok = (den > 0) & (bu >= 0) & (bv >= 0) & (bu + bv <= den)
    with np.errstate(divide="ignore", invalid="ignore"):
        t = np.where(ok, tn / np.where(ok, den, f32(1)), f32(0))
    return ok & (t > tmin) & (t < tmax), t


def _sph_test(S, o, d, a, tmin, tmax):
    oc = o - S["c"]
    b = f32(2.0) * dot(oc, d)
    cc = dot(oc, oc) - S["r2"]
    disc = b * b - (f32(4.0) * a) * cc
    ok = disc > 0
    with np.errstate(invalid="ignore", divide="ignore"):
        sq = np.sqrt(np.where(ok, disc, f32(0)))
        a2 = f32(2.0) * a
        t1 = (-b - sq) / a2
        t2 = (-b + sq) / a2
    t = np.where(t1 > tmin, t1, t2)
    return ok & (t > tmin) & (t < tmax), t


def _closest(sc, o, d, tmin, tmax):
    best = np.full(o.x.shape, tmax, f32)
    ids = np.full(o.x.shape, -1, np.int64)
    for k, T in enumerate(sc.tris):
        hit, t = _tri_test(T, o, d, tmin, best)
        best = np.where(hit, t, best)
        ids = np.where(hit, k, ids)
    if sc.sph:
        a = dot(d, d)
        for k, S in enumerate(sc.sph):
            hit, t = _sph_test(S, o, d, a, tmin, best)
            best = np.where(hit, t, best)
            ids = np.where(hit, len(sc.tris) + k, ids)
    return ids, best


def _occluded(sc, o, d, tmin, tmax):
    occ = np.zeros(o.x.shape, bool)
    for T in sc.tris:
        hit, _ = _tri_test(T, o, d, tmin, tmax)
        occ |= hit
    if sc.sph:
        a = dot(d, d)
        for S in sc.sph:
            hit, _ = _sph_test(S, o, d, a, tmin, tmax)
            occ |= hit
    return occ


def _gather(sc, ids, key, shape):
    """Per-ray gather of a V-valued primitive field."""
    x = np.zeros(shape, f32)
    y = np.zeros(shape, f32)
    z = np.zeros(shape, f32)
    prims = sc.tris + sc.sph
    for k in np.unique(ids[ids >= 0]):
        m = ids == k
        v = prims[k][key]
        x = np.where(m, v.x, x)
        y = np.where(m, v.y, y)
        z = np.where(m, v.z, z)
    return V(x, y, z)


def trace(sc, xs, ys, seeds, ns, bounces):
    """Per-sample accumulatedColor for arrays of (x, y, seed, n)."""
    xs = np.asarray(xs)
    shape = xs.shape
    i = (np.asarray(seeds, np.uint64) + np.asarray(ns, np.uint64)).astype(np.uint32)
    jx, jy = halton(i, 0), halton(i, 1)
    s = ((xs.astype(f32) + jx) / f32(sc.W)) * f32(2.0) - f32(1.0)
    t = -(((np.asarray(ys).astype(f32) + jy) / f32(sc.H)) * f32(2.0) - f32(1.0))
    d = normalize((sc.u.scale(s * sc.halfW) + sc.v.scale(t * sc.halfH)) - sc.w)
    o = V(np.broadcast_to(sc.pos.x, shape), np.broadcast_to(sc.pos.y, shape),
          np.broadcast_to(sc.pos.z, shape))
    acc = V(np.zeros(shape, f32), np.zeros(shape, f32), np.zeros(shape, f32))
    thr = V(np.ones(shape, f32), np.ones(shape, f32), np.ones(shape, f32))
    alive = np.ones(shape, bool)
    tmin, tmax = f32(0.001), f32(1000.0)
    is_light = np.array([p["light"] for p in sc.tris + sc.sph] + [False])
    nT = len(sc.tris)
    for b in range(bounces):
        ids, th = _closest(sc, o, d, tmin, tmax)
        alive &= ids >= 0
        lit = alive & is_light[ids]
        acc = _gather(sc, np.where(lit, ids, -1), "emissive", shape).where(lit, acc)
        alive &= ~lit
        hp = o + d.scale(th)
        N = _gather(sc, np.where(alive & (ids < nT), ids, -1), "N", shape)
        right = _gather(sc, np.where(alive & (ids < nT), ids, -1), "right", shape)
        fwd = _gather(sc, np.where(alive & (ids < nT), ids, -1), "fwd", shape)
        sm = alive & (ids >= nT)
        if sm.any():
            Ns = normalize(hp - _gather(sc, np.where(sm, ids, -1), "c", shape))
            rs = normalize(cross(Ns, V(f32(0.0072), f32(1.0), f32(0.0034))))
            fs = cross(rs, Ns)
            N, right, fwd = Ns.where(sm, N), rs.where(sm, right), fs.where(sm, fwd)
        diffuse = _gather(sc, np.where(alive, ids, -1), "diffuse", shape)
        p = hp + N.scale(f32(1e-3))
        ux = halton(i, 2 + 5 * b) * f32(2.0) - f32(1.0)
        uy = halton(i, 3 + 5 * b) * f32(2.0) - f32(1.0)
        q = (sc.lc + V(f32(0.25), f32(0.0), f32(0.0)).scale(ux)) + V(f32(0.0), f32(0.0), f32(0.25)).scale(uy)
        L = q - p
        dist = np.sqrt(dot(L, L))
        inv = f32(1.0) / np.maximum(dist, f32(1e-3))
        L = L.scale(inv)
        lc = V(np.broadcast_to(sc.lcol.x, shape), np.broadcast_to(sc.lcol.y, shape),
               np.broadcast_to(sc.lcol.z, shape)).scale(inv * inv)
        lc = lc.scale(saturate(dot(-L, V(f32(0.0), f32(-1.0), f32(0.0)))))
        lc = lc.scale(saturate(dot(N, L)))
        thr = thr.mul(diffuse).where(alive, thr)
        occ = _occluded(sc, p, L, f32(0.0), dist - f32(1e-3))
        acc = (acc + lc.mul(thr)).where(alive & ~occ, acc)
        if b + 1 < bounces:
            cu, cv = halton(i, 4 + 5 * b), halton(i, 5 + 5 * b)
            sp, cp = sincos(f32(6.28318548) * cu)
            ct = np.sqrt(cv)
            st = np.sqrt(f32(1.0) - ct * ct)
            nd = (right.scale(st * cp) + N.scale(ct)) + fwd.scale(st * sp)
            d = nd.where(alive, d)
            o = p.where(alive, o)
    return np.stack([acc.x, acc.y, acc.z], -1)


def render(sc, seeds, spp, bounces, sample_base=0):
    """Full-frame render; returns (H, W, 4) float32 rgba32F."""
    H, W = sc.H, sc.W
    ys, xs = np.mgrid[0:H, 0:W]
    xs, ys = xs.ravel(), ys.ravel()
    sd = np.asarray(seeds, np.uint32).reshape(-1)
    lum = np.zeros((H * W, 3), f32)
    for n in range(spp):
        lum = lum + trace(sc, xs, ys, sd, np.full(xs.shape, sample_base + n), bounces)
    out = np.ones((H * W, 4), f32)
    out[:, :3] = lum / f32(spp)
    return out.reshape(H, W, 4)
