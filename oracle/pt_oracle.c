/*
 * pt_oracle.c — CPU ORACLE (test infrastructure only; see pt_oracle.h).
 *
 * Scalar C restatement of `kernel pathTrace` (RTrace/raytrace.metal:11-111)
 * with the helpers of RTrace/sampling.metal, evaluated under the arithmetic
 * contract of DESIGN.md §3 (fp32, round-to-nearest, no implicit contraction;
 * dot/cross use explicit fmaf; IEEE div/sqrt; portable sincos).
 * Build: -O2 -ffp-contract=off -fno-fast-math (oracle/Makefile).
 * Every function cites the reference lines it restates.
 */
#include "pt_oracle.h"

#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

typedef struct { float x, y, z; } v3;

static inline v3 mk(float x, float y, float z) { v3 r = {x, y, z}; return r; }
static inline v3 ld3(const rt_float3* p) { return mk(p->x, p->y, p->z); }
static inline v3 add(v3 a, v3 b) { return mk(a.x + b.x, a.y + b.y, a.z + b.z); }
static inline v3 sub(v3 a, v3 b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }
static inline v3 mul(v3 a, v3 b) { return mk(a.x * b.x, a.y * b.y, a.z * b.z); }
static inline v3 scl(v3 a, float s) { return mk(a.x * s, a.y * s, a.z * s); }
static inline v3 neg(v3 a) { return mk(-a.x, -a.y, -a.z); }
/* contract: dot(a,b) = fma(a.z,b.z, fma(a.y,b.y, a.x*b.x)) */
static inline float dot(v3 a, v3 b) { return fmaf(a.z, b.z, fmaf(a.y, b.y, a.x * b.x)); }
/* contract: cross component = fma(a1,b2, -(a2*b1)) */
static inline v3 cross(v3 a, v3 b) {
    return mk(fmaf(a.y, b.z, -(a.z * b.y)), fmaf(a.z, b.x, -(a.x * b.z)),
              fmaf(a.x, b.y, -(a.y * b.x)));
}
static inline float len(v3 a) { return sqrtf(dot(a, a)); }
/* contract: normalize(v) = v * (1 / sqrt(dot(v,v))) */
static inline v3 nrm(v3 a) { return scl(a, 1.0f / sqrtf(dot(a, a))); }
static inline float saturate(float x) { return fminf(fmaxf(x, 0.0f), 1.0f); }

/* ---- sampling.metal:97-122 --------------------------------------------- */
static const uint32_t kPrimes[24] = {2,  3,  5,  7,  11, 13, 17, 19, 23, 29, 31, 37,
                                     41, 43, 47, 53, 59, 61, 67, 71, 73, 79, 83, 89};

float pto_halton(uint32_t i, uint32_t d) {
    const uint32_t b = kPrimes[d];
    float f = 1.0f;
    const float invB = 1.0f / (float)b;
    float r = 0.0f;
    while (i > 0) {
        f = f * invB;
        r = r + f * (float)(i % b);
        i = i / b;
    }
    return r;
}

/* ---- portable sincos, stands in for MSL sincos ------- */
void pto_sincos(float x, float* s_out, float* c_out) {
    const float k = rintf(x * 0.636619772f);
    float r = fmaf(-k, 1.57079637e+00f, x);
    r = fmaf(-k, -4.37113883e-08f, r);
    const int q = ((int)k) & 3;
    const float r2 = r * r;
    const float s = fmaf(r * r2, fmaf(r2, fmaf(r2, -1.9515295891e-4f, 8.3321608736e-3f),
                                      -1.6666654611e-1f), r);
    const float c = fmaf(r2 * r2, fmaf(r2, fmaf(r2, 2.443315711809948e-5f,
                                                -1.388731625493765e-3f), 4.166664568298827e-2f),
                         fmaf(-0.5f, r2, 1.0f));
    switch (q) {
        case 0: *s_out = s; *c_out = c; break;
        case 1: *s_out = c; *c_out = -s; break;
        case 2: *s_out = -s; *c_out = -c; break;
        default: *s_out = -c; *c_out = s; break;
    }
}

/* ---- camera (sampling.metal:125-157) ----------------------------------- */
typedef struct {
    v3 pos, u, v, w;
    float halfW, halfH;
    int32_t W, H;
} cam_t;

static void cam_setup(const CameraGPU* c, cam_t* o) {
    o->W = c->resolution.x;
    o->H = c->resolution.y;
    const float aspect = (float)(c->resolution.x / c->resolution.y); /* integer division :132 */
    o->halfW = tanf(c->horizontalFov / 2.0f);                        /* :133 */
    o->halfH = o->halfW / aspect;                                    /* :134 */
    o->w = neg(nrm(ld3(&c->direction)));                             /* :137 */
    o->u = nrm(cross(ld3(&c->up), o->w));                            /* :138 */
    o->v = nrm(cross(o->w, o->u));                                   /* :139 */
    o->pos = ld3(&c->position);
}

static v3 cam_dir(const cam_t* c, int32_t x, int32_t y, float jx, float jy) {
    const float s = (((float)x + jx) / (float)c->W) * 2.0f - 1.0f;     /* :141 */
    const float t = -((((float)y + jy) / (float)c->H) * 2.0f - 1.0f);  /* :142 */
    const float sh = s * c->halfW, th = t * c->halfH;                 /* :147 */
    const v3 a = scl(c->u, sh), b = scl(c->v, th);
    return nrm(sub(add(a, b), c->w));
}

void pto_camera_ray(const CameraGPU* cam, int32_t x, int32_t y, float jx, float jy, float dir[3]) {
    cam_t c;
    cam_setup(cam, &c);
    v3 d = cam_dir(&c, x, y, jx, jy);
    dir[0] = d.x; dir[1] = d.y; dir[2] = d.z;
}

/* ---- primitives ---------------------------------------------------------- */
typedef struct {
    v3 v0, e1, e2, n;    /* n = cross(e1,e2): unnormalized geometric normal      */
    v3 N, right, fwd;    /* getTriangleNormal (sampling.metal:16-26) + frame     */
    v3 diffuse, emissive;
    float metallic, roughness;  /* MIS integrator only (Sources/.../shaders.metal) */
    int light;           /* length(emissive) > 0 (raytrace.metal:57)              */
} tri_t;

typedef struct {
    v3 c;
    float r2;
    v3 diffuse, emissive;
    int light;
} sph_t;

static const v3 kFrameRef = {0.0072f, 1.0f, 0.0034f}; /* sampling.metal:57 */

/* alignHemisphereWithNormal frame (sampling.metal:51-66): right, forward */
static void frame_of(v3 N, v3* right, v3* fwd) {
    *right = nrm(cross(N, kFrameRef));
    *fwd = cross(*right, N);
}

/* Möller–Trumbore in the division-free-barycentric form of DESIGN.md §3.5
 * (stands in for Apple's closed intersector<triangle_data>, raytrace.metal:26-30). */
static inline int tri_hit(const tri_t* T, v3 o, v3 d, float tmin, float tmax, float* t_out) {
    const v3 tv = sub(o, T->v0);
    const v3 c = cross(tv, d);
    float den = dot(T->n, d);
    float bu = -dot(T->e2, c);
    float bv = dot(T->e1, c);
    float tn = -dot(T->n, tv);
    if (!(den > 0.0f) && !(den < 0.0f)) return 0;
    if (den < 0.0f) { den = -den; bu = -bu; bv = -bv; tn = -tn; }
    if (!(bu >= 0.0f && bv >= 0.0f && bu + bv <= den)) return 0;
    const float t = tn / den;
    if (t > tmin && t < tmax) { *t_out = t; return 1; }
    return 0;
}

/* intersectSphere quadratic (Sources/gpuRaytracer/shaders_old.metal:108-136),
 * with the corrected root rule of DESIGN.md §3.6. */
static inline int sph_hit(const sph_t* S, v3 o, v3 d, float a, float tmin, float tmax, float* t_out) {
    const v3 oc = sub(o, S->c);
    const float b = 2.0f * dot(oc, d);
    const float cc = dot(oc, oc) - S->r2;
    const float disc = b * b - (4.0f * a) * cc;
    if (!(disc > 0.0f)) return 0;
    const float sq = sqrtf(disc);
    const float a2 = 2.0f * a;
    const float t1 = (-b - sq) / a2;
    const float t2 = (-b + sq) / a2;
    const float t = (t1 > tmin) ? t1 : t2;
    if (t > tmin && t < tmax) { *t_out = t; return 1; }
    return 0;
}

typedef struct {
    cam_t cam;
    v3 light_center, light_color;
    tri_t* tris;
    uint32_t nT;
    sph_t* sph;
    uint32_t nS;
} scene_t;

static int is_light(v3 e) { return len(e) > 0.0f; }

static int scene_build(scene_t* s, const CameraGPU* cam, const MaterialGPU* mats,
                       const SquareLightGPU* light, const rt_float3* verts, uint32_t nT,
                       const SphereGPU* spheres, uint32_t nS) {
    memset(s, 0, sizeof(*s));
    cam_setup(cam, &s->cam);
    s->light_center = ld3(&light->center);
    s->light_color = mk(light->color.x, light->color.y, light->color.z); /* raytrace.metal:22 */
    s->nT = nT;
    s->nS = nS;
    s->tris = (tri_t*)calloc(nT ? nT : 1, sizeof(tri_t));
    s->sph = (sph_t*)calloc(nS ? nS : 1, sizeof(sph_t));
    if (!s->tris || !s->sph) return -1;
    for (uint32_t k = 0; k < nT; ++k) {
        tri_t* T = &s->tris[k];
        const v3 a = ld3(&verts[3 * k + 0]), b = ld3(&verts[3 * k + 1]), c = ld3(&verts[3 * k + 2]);
        T->v0 = a;
        T->e1 = sub(b, a);              /* sampling.metal:23 */
        T->e2 = sub(c, a);              /* sampling.metal:24 */
        T->n = cross(T->e1, T->e2);
        T->N = nrm(T->n);               /* sampling.metal:25 */
        frame_of(T->N, &T->right, &T->fwd);
        T->diffuse = mk(mats[k].diffuse.x, mats[k].diffuse.y, mats[k].diffuse.z);
        T->emissive = ld3(&mats[k].emissive);
        T->metallic = mats[k].metallic;
        T->roughness = mats[k].roughness;
        T->light = is_light(T->emissive);
    }
    for (uint32_t k = 0; k < nS; ++k) {
        sph_t* S = &s->sph[k];
        S->c = ld3(&spheres[k].center);
        S->r2 = spheres[k].radius * spheres[k].radius;
        const MaterialGPU* m = &spheres[k].material;
        S->diffuse = mk(m->diffuse.x, m->diffuse.y, m->diffuse.z);
        S->emissive = ld3(&m->emissive);
        S->light = is_light(S->emissive);
    }
    return 0;
}

static void scene_free(scene_t* s) {
    free(s->tris);
    free(s->sph);
}

static __thread uint64_t tl_tests;

/* closest hit, accept_any_intersection(false) (raytrace.metal:48-49):
 * returns primitive id (triangles first, then spheres) or -1. */
static int closest(const scene_t* s, v3 o, v3 d, float tmin, float tmax, float* t_out) {
    float best = tmax;
    int id = -1;
    float t;
    for (uint32_t k = 0; k < s->nT; ++k)
        if (tri_hit(&s->tris[k], o, d, tmin, best, &t)) { best = t; id = (int)k; }
    if (s->nS) {
        const float a = dot(d, d);
        for (uint32_t k = 0; k < s->nS; ++k)
            if (sph_hit(&s->sph[k], o, d, a, tmin, best, &t)) { best = t; id = (int)(s->nT + k); }
    }
    tl_tests += s->nT + s->nS;
    *t_out = best;
    return id;
}

/* Primitive id of the closest hit of each pixel's camera ray through the
 * pixel centre (jitter 0.5, 0.5; sampling.metal:125-157 + raytrace.metal:48-49),
 * -1 on a miss: the scene geometry as the camera sees it, compared with the
 * reference's example.png (tests/test_oracle.py). ids: H*W int32. */
int pto_primary_ids(const CameraGPU* cam, const MaterialGPU* mats, const SquareLightGPU* light,
                    const rt_float3* verts, uint32_t n_tri, int32_t* ids) {
    scene_t s;
    if (scene_build(&s, cam, mats, light, verts, n_tri, NULL, 0) != 0) return -1;
    for (int32_t y = 0; y < s.cam.H; ++y)
        for (int32_t x = 0; x < s.cam.W; ++x) {
            float t;
            ids[(size_t)y * s.cam.W + x] =
                closest(&s, s.cam.pos, cam_dir(&s.cam, x, y, 0.5f, 0.5f), 0.001f, 1000.0f, &t);
        }
    scene_free(&s);
    return 0;
}

/* any hit, accept_any_intersection(true) (raytrace.metal:79-85) */
static int occluded(const scene_t* s, v3 o, v3 d, float tmin, float tmax) {
    float t;
    for (uint32_t k = 0; k < s->nT; ++k) {
        if (tri_hit(&s->tris[k], o, d, tmin, tmax, &t)) { tl_tests += k + 1; return 1; }
    }
    tl_tests += s->nT;
    if (s->nS) {
        const float a = dot(d, d);
        for (uint32_t k = 0; k < s->nS; ++k)
            if (sph_hit(&s->sph[k], o, d, a, tmin, tmax, &t)) { tl_tests += k + 1; return 1; }
        tl_tests += s->nS;
    }
    return 0;
}

/* sampleAreaLight (sampling.metal:198-236) */
static v3 area_light(const scene_t* s, float ux, float uy, v3 p, v3* ldir, float* ldist) {
    ux = ux * 2.0f - 1.0f;                                  /* :205 */
    uy = uy * 2.0f - 1.0f;
    const v3 ln = mk(0.0f, -1.0f, 0.0f);                    /* :207 */
    const v3 right = mk(0.25f, 0.0f, 0.0f), up = mk(0.0f, 0.0f, 0.25f);
    const v3 q = add(add(s->light_center, scl(right, ux)), scl(up, uy)); /* :211-213 */
    v3 L = sub(q, p);                                       /* :216 */
    const float dist = len(L);                              /* :218 */
    const float inv = 1.0f / fmaxf(dist, 1e-3f);            /* :220 */
    L = scl(L, inv);                                        /* :223 */
    v3 col = scl(s->light_color, inv * inv);                /* :226-229 */
    col = scl(col, saturate(dot(neg(L), ln)));              /* :233 */
    *ldir = L;
    *ldist = dist;
    return col;
}

void pto_sample_area_light(const SquareLightGPU* light, float ux, float uy, const float p[3],
                           float ldir[3], float* ldist, float color[3]) {
    scene_t s;
    memset(&s, 0, sizeof(s));
    s.light_center = ld3(&light->center);
    s.light_color = mk(light->color.x, light->color.y, light->color.z);
    v3 L;
    v3 c = area_light(&s, ux, uy, mk(p[0], p[1], p[2]), &L, ldist);
    ldir[0] = L.x; ldir[1] = L.y; ldir[2] = L.z;
    color[0] = c.x; color[1] = c.y; color[2] = c.z;
}

/* sampleCosineWeightedHemisphere (sampling.metal:39-49) + align (:51-66) */
static v3 cos_dir(float ux, float uy, v3 N, v3 right, v3 fwd) {
    const float phi = 6.28318548f * ux; /* 2.0f * M_PI_F folded */
    float sp, cp;
    pto_sincos(phi, &sp, &cp);
    const float ct = sqrtf(uy);
    const float st = sqrtf(1.0f - ct * ct);
    const float hx = st * cp, hy = ct, hz = st * sp;
    return add(add(scl(right, hx), scl(N, hy)), scl(fwd, hz));
}

void pto_cosine_direction(float ux, float uy, const float n[3], float d[3]) {
    v3 N = mk(n[0], n[1], n[2]), r, f;
    frame_of(N, &r, &f);
    v3 o = cos_dir(ux, uy, N, r, f);
    d[0] = o.x; d[1] = o.y; d[2] = o.z;
}

/* One sample: raytrace.metal:37-102 */
static v3 trace(const scene_t* s, uint32_t seed, int32_t x, int32_t y, uint32_t n, uint32_t B) {
    const uint32_t i = seed + n;                           /* :37-40 offset + n */
    const float jx = pto_halton(i, 0), jy = pto_halton(i, 1);
    v3 o = s->cam.pos;
    v3 d = cam_dir(&s->cam, x, y, jx, jy);                  /* :42 */
    const float tmin = 0.001f, tmax = 1000.0f;              /* sampling.metal:154-155 */
    v3 acc = mk(0.0f, 0.0f, 0.0f), thr = mk(1.0f, 1.0f, 1.0f);
    for (uint32_t b = 0; b < B; ++b) {                       /* :47 */
        float t;
        const int id = closest(s, o, d, tmin, tmax, &t);     /* :48-49 */
        if (id < 0) break;                                  /* :51-53 */
        v3 N, right, fwd, diffuse;
        if ((uint32_t)id < s->nT) {
            const tri_t* T = &s->tris[id];
            if (T->light) { acc = T->emissive; break; }     /* :57-60 overwrite */
            N = T->N; right = T->right; fwd = T->fwd; diffuse = T->diffuse;
        } else {
            const sph_t* S = &s->sph[id - (int)s->nT];
            if (S->light) { acc = S->emissive; break; }
            N = nrm(sub(add(o, scl(d, t)), S->c));
            frame_of(N, &right, &fwd);
            diffuse = S->diffuse;
        }
        const v3 p = add(add(o, scl(d, t)), scl(N, 1e-3f));  /* :67 */
        v3 L;
        float dist;
        const float lu = pto_halton(i, 2 + b * 5 + 0), lv = pto_halton(i, 2 + b * 5 + 1);
        v3 lc = area_light(s, lu, lv, p, &L, &dist);         /* :72-74 */
        lc = scl(lc, saturate(dot(N, L)));                   /* :75 */
        thr = mul(thr, diffuse);                             /* :76 */
        if (!occluded(s, p, L, 0.0f, dist - 1e-3f))          /* :79-85 */
            acc = add(acc, mul(lc, thr));                    /* :87-89 */
        if (b + 1 < B) { /* the last direction is never traced (A.7) */
            const float cu = pto_halton(i, 2 + b * 5 + 2), cv = pto_halton(i, 2 + b * 5 + 3);
            d = cos_dir(cu, cv, N, right, fwd);              /* :93-97 */
            o = p;                                           /* :99-100 */
        }
    }
    return acc;
}

void pto_trace_sample(const CameraGPU* cam, const MaterialGPU* mats, const SquareLightGPU* light,
                      const rt_float3* verts, uint32_t n_tri, const SphereGPU* spheres,
                      uint32_t n_sph, uint32_t seed, int32_t x, int32_t y, uint32_t n,
                      uint32_t bounces, float acc[3]) {
    scene_t s;
    if (scene_build(&s, cam, mats, light, verts, n_tri, spheres, n_sph)) return;
    v3 a = trace(&s, seed, x, y, n, bounces);
    acc[0] = a.x; acc[1] = a.y; acc[2] = a.z;
    scene_free(&s);
}

int pto_ray_triangle(const float o[3], const float d[3], const float v0[3], const float v1[3],
                     const float v2[3], float tmin, float tmax, float* t) {
    tri_t T;
    memset(&T, 0, sizeof(T));
    T.v0 = mk(v0[0], v0[1], v0[2]);
    T.e1 = sub(mk(v1[0], v1[1], v1[2]), T.v0);
    T.e2 = sub(mk(v2[0], v2[1], v2[2]), T.v0);
    T.n = cross(T.e1, T.e2);
    return tri_hit(&T, mk(o[0], o[1], o[2]), mk(d[0], d[1], d[2]), tmin, tmax, t);
}

int pto_ray_sphere(const float o[3], const float d[3], const float c[3], float radius,
                   float tmin, float tmax, float* t) {
    sph_t S;
    memset(&S, 0, sizeof(S));
    S.c = mk(c[0], c[1], c[2]);
    S.r2 = radius * radius;
    v3 D = mk(d[0], d[1], d[2]);
    return sph_hit(&S, mk(o[0], o[1], o[2]), D, dot(D, D), tmin, tmax, t);
}

/* ---- render -------------------------------------------------------------- */
typedef struct {
    const scene_t* s;
    const uint32_t* seeds;
    uint32_t spp, B, base, row_start, row_step, row_count;
    const float* sum_in;
    float* sum_out;
    float* out;
    uint32_t next_row;
    pthread_mutex_t mu;
    uint64_t tests;
} job_t;

static void render_row(job_t* J, uint32_t j) {
    const scene_t* s = J->s;
    const int32_t W = s->cam.W;
    const int32_t y = (int32_t)(J->row_start + j * J->row_step);
    const uint32_t S = J->sum_in ? J->base + J->spp : J->spp;
    for (int32_t x = 0; x < W; ++x) {
        const size_t o = (size_t)j * (size_t)W + (size_t)x;
        const uint32_t seed = J->seeds[(size_t)y * (size_t)W + (size_t)x]; /* :37 */
        v3 lum = mk(0.0f, 0.0f, 0.0f);                                     /* :32 */
        if (J->sum_in) lum = mk(J->sum_in[4 * o], J->sum_in[4 * o + 1], J->sum_in[4 * o + 2]);
        for (uint32_t n = 0; n < J->spp; ++n)                               /* :34 */
            lum = add(lum, trace(s, seed, x, y, J->base + n, J->B));        /* :103 */
        if (J->sum_out) {
            J->sum_out[4 * o] = lum.x; J->sum_out[4 * o + 1] = lum.y;
            J->sum_out[4 * o + 2] = lum.z; J->sum_out[4 * o + 3] = (float)S;
        }
        if (J->out) {                                                       /* :106-109 */
            const float fs = (float)S;
            J->out[4 * o] = lum.x / fs; J->out[4 * o + 1] = lum.y / fs;
            J->out[4 * o + 2] = lum.z / fs; J->out[4 * o + 3] = 1.0f;
        }
    }
}

static void* worker(void* arg) {
    job_t* J = (job_t*)arg;
    tl_tests = 0;
    for (;;) {
        pthread_mutex_lock(&J->mu);
        const uint32_t j = J->next_row++;
        pthread_mutex_unlock(&J->mu);
        if (j >= J->row_count) break;
        render_row(J, j);
    }
    pthread_mutex_lock(&J->mu);
    J->tests += tl_tests;
    pthread_mutex_unlock(&J->mu);
    return NULL;
}

static uint64_t g_last_tests;
uint64_t pto_last_tests(void) { return g_last_tests; }

int pto_render(const CameraGPU* cam, const MaterialGPU* mats, const SquareLightGPU* light,
               const rt_float3* verts, uint32_t n_tri, const SphereGPU* spheres, uint32_t n_sph,
               const uint32_t* seeds, uint32_t spp, uint32_t bounces, uint32_t sample_base,
               uint32_t row_start, uint32_t row_step, uint32_t row_count, const float* sum_in,
               float* sum_out, float* out, int nthreads) {
    if (!cam || !light || !seeds || bounces > 4 || cam->resolution.x <= 0 || cam->resolution.y <= 0)
        return -1;
    if (n_tri && (!mats || !verts)) return -1;
    if (n_sph && !spheres) return -1;
    if (row_step == 0) row_step = 1;
    if (row_start >= (uint32_t)cam->resolution.y) return -1;
    if (row_count == 0) row_count = ((uint32_t)cam->resolution.y - 1u - row_start) / row_step + 1u;
    if ((uint64_t)row_start + (uint64_t)(row_count - 1) * row_step >= (uint64_t)cam->resolution.y)
        return -1;
    scene_t s;
    if (scene_build(&s, cam, mats, light, verts, n_tri, spheres, n_sph)) return -1;
    job_t J;
    memset(&J, 0, sizeof(J));
    J.s = &s; J.seeds = seeds; J.spp = spp; J.B = bounces; J.base = sample_base;
    J.row_start = row_start; J.row_step = row_step; J.row_count = row_count;
    J.sum_in = sum_in; J.sum_out = sum_out; J.out = out;
    pthread_mutex_init(&J.mu, NULL);
    if (nthreads <= 1) {
        worker(&J);
    } else {
        pthread_t* th = (pthread_t*)calloc((size_t)nthreads, sizeof(pthread_t));
        int started = 0;
        for (int k = 0; k < nthreads; ++k)
            if (pthread_create(&th[k], NULL, worker, &J) == 0) ++started;
        if (started == 0) worker(&J);
        for (int k = 0; k < started; ++k) pthread_join(th[k], NULL);
        free(th);
    }
    pthread_mutex_destroy(&J.mu);
    g_last_tests = J.tests;
    scene_free(&s);
    return 0;
}

/* ---- scene builders (RTrace/scene.swift) ---------------------------------- */
static const float kSwiftPi = 3.14159250f; /* Swift Float.pi is rounded toward zero */

static rt_float3 f3(float x, float y, float z) {
    rt_float3 r;
    memset(&r, 0, sizeof(r));
    r.x = x; r.y = y; r.z = z;
    return r;
}

static MaterialGPU material(float r, float g, float b, float metallic, float roughness,
                            float er, float eg, float eb) {
    MaterialGPU m;
    memset(&m, 0, sizeof(m));
    m.diffuse.x = r; m.diffuse.y = g; m.diffuse.z = b; m.diffuse.w = 1.0f;
    m.metallic = metallic;
    m.roughness = roughness;
    m.emissive = f3(er, eg, eb);
    return m;
}

/* createRotatedBoxVertices (scene.swift:177-210) */
static void box_vertices(float cx, float cy, float cz, float w, float h, float d, float rotY,
                         rt_float3 out[8]) {
    const float hw = w / 2, hh = h / 2, hd = d / 2;
    const float base[8][3] = {{-hw, -hh, -hd}, {hw, -hh, -hd}, {hw, hh, -hd}, {-hw, hh, -hd},
                              {-hw, -hh, hd},  {hw, -hh, hd},  {hw, hh, hd},  {-hw, hh, hd}};
    volatile float angle = rotY; /* run-time libm, never compile-time folded */
    const float c = cosf(angle), s = sinf(angle);
    for (int k = 0; k < 8; ++k) {
        const float x = base[k][0], y = base[k][1], z = base[k][2];
        /* columns (c,0,s,0),(0,1,0,0),(-s,0,c,0),(0,0,0,1) */
        const float rx = c * x + (-s) * z;
        const float rz = s * x + c * z;
        out[k] = f3(rx + cx, y + cy, rz + cz);
    }
}

/* createBoxTriangles face order (scene.swift:212-240) */
static const int kBoxFaces[12][3] = {{0, 2, 1}, {0, 3, 2}, {4, 5, 6}, {4, 6, 7},
                                     {0, 4, 7}, {0, 7, 3}, {1, 6, 5}, {1, 2, 6},
                                     {0, 5, 4}, {0, 1, 5}, {3, 6, 2}, {3, 7, 6}};

static int cornell(int32_t width, int32_t height, float lsize, CameraGPU* cam, MaterialGPU* mats,
                   rt_float3* verts, SquareLightGPU* light, uint32_t* n_tri) {
    if (!cam || !mats || !verts || !light || width <= 0 || height <= 0) return -1;
    memset(cam, 0, sizeof(*cam));
    /* scene.swift:16-18; Camera defaults :290-296 */
    cam->position = f3(0, 0, 9);
    {
        v3 dv = nrm(sub(mk(0, 0, -2.5f), mk(0, 0, 9)));
        cam->direction = f3(dv.x, dv.y, dv.z);
    }
    cam->up = f3(0, 1, 0);
    cam->resolution.x = width;
    cam->resolution.y = height;
    cam->horizontalFov = kSwiftPi / 4.0f;
    cam->ev100 = 5.0f;

    const float half = 5.0f / 2.0f; /* :20-21 */
    const float lightY = half - 0.01f;
    const float hw = lsize / 2, hd = lsize / 2;
    const rt_float3 L0 = f3(0 - hw, lightY, 0 - hd), L1 = f3(0 + hw, lightY, 0 - hd);
    const rt_float3 L2 = f3(0 + hw, lightY, 0 + hd), L3 = f3(0 - hw, lightY, 0 + hd);
    const MaterialGPU lightM = material(1.0f, 0.95f, 0.9f, 0.0f, 0.0f, 1, 1, 1); /* :37-43 */

    const MaterialGPU red = material(0.9f, 0.0f, 0.0f, 0.05f, 0.3f, 0, 0, 0);   /* :72 */
    const MaterialGPU green = material(0.0f, 0.7f, 0.0f, 0.05f, 0.8f, 0, 0, 0); /* :73 */
    const MaterialGPU white = material(0.9f, 0.9f, 0.9f, 0.05f, 0.8f, 0, 0, 0); /* :74 */
    const MaterialGPU boxM = material(0.9f, 0.9f, 0.9f, 0.05f, 0.3f, 0, 0, 0);  /* :75 */

    int k = 0;
#define TRI(a, b, c, m) do { verts[3*k] = (a); verts[3*k+1] = (b); verts[3*k+2] = (c); mats[k] = (m); ++k; } while (0)
    const float h = half;
    TRI(f3(-h, -h, -h), f3(h, h, -h), f3(-h, h, -h), white);  /* back :81-90 */
    TRI(f3(-h, -h, -h), f3(h, -h, -h), f3(h, h, -h), white);
    TRI(f3(-h, -h, -h), f3(-h, h, h), f3(-h, -h, h), red);    /* left :93-102 */
    TRI(f3(-h, -h, -h), f3(-h, h, -h), f3(-h, h, h), red);
    TRI(f3(h, -h, -h), f3(h, h, h), f3(h, h, -h), green);     /* right :105-114 */
    TRI(f3(h, -h, -h), f3(h, -h, h), f3(h, h, h), green);
    TRI(f3(-h, -h, -h), f3(h, -h, h), f3(h, -h, -h), white);  /* floor :117-126 */
    TRI(f3(-h, -h, -h), f3(-h, -h, h), f3(h, -h, h), white);
    TRI(f3(-h, h, -h), f3(h, h, h), f3(-h, h, h), white);     /* ceiling :129-138 */
    TRI(f3(-h, h, -h), f3(h, h, -h), f3(h, h, h), white);
    {
        rt_float3 bv[8];
        const float tallH = 2.8f;
        box_vertices(-1.0f, -half + tallH / 2 - 0.05f, -1.5f, 1.2f, tallH, 1.2f,
                     kSwiftPi / 2.4f, bv);                       /* :141-155 */
        for (int f = 0; f < 12; ++f) TRI(bv[kBoxFaces[f][0]], bv[kBoxFaces[f][1]], bv[kBoxFaces[f][2]], boxM);
        const float shortH = 1.2f;
        box_vertices(0.7f, -half + shortH / 2 - 0.05f, 1.2f, 1.2f, shortH, 1.2f,
                     -kSwiftPi / 2.5f, bv);                      /* :158-172 */
        for (int f = 0; f < 12; ++f) TRI(bv[kBoxFaces[f][0]], bv[kBoxFaces[f][1]], bv[kBoxFaces[f][2]], boxM);
    }
    TRI(L0, L1, L2, lightM); /* :58-59 */
    TRI(L0, L2, L3, lightM);
#undef TRI
    *n_tri = (uint32_t)k;

    /* convertSquareLight (computeShader.swift:33-41), emittedLuminance (scene.swift:257-270) */
    memset(light, 0, sizeof(*light));
    light->center = f3(0, lightY, 0);
    light->color = lightM.diffuse;
    {
        const float flux = 100.0f * 12.0f;
        const float area = lsize * lsize;
        const float lum = (flux / area) / kSwiftPi;
        light->emittedRadiance = f3(1.0f * lum, 0.95f * lum, 0.9f * lum);
    }
    light->width = lsize;
    light->depth = lsize;
    return 0;
}

int pto_cornell_box(int32_t width, int32_t height, CameraGPU* cam, MaterialGPU* mats,
                    rt_float3* verts, SquareLightGPU* light, uint32_t* n_tri) {
    return cornell(width, height, 1.0f, cam, mats, verts, light, n_tri);
}

/* Sources/gpuRaytracer/main.swift:21-67: lightWidth = lightDepth = 1.5 */
int pto_cornell_box_mis(int32_t width, int32_t height, CameraGPU* cam, MaterialGPU* mats,
                        rt_float3* verts, SquareLightGPU* light, uint32_t* n_tri) {
    return cornell(width, height, 1.5f, cam, mats, verts, light, n_tri);
}

/* PCG32 (O'Neill), srandom(initstate=seed, initseq=54) */
typedef struct { uint64_t state, inc; } pcg_t;
static uint32_t pcg_next(pcg_t* r) {
    const uint64_t old = r->state;
    r->state = old * 6364136223846793005ULL + r->inc;
    const uint32_t xs = (uint32_t)(((old >> 18u) ^ old) >> 27u);
    const uint32_t rot = (uint32_t)(old >> 59u);
    return (xs >> rot) | (xs << ((-rot) & 31u));
}
static void pcg_seed(pcg_t* r, uint64_t initstate, uint64_t initseq) {
    r->state = 0;
    r->inc = (initseq << 1u) | 1u;
    pcg_next(r);
    r->state += initstate;
    pcg_next(r);
}
static float pcg_uniform(pcg_t* r, float lo, float hi) {
    return lo + (hi - lo) * ((float)(pcg_next(r) >> 8) * 5.9604645e-08f);
}

int pto_random_spheres(int32_t width, int32_t height, uint32_t n_spheres, uint64_t seed,
                       CameraGPU* cam, MaterialGPU* mats, rt_float3* verts,
                       SquareLightGPU* light, uint32_t* n_tri, SphereGPU* spheres) {
    MaterialGPU m36[36];
    rt_float3 v108[108];
    uint32_t n;
    if (pto_cornell_box(width, height, cam, m36, v108, light, &n)) return -1;
    if (!spheres && n_spheres) return -1;
    int k = 0;
    for (int t = 0; t < 36; ++t) {
        if (t >= 10 && t < 34) continue; /* walls 0-9 and light 34-35 */
        mats[k] = m36[t];
        verts[3 * k] = v108[3 * t]; verts[3 * k + 1] = v108[3 * t + 1]; verts[3 * k + 2] = v108[3 * t + 2];
        ++k;
    }
    *n_tri = (uint32_t)k;
    pcg_t r;
    pcg_seed(&r, seed, 54u);
    for (uint32_t i = 0; i < n_spheres; ++i) {
        SphereGPU* S = &spheres[i];
        memset(S, 0, sizeof(*S));
        const float cx = pcg_uniform(&r, -2.3f, 2.3f);
        const float cy = pcg_uniform(&r, -2.3f, 2.2f);
        const float cz = pcg_uniform(&r, -2.3f, 2.3f);
        const float rad = pcg_uniform(&r, 0.05f, 0.20f);
        const float ar = pcg_uniform(&r, 0.1f, 0.9f);
        const float ag = pcg_uniform(&r, 0.1f, 0.9f);
        const float ab = pcg_uniform(&r, 0.1f, 0.9f);
        S->center = f3(cx, cy, cz);
        S->radius = rad;
        S->material = material(ar, ag, ab, 0.0f, 1.0f, 0, 0, 0);
    }
    return 0;
}

void pto_seed_splitmix(uint64_t key, uint32_t* seeds, size_t n) {
    for (size_t p = 0; p < n; ++p) {
        uint64_t z = key + (uint64_t)p + 0x9E3779B97F4A7C15ULL;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
        z = z ^ (z >> 31);
        seeds[p] = (uint32_t)(z & 0xFFFFFu); /* renderer.swift:100 range [0, 2^20) */
    }
}

/* ---- image.swift:35-65 ----------------------------------------------------- */
static uint16_t f32_to_f16(float f) {
    uint32_t x;
    memcpy(&x, &f, 4);
    const uint32_t sign = (x >> 16) & 0x8000u;
    const uint32_t ex = (x >> 23) & 0xFFu;
    uint32_t man = x & 0x7FFFFFu;
    if (ex == 0xFFu) return (uint16_t)(sign | 0x7C00u | (man ? 0x200u : 0u));
    int e = (int)ex - 127 + 15;
    if (e >= 31) return (uint16_t)(sign | 0x7C00u);
    if (e <= 0) {
        if (e < -10) return (uint16_t)sign;
        man |= 0x800000u;
        const int shift = 14 - e;
        uint32_t h = man >> shift;
        const uint32_t rem = man & ((1u << shift) - 1u), halfway = 1u << (shift - 1);
        if (rem > halfway || (rem == halfway && (h & 1u))) ++h;
        return (uint16_t)(sign | h);
    }
    uint32_t h = ((uint32_t)e << 10) | (man >> 13);
    const uint32_t rem = man & 0x1FFFu;
    if (rem > 0x1000u || (rem == 0x1000u && (h & 1u))) ++h;
    return (uint16_t)(sign | h);
}

static float f16_to_f32(uint16_t h) {
    const uint32_t sign = ((uint32_t)h & 0x8000u) << 16;
    const uint32_t ex = ((uint32_t)h >> 10) & 0x1Fu;
    uint32_t man = (uint32_t)h & 0x3FFu;
    uint32_t x;
    if (ex == 0) {
        if (man == 0) {
            x = sign;
        } else {
            int e = -1;
            do { ++e; man <<= 1; } while (!(man & 0x400u));
            x = sign | ((uint32_t)(127 - 15 - e) << 23) | ((man & 0x3FFu) << 13);
        }
    } else if (ex == 0x1Fu) {
        x = sign | 0x7F800000u | (man << 13);
    } else {
        x = sign | ((ex - 15 + 127) << 23) | (man << 13);
    }
    float f;
    memcpy(&f, &x, 4);
    return f;
}

/* RTrace/image.swift:35-65: the rgba16F texture read back as Float16
 * (:35-38; renderer.swift:74-82 is the texture format), then per RGB channel
 * value *= exposure (2, :41,54); value = value/(value+1) (:55);
 * value = pow(value, 1/gamma) (gamma 2.2, :42,56); max(0, min(1, value)) (:59);
 * UInt8(value*255), truncating (:60); alpha 255 (:63).  pow is the contract's
 * portable pow (pto_pow); a NaN (fp16 inf after Reinhard)
 * skips it, and min(1.0, NaN) is 1.0 in Swift as in C's fminf. */
void pto_tonemap_rgba8(const float* in, size_t n, uint8_t* out) {
    const float exposure = 2.0f, gamma = 2.2f;
    for (size_t i = 0; i < n; ++i) {
        for (int c = 0; c < 3; ++c) {
            float v = f16_to_f32(f32_to_f16(in[4 * i + c]));
            v *= exposure;
            v = v / (v + 1.0f);
            if (v == v) v = pto_pow(v, 1.0f / gamma);
            v = fmaxf(0.0f, fminf(1.0f, v));
            out[4 * i + c] = (uint8_t)(v * 255.0f);
        }
        out[4 * i + 3] = 255;
    }
}


/* ========================================================================
 * MIS integrator: kernel drawTriangle of the SwiftPM build
 * (Sources/gpuRaytracer/shaders.metal:635-707) and its helpers, restated
 * under the same contract.  Every line cites the
 * reference statement it follows.
 * ======================================================================== */

static const float kPiF = 3.14159274f;      /* M_PI_F */
static const float kInvPiF = 0.318309873f;  /* 1.0 / M_PI_F, Fd_Lambert :210-212 */

static float c01(float x) { return fminf(1.0f, fmaxf(0.0f, x)); }
static v3 divs(v3 a, float s) { return mk(a.x / s, a.y / s, a.z / s); }

/* hash, randomFloat, hashRandom (:58-85) */
static uint32_t mis_hash(uint32_t x) {
    x ^= x >> 16;
    x *= 0x7feb352dU;
    x ^= x >> 15;
    x *= 0x846ca68bU;
    x ^= x >> 16;
    return x;
}
static float random_float(uint32_t seed) {
    /* float(hash) / (float(0xffffffffU) + 1.0): the denominator is 2^32 in
     * float, so the quotient is the exact product below */
    return (float)mis_hash(seed) * 2.3283064365386963e-10f;
}

/* buildOrthonormalBasis (:159-172) */
static void mis_onb(v3 n, v3* t, v3* b) {
    v3 a;
    if (fabsf(n.x) > 0.9f) a = mk(0.0f, 1.0f, 0.0f);
    else a = mk(1.0f, 0.0f, 0.0f);
    *t = nrm(sub(a, scl(n, dot(a, n))));
    *b = cross(n, *t);
}

/* D_GGX, F_Schlick, V_SmithGGXCorrelated, smithG1_GGX (:186-208) */
static float d_ggx(float NoH, float a) {
    const float a2 = a * a;
    const float f = (NoH * a2 - NoH) * NoH + 1.0f;
    return a2 / (kPiF * f * f);
}
static float pow5(float x) { const float x2 = x * x; return (x2 * x2) * x; } /* DESIGN §3.11 */
static v3 f_schlick(float LoH, v3 f0) {
    const float p = pow5(1.0f - LoH);
    return mk(f0.x + (1.0f - f0.x) * p, f0.y + (1.0f - f0.y) * p, f0.z + (1.0f - f0.z) * p);
}
static float v_smith(float NoV, float NoL, float a) {
    const float a2 = a * a;
    const float GGXL = NoV * sqrtf((-NoL * a2 + NoL) * NoL + a2);
    const float GGXV = NoL * sqrtf((-NoV * a2 + NoV) * NoV + a2);
    return 0.5f / (GGXV + GGXL);
}
static float smith_g1(float NoV, float roughness) {
    const float a = roughness * roughness;
    const float a2 = a * a;
    const float NoV2 = NoV * NoV;
    return 2.0f / (1.0f + sqrtf(1.0f + a2 * (1.0f - NoV2) / NoV2));
}

typedef enum { MIS_HIT, MIS_HIT_LIGHT, MIS_MISS } mis_type;
typedef struct {          /* IntersectionGPU (:14-20) */
    mis_type type;
    v3 point;
    v3 ro, rd;            /* ray */
    v3 normal;
    const tri_t* mat;     /* material (diffuse, metallic, roughness) */
} mis_isect;

typedef struct {
    v3 center, tangent, bitangent, radiance;
    float width, depth;
} mis_light;

/* getClosestIntersection (:459-509), rays in (min, max) per DESIGN.md §3.5 */
static mis_isect closest_isect(const scene_t* s, v3 o, v3 d, float tmin, float tmax) {
    mis_isect r;
    memset(&r, 0, sizeof(r));
    float t;
    const int id = closest(s, o, d, tmin, tmax, &t);
    if (id < 0) { r.type = MIS_MISS; return r; }
    const tri_t* T = &s->tris[id];
    r.point = add(o, scl(d, t));
    r.mat = T;
    if (T->light) { r.type = MIS_HIT_LIGHT; return r; }
    r.type = MIS_HIT;
    r.ro = o;
    r.rd = d;
    r.normal = T->N;  /* getTriangleNormal (:447-457) */
    return r;
}

/* calculateBRDFContribution (:259-289) */
static v3 brdf(v3 ray_d, v3 n, const tri_t* m, v3 l) {
    const v3 v = neg(nrm(ray_d));
    const v3 h = nrm(add(v, l));
    const float NoV = fabsf(dot(n, v)) + 1e-5f;
    const float NoL = c01(dot(n, l));
    const float NoH = c01(dot(n, h));
    const float LoH = c01(dot(l, h));
    const v3 f0 = mk(0.04f + (m->diffuse.x - 0.04f) * m->metallic,   /* mix(0.04, diffuse, metallic) */
                     0.04f + (m->diffuse.y - 0.04f) * m->metallic,
                     0.04f + (m->diffuse.z - 0.04f) * m->metallic);
    const float D = d_ggx(NoH, m->roughness);
    const v3 F = f_schlick(LoH, f0);
    const float G = v_smith(NoV, NoL, m->roughness);
    const float den = 4.0f * NoV * NoL + 1e-7f;
    const v3 Fr = divs(scl(F, D * G), den);
    const v3 Fd = scl(m->diffuse, kInvPiF);
    const v3 kD = scl(sub(mk(1.0f, 1.0f, 1.0f), F), 1.0f - m->metallic);
    return scl(mul(kD, add(Fd, Fr)), NoL);
}

/* calculateSquareLightPdf (:315-326) */
static float light_pdf(const mis_light* L, v3 origin, v3 dir) {
    const v3 toL = sub(L->center, origin);
    const float dist = len(toL);
    const float cosT = fmaxf(0.0f, dot(neg(dir), mk(0.0f, -1.0f, 0.0f)));
    const float area = L->width * L->depth;
    return (dist * dist) / (area * cosT + 1e-6f);
}

/* calculateCosineWeightedPdf (:376-380) */
static float cosine_pdf(v3 n, v3 d) { return fmaxf(0.0f, dot(n, d)) / kPiF; }

/* calculateVNDFPdf (:437-445) */
static float vndf_pdf(v3 V, v3 n, v3 L, float roughness) {
    const v3 h = nrm(add(V, L));
    const float NoH = fabsf(dot(n, h));
    const float VoH = fabsf(dot(V, h));
    const float NoV = fabsf(dot(n, V));
    const float D = d_ggx(NoH, roughness);
    const float G1 = smith_g1(NoV, roughness);
    return (D * G1 * VoH) / (4.0f * NoV);
}

/* powerHeuristic, beta = 1 (:132-137): pow(x, 1) = x */
static float power_h(float p1, float p2, float p3, uint32_t spp) {
    const float n = (float)spp;
    const float a = n * p1;
    const float sum = a + n * p2 + n * p3;
    return a / (sum + 1e-6f);
}

/* cosineWeightedRay (:355-374): direction */
static v3 cosine_ray_dir(v3 n, float ux, float uy) {
    const float phi = 2.0f * kPiF * ux;
    const float cosT = sqrtf(uy);
    const float sinT = sqrtf(1.0f - uy);
    v3 t, b;
    mis_onb(n, &t, &b);
    float sp, cp;
    pto_sincos(phi, &sp, &cp);
    return nrm(add(add(scl(t, cp * sinT), scl(b, sp * sinT)), scl(n, cosT)));
}

/* vndfRay (:382-435): direction */
static v3 vndf_ray_dir(v3 V, v3 n, float roughness, float ux, float uy) {
    const float alpha = roughness * roughness;
    v3 T, B;
    mis_onb(n, &T, &B);
    const v3 Ve = nrm(mk(alpha * dot(V, T), alpha * dot(V, B), dot(V, n)));
    const v3 T1 = nrm(mk(Ve.z, 0.0f, -Ve.x));
    const v3 T2 = cross(Ve, T1);
    const float phi = 2.0f * kPiF * ux;
    const float lenVe = len(Ve);
    const float ctm = lenVe / sqrtf(1.0f + lenVe * lenVe);
    const float ct = ctm + (1.0f - ctm) * uy;
    const float st = sqrtf(1.0f - ct * ct);
    float sp, cp;
    pto_sincos(phi, &sp, &cp);
    const v3 h = nrm(add(add(scl(T1, cp * st), scl(T2, sp * st)), scl(Ve, ct)));
    const v3 Nh = nrm(mk(alpha * h.x, alpha * h.y, fmaxf(0.0f, h.z)));
    const v3 wH = nrm(add(add(scl(T, Nh.x), scl(B, Nh.y)), scl(n, Nh.z)));
    const v3 I = neg(V);
    return sub(I, scl(wH, 2.0f * dot(wH, I)));  /* reflect(I, wH) = I - 2*dot(wH,I)*wH */
}

/* calculateDirectLightSamplingContribution (:519-541) */
static v3 direct_light(const scene_t* s, const mis_light* L, const mis_isect* x, float ux,
                       float uy, uint32_t spp, int use_power) {
    v3 direct = mk(0.0f, 0.0f, 0.0f);
    /* directSquareLightRay(point + normal * 1e-4, light, u) (:291-313) */
    const v3 origin = add(x->point, scl(x->normal, 1e-4f));
    const float sx = (ux - 0.5f) * L->width;
    const float sy = (uy - 0.5f) * L->depth;
    const v3 sp = add(add(L->center, scl(L->tangent, sx)), scl(L->bitangent, sy));
    const v3 toL = sub(sp, origin);
    const float dist = len(toL);
    const v3 ldir = divs(toL, dist);
    const mis_isect li = closest_isect(s, origin, ldir, 0.001f, dist);
    if (li.type == MIS_HIT_LIGHT) {
        const float dl_pdf = light_pdf(L, x->point, ldir);
        const v3 c = brdf(x->rd, x->normal, x->mat, ldir);
        if (use_power) {
            const float cos_pdf = cosine_pdf(x->normal, ldir);
            const float v_pdf = vndf_pdf(neg(x->rd), x->normal, ldir, x->mat->roughness);
            const float w = power_h(dl_pdf, cos_pdf, v_pdf, spp);
            direct = add(direct, divs(mul(scl(c, w), L->radiance), dl_pdf));
        } else {
            direct = add(direct, divs(mul(c, L->radiance), dl_pdf));
        }
    }
    return direct;
}

/* recursiveMultiImportanceSampling (:543-625) */
static v3 mis_estimate(const scene_t* s, const mis_light* L, const mis_isect* x, uint32_t samples) {
    const uint32_t S = samples / 3;
    v3 dl = mk(0, 0, 0), cs = mk(0, 0, 0), vn = mk(0, 0, 0);
    for (uint32_t i = 0; i < S; ++i)  /* :553-560, haltonRandom(i, 0) */
        dl = add(dl, direct_light(s, L, x, pto_halton(i, 0), pto_halton(i, 1), S, 1));
    const v3 origin = add(x->point, scl(x->normal, 1e-4f));
    const v3 V = neg(x->rd);
    for (uint32_t i = 0; i < S; ++i) {  /* :562-591 */
        const v3 dir = cosine_ray_dir(x->normal, pto_halton(i + S, 2), pto_halton(i + S, 3));
        const float cos_pdf = cosine_pdf(x->normal, dir);
        const float dl_pdf = light_pdf(L, x->point, dir);
        const float v_pdf = vndf_pdf(V, x->normal, dir, x->mat->roughness);
        const float w = power_h(cos_pdf, dl_pdf, v_pdf, S);
        const mis_isect y = closest_isect(s, origin, dir, 0.001f, 1000.0f);
        const v3 c = brdf(x->rd, x->normal, x->mat, dir);
        if (y.type == MIS_HIT_LIGHT) {
            cs = add(cs, divs(mul(scl(c, w), L->radiance), cos_pdf));
        } else if (y.type == MIS_HIT) {
            const v3 nee = direct_light(s, L, &y, pto_halton(i, 6), pto_halton(i, 7), 1, 0);
            cs = add(cs, mul(divs(c, cos_pdf), nee));
        }
    }
    for (uint32_t i = 0; i < S; ++i) {  /* :593-623 */
        const v3 dir = vndf_ray_dir(V, x->normal, x->mat->roughness, pto_halton(i + 2 * S, 4),
                                    pto_halton(i + 2 * S, 5));
        const float v_pdf = vndf_pdf(V, x->normal, dir, x->mat->roughness);
        const float cos_pdf = cosine_pdf(x->normal, dir);
        const float dl_pdf = light_pdf(L, x->point, dir);
        const float w = power_h(v_pdf, dl_pdf, cos_pdf, S);
        const mis_isect y = closest_isect(s, origin, dir, 0.001f, 1000.0f);
        const v3 c = brdf(x->rd, x->normal, x->mat, dir);
        if (y.type == MIS_HIT_LIGHT) {
            vn = add(vn, divs(mul(scl(c, w), L->radiance), v_pdf));
        } else if (y.type == MIS_HIT) {
            const v3 nee = direct_light(s, L, &y, pto_halton(i + S, 6), pto_halton(i + S, 7), 1, 0);
            vn = add(vn, mul(divs(c, v_pdf), nee));
        }
    }
    return divs(add(add(dl, cs), vn), (float)S);
}

/* portable log / exp / pow of DESIGN.md §3.11 (cephes logf / expf) */
static uint32_t fbits(float x) { uint32_t u; memcpy(&u, &x, 4); return u; }
static float bitsf(uint32_t u) { float x; memcpy(&x, &u, 4); return x; }
static float log_pt(float x) {
    const uint32_t bx = fbits(x);
    int e = (int)(bx >> 23) - 126;
    float m = bitsf((bx & 0x007FFFFFu) | 0x3F000000u);
    if (m < 0.707106781f) { e -= 1; m = m + m - 1.0f; } else { m = m - 1.0f; }
    const float z = m * m;
    float y = 7.0376836292e-2f;
    y = fmaf(y, m, -1.1514610310e-1f);
    y = fmaf(y, m, 1.1676998740e-1f);
    y = fmaf(y, m, -1.2420140846e-1f);
    y = fmaf(y, m, 1.4249322787e-1f);
    y = fmaf(y, m, -1.6668057665e-1f);
    y = fmaf(y, m, 2.0000714765e-1f);
    y = fmaf(y, m, -2.4999993993e-1f);
    y = fmaf(y, m, 3.3333331174e-1f);
    y = (y * m) * z;
    const float fe = (float)e;
    y = fmaf(fe, -2.12194440e-4f, y);
    y = fmaf(-0.5f, z, y);
    return fmaf(fe, 0.693359375f, m + y);
}
static float exp_pt(float x) {
    const float z = floorf(x * 1.44269504088896341f + 0.5f);
    float r = fmaf(-z, 0.693359375f, x);
    r = fmaf(-z, -2.12194440e-4f, r);
    float p = 1.9875691500e-4f;
    p = fmaf(p, r, 1.3981999507e-3f);
    p = fmaf(p, r, 8.3334519073e-3f);
    p = fmaf(p, r, 4.1665795894e-2f);
    p = fmaf(p, r, 1.6666665459e-1f);
    p = fmaf(p, r, 5.0000001201e-1f);
    const float y = fmaf(p, r * r, r) + 1.0f;
    return y * bitsf((uint32_t)((int)z + 127) << 23);
}
float pto_pow(float x, float y) {
    if (!(x > 7.88860905e-31f)) return 0.0f;
    return exp_pt(y * log_pt(x));
}

typedef struct {
    const scene_t* s;
    mis_light L;
    uint32_t camera_rays, samples, row_start, row_step, row_count;
    float exposure;
    float* out;
    uint8_t* out8;
    uint32_t next_row;
    pthread_mutex_t mu;
} mis_job_t;

static void mis_row(mis_job_t* J, uint32_t j) {
    const scene_t* s = J->s;
    const int32_t W = s->cam.W;
    const uint32_t y = J->row_start + j * J->row_step;
    for (int32_t xi = 0; xi < W; ++xi) {
        const uint32_t x = (uint32_t)xi;
        v3 acc = mk(0.0f, 0.0f, 0.0f);                       /* :645 */
        for (uint32_t i = 0; i < J->camera_rays; ++i) {      /* :652 */
            const uint32_t sample_id = (y * 800u + x) * i;   /* hashRandom :73 */
            const float jx = random_float(x + y * 800u + sample_id);            /* :77,81 */
            const float jy = random_float(y + x * 600u + sample_id + 12345u);   /* :78,82 */
            const v3 d = cam_dir(&s->cam, (int32_t)x, (int32_t)y, jx, jy);     /* :214-246 */
            const mis_isect h = closest_isect(s, s->cam.pos, d, 0.001f, 1000.0f); /* :660 */
            if (h.type == MIS_MISS) {
            } else if (h.type == MIS_HIT_LIGHT) {
                acc = add(acc, J->L.radiance);                 /* :669-670 */
            } else {
                acc = add(acc, mis_estimate(s, &J->L, &h, J->samples)); /* :674-676 */
            }
        }
        const size_t o = (size_t)j * (size_t)W + (size_t)xi;
        const float nc = (float)J->camera_rays;
        if (J->out) {  /* textBuffer (:705) + the divisor */
            J->out[4 * o] = acc.x; J->out[4 * o + 1] = acc.y;
            J->out[4 * o + 2] = acc.z; J->out[4 * o + 3] = nc;
        }
        if (J->out8) {  /* :688-706 */
            const float e[3] = {acc.x / nc * J->exposure, acc.y / nc * J->exposure,
                                acc.z / nc * J->exposure};
            for (int k = 0; k < 3; ++k) {
                const float tm = c01(e[k] / (e[k] + 1.0f));
                const float g = pto_pow(tm, 1.0f / 2.2f);
                J->out8[4 * o + k] = (uint8_t)(g * 255.0f);
            }
            J->out8[4 * o + 3] = 255;
        }
    }
}

static void* mis_worker(void* arg) {
    mis_job_t* J = (mis_job_t*)arg;
    for (;;) {
        pthread_mutex_lock(&J->mu);
        const uint32_t j = J->next_row++;
        pthread_mutex_unlock(&J->mu);
        if (j >= J->row_count) break;
        mis_row(J, j);
    }
    return NULL;
}

int pto_render_mis(const CameraGPU* cam, const MaterialGPU* mats, const SquareLightGPU* light,
                   const rt_float3* verts, uint32_t n_tri, uint32_t camera_rays,
                   uint32_t mis_samples, uint32_t row_start, uint32_t row_step,
                   uint32_t row_count, float* out, uint8_t* out8, int nthreads) {
    if (!cam || !light || !mats || !verts || n_tri == 0 || camera_rays == 0 || mis_samples < 3)
        return -1;
    if (cam->resolution.x <= 0 || cam->resolution.y <= 0) return -1;
    if (row_step == 0) row_step = 1;
    if (row_start >= (uint32_t)cam->resolution.y) return -1;
    if (row_count == 0) row_count = ((uint32_t)cam->resolution.y - 1u - row_start) / row_step + 1u;
    if ((uint64_t)row_start + (uint64_t)(row_count - 1) * row_step >= (uint64_t)cam->resolution.y)
        return -1;
    scene_t s;
    if (scene_build(&s, cam, mats, light, verts, n_tri, NULL, 0)) return -1;
    mis_job_t J;
    memset(&J, 0, sizeof(J));
    J.s = &s;
    J.L.center = ld3(&light->center);
    mis_onb(mk(0.0f, -1.0f, 0.0f), &J.L.tangent, &J.L.bitangent);  /* :292-293 */
    J.L.radiance = ld3(&light->emittedRadiance);
    J.L.width = light->width;
    J.L.depth = light->depth;
    {
        volatile float ev = cam->ev100;                        /* cameraExposure :145-150 */
        J.exposure = 1.0f / (1.2f * powf(2.0f, ev));
    }
    J.camera_rays = camera_rays;
    J.samples = mis_samples;
    J.row_start = row_start;
    J.row_step = row_step;
    J.row_count = row_count;
    J.out = out;
    J.out8 = out8;
    pthread_mutex_init(&J.mu, NULL);
    if (nthreads <= 1) {
        mis_worker(&J);
    } else {
        pthread_t* th = (pthread_t*)calloc((size_t)nthreads, sizeof(pthread_t));
        int started = 0;
        for (int k = 0; k < nthreads; ++k)
            if (pthread_create(&th[k], NULL, mis_worker, &J) == 0) ++started;
        if (started == 0) mis_worker(&J);
        for (int k = 0; k < started; ++k) pthread_join(th[k], NULL);
        free(th);
    }
    pthread_mutex_destroy(&J.mu);
    scene_free(&s);
    return 0;
}
