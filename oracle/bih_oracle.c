/*
 * bih_oracle.c -- TEST INFRASTRUCTURE ONLY (see bih_oracle.h).
 *
 * Plain-C, strict IEEE binary32 restatement of the reference's hot path.
 * Compile with -ffp-contract=off and without -ffast-math (oracle/Makefile).
 * Every function cites the reference file:line it restates; paths are
 * relative to BIH_Raytracer/BIH_Raytracer/.
 */
#include "bih_oracle.h"

#include <float.h>
#include <math.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#ifdef _OPENMP
#include <omp.h>
#endif

/* ------------------------------------------------------------------ */
/* small helpers                                                        */
/* ------------------------------------------------------------------ */
static inline uint32_t f2u(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }
static inline float u2f(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }

/* CUDA __clz: count leading zeros, __clz(0) == 32. */
static inline int clz32(uint32_t x) { return x ? __builtin_clz(x) : 32; }

/* Total order used by atomicMaxFloat / atomicMinFloat (CUDAKernels.cu:52-66):
 * signed-int compare for non-negative values, unsigned for negative ones,
 * i.e. the IEEE totalOrder on non-NaN floats (-0 < +0). */
static inline int32_t tkey(float f) {
    uint32_t u = f2u(f);
    return (u & 0x80000000u) ? (int32_t)(~u) ^ (int32_t)0x80000000 : (int32_t)u;
}
static inline float tmax(float a, float b) { return tkey(b) > tkey(a) ? b : a; }
static inline float tmin(float a, float b) { return tkey(b) < tkey(a) ? b : a; }

/* std::minmax over an initializer list: leftmost smallest, rightmost
 * largest (App.cpp:123-125). */
static inline float first_min3(float a, float b, float c) {
    float m = a; if (b < m) m = b; if (c < m) m = c; return m;
}
static inline float last_max3(float a, float b, float c) {
    float m = a; if (!(b < m)) m = b; if (!(c < m)) m = c; return m;
}

/* ------------------------------------------------------------------ */
/* Morton codes -- Renderer.cpp:114-145                                 */
/* ------------------------------------------------------------------ */
static inline uint32_t expand_bits(uint32_t v) {
    v = (v * 0x00010001u) & 0xFF0000FFu;
    v = (v * 0x00000101u) & 0x0F00F00Fu;
    v = (v * 0x00000011u) & 0xC30C30C3u;
    v = (v * 0x00000005u) & 0x49249249u;
    return v;
}

uint32_t ob_morton3d(float x, float y, float z) {
    /* CUDA min/max(float,float) == fminf/fmaxf (NaN -> other operand) */
    x = fminf(fmaxf(x * 1024.0f, 0.0f), 1023.0f);
    y = fminf(fmaxf(y * 1024.0f, 0.0f), 1023.0f);
    z = fminf(fmaxf(z * 1024.0f, 0.0f), 1023.0f);
    uint32_t xx = expand_bits((uint32_t)x);
    uint32_t yy = expand_bits((uint32_t)y);
    uint32_t zz = expand_bits((uint32_t)z);
    return xx * 4 + yy * 2 + zz;
}

/* ------------------------------------------------------------------ */
/* Build: App.cpp:103-164 (host prep), Renderer.cpp:422-503 (pipeline), */
/* CUDAKernels.cu:591-710 (BuildTree), :497-549 (FindClipPlanes)        */
/* ------------------------------------------------------------------ */
typedef struct { uint32_t code; uint32_t idx; } kv_t;

static int kv_cmp(const void *a, const void *b) {
    const kv_t *x = (const kv_t *)a, *y = (const kv_t *)b;
    if (x->code != y->code) return x->code < y->code ? -1 : 1;
    return x->idx < y->idx ? -1 : (x->idx > y->idx);   /* stability */
}

static void karras_node(const uint32_t *umc, int U, uint32_t idx, ob_tree *T) {
    /* BuildTree, CUDAKernels.cu:591-710, with its uint32/int mixing. */
    uint32_t cur = umc[idx];
    uint32_t pre[2] = {0xFFFFFFFFu, 0xFFFFFFFFu};
    if (idx) pre[0] = (uint32_t)clz32(cur ^ umc[idx - 1]);
    if (idx < (uint32_t)(U - 1)) pre[1] = (uint32_t)clz32(cur ^ umc[idx + 1]);
    int32_t diff = (int32_t)(pre[1] - pre[0]);
    int d = (0 < diff) - (diff < 0);                       /* signum */
    int lcp_min = (int32_t)pre[1 - ((d + 1) / 2)];
    int lmax = 1, lcp = -2, li;
    do {
        lmax *= 2;
        li = (int32_t)(idx + (uint32_t)(lmax * d));
        lcp = (li < 0 || li > U - 1) ? -1 : clz32(cur ^ umc[li]);
    } while (lcp > lcp_min);
    int l = 0;
    for (int t = lmax / 2; t >= 1; t /= 2) {
        int ti = (int32_t)(idx + (uint32_t)((l + t) * d));
        lcp = (ti < 0 || ti > U - 1) ? -1 : clz32(cur ^ umc[ti]);
        if (lcp > lcp_min) l += t;
    }
    int other = (int32_t)(idx + (uint32_t)(l * d));
    int lcp_ends = clz32(cur ^ umc[other]);
    int s = 0, t = l;
    for (;;) {
        t = (int)ceilf((float)t / 2.0f);                   /* __float2int_ru(t/2.0f) */
        int ti = (int32_t)(idx + (uint32_t)((s + t) * d));
        lcp = (ti < 0 || ti > U - 1) ? -1 : clz32(cur ^ umc[ti]);
        if (lcp > lcp_ends) s += t;
        if (t == 1) break;
    }
    int split = (int32_t)(idx + (uint32_t)(s * d)) + (d < 0 ? d : 0);
    T->children[2 * idx + 0] = split;
    T->children[2 * idx + 1] = split + 1;
    uint32_t mn = idx < (uint32_t)other ? idx : (uint32_t)other;
    uint32_t mx = idx > (uint32_t)other ? idx : (uint32_t)other;
    T->is_leaf[2 * idx + 0] = (mn == (uint32_t)split);
    T->is_leaf[2 * idx + 1] = (mx == (uint32_t)(split + 1));
    if (T->is_leaf[2 * idx + 0]) T->leaf_parent[split] = (int32_t)idx;
    else T->parent[split] = (int32_t)idx;
    if (T->is_leaf[2 * idx + 1]) T->leaf_parent[split + 1] = (int32_t)idx;
    else T->parent[split + 1] = (int32_t)idx;
    int lcp_ch = clz32(umc[split] ^ umc[split + 1]);
    T->axis[idx] = (lcp_ch + 1) % 3;
}

int ob_build(const float *v, int32_t n, ob_tree **out) {
    if (!out || n < 0 || (n > 0 && !v)) return -1;
    ob_tree *T = (ob_tree *)calloc(1, sizeof(ob_tree));
    if (!T) return -4;
    T->n_tris = n;
    size_t n3 = (size_t)n * 3, nn = n > 0 ? (size_t)n : 1;
    T->lo = (float *)malloc(n3 * 4 + 4); T->hi = (float *)malloc(n3 * 4 + 4);
    T->center = (float *)malloc(n3 * 4 + 4); T->norm = (float *)malloc(n3 * 4 + 4);
    T->morton = (uint32_t *)malloc(nn * 4); T->tri_idx = (uint32_t *)malloc(nn * 4);
    T->unique_mc = (uint32_t *)malloc(nn * 4); T->dup_cnt = (uint32_t *)malloc(nn * 4);
    T->first_idx = (int32_t *)malloc(nn * 4); T->leaf_parent = (int32_t *)malloc(nn * 4);
    T->clip = (float *)malloc(nn * 8); T->axis = (int32_t *)malloc(nn * 4);
    T->children = (int32_t *)malloc(nn * 8); T->is_leaf = (uint8_t *)malloc(nn * 2);
    T->parent = (int32_t *)malloc(nn * 4);
    T->tris = (float *)malloc((size_t)nn * 36);
    if (!T->lo || !T->hi || !T->center || !T->norm || !T->morton || !T->tri_idx ||
        !T->unique_mc || !T->dup_cnt || !T->first_idx || !T->leaf_parent || !T->clip ||
        !T->axis || !T->children || !T->is_leaf || !T->parent || !T->tris) {
        ob_free(T); return -4;
    }
    if (n == 0) { T->n_unique = 0; *out = T; return 0; }
    memcpy(T->tris, v, (size_t)n * 36);

    /* host prep, App.cpp:103-156 */
    float slo[3] = {v[0], v[1], v[2]}, shi[3] = {v[0], v[1], v[2]};
    for (int32_t i = 0; i < n; ++i) {
        const float *p = v + 9 * (size_t)i;
        for (int a = 0; a < 3; ++a) {
            float lo = first_min3(p[a], p[3 + a], p[6 + a]);
            float hi = last_max3(p[a], p[3 + a], p[6 + a]);
            T->lo[3 * (size_t)i + a] = lo;
            T->hi[3 * (size_t)i + a] = hi;
            T->center[3 * (size_t)i + a] = (lo + hi) / 2.0f;
            /* std::minmax({lo, hi, slo, shi}) */
            slo[a] = (slo[a] < lo) ? slo[a] : lo;
            shi[a] = (shi[a] < hi) ? hi : shi[a];
        }
    }
    for (int a = 0; a < 3; ++a) { T->scene_lo[a] = slo[a]; T->scene_hi[a] = shi[a]; }
    for (int32_t i = 0; i < n; ++i)
        for (int a = 0; a < 3; ++a) {
            float num = T->center[3 * (size_t)i + a] - slo[a];
            float den = shi[a] - slo[a];
            T->norm[3 * (size_t)i + a] = num / den;
        }

    /* Morton + stable sort by key, Renderer.cpp:422-445 */
    kv_t *kv = (kv_t *)malloc((size_t)n * sizeof(kv_t));
    if (!kv) { ob_free(T); return -4; }
    for (int32_t i = 0; i < n; ++i) {
        kv[i].code = ob_morton3d(T->norm[3 * (size_t)i], T->norm[3 * (size_t)i + 1],
                                 T->norm[3 * (size_t)i + 2]);
        kv[i].idx = (uint32_t)i;
    }
    qsort(kv, (size_t)n, sizeof(kv_t), kv_cmp);
    for (int32_t i = 0; i < n; ++i) { T->morton[i] = kv[i].code; T->tri_idx[i] = kv[i].idx; }
    free(kv);

    /* reduce_by_key + unique_by_key_copy, Renderer.cpp:450-472 */
    int32_t U = 0;
    for (int32_t i = 0; i < n; ++i) {
        if (i == 0 || T->morton[i] != T->morton[i - 1]) {
            T->unique_mc[U] = T->morton[i];
            T->first_idx[U] = i;
            T->dup_cnt[U] = 1;
            ++U;
        } else {
            T->dup_cnt[U - 1]++;
        }
    }
    T->n_unique = U;

    /* initial values, GPUArrayManager.cpp:60-85 */
    for (int32_t k = 0; k < U; ++k) T->leaf_parent[k] = -1;
    for (int32_t i = 0; i < U - 1; ++i) {
        T->parent[i] = -1;
        T->children[2 * i] = T->children[2 * i + 1] = -1;
        T->axis[i] = -1;
        T->clip[2 * i] = -FLT_MAX;
        T->clip[2 * i + 1] = FLT_MAX;
        T->is_leaf[2 * i] = T->is_leaf[2 * i + 1] = 0;
    }
    for (int32_t i = 0; i + 1 < U; ++i) karras_node(T->unique_mc, U, (uint32_t)i, T);

    /* FindClipPlanes, CUDAKernels.cu:497-549 */
    for (int32_t k = 0; k < U && U > 1; ++k) {
        int32_t f = T->first_idx[k];
        uint32_t c = T->dup_cnt[k];
        const float *l0 = T->lo + 3 * (size_t)T->tri_idx[f];
        const float *h0 = T->hi + 3 * (size_t)T->tri_idx[f];
        float blo[3] = {l0[0], l0[1], l0[2]}, bhi[3] = {h0[0], h0[1], h0[2]};
        for (int32_t i = f; i < f + (int32_t)c; ++i) {
            const float *l = T->lo + 3 * (size_t)T->tri_idx[i];
            const float *h = T->hi + 3 * (size_t)T->tri_idx[i];
            for (int a = 0; a < 3; ++a) { blo[a] = tmin(blo[a], l[a]); bhi[a] = tmax(bhi[a], h[a]); }
        }
        int32_t prev = k, par = T->leaf_parent[k];
        while (par != -1) {
            int ax = T->axis[par];
            if (T->children[2 * par] == prev) T->clip[2 * par] = tmax(T->clip[2 * par], bhi[ax]);
            if (T->children[2 * par + 1] == prev) T->clip[2 * par + 1] = tmin(T->clip[2 * par + 1], blo[ax]);
            prev = par;
            par = T->parent[par];
        }
    }
    *out = T;
    return 0;
}

void ob_free(ob_tree *T) {
    if (!T) return;
    free(T->lo); free(T->hi); free(T->center); free(T->norm); free(T->morton);
    free(T->tri_idx); free(T->unique_mc); free(T->dup_cnt); free(T->first_idx);
    free(T->leaf_parent); free(T->clip); free(T->axis); free(T->children);
    free(T->is_leaf); free(T->parent); free(T->tris); free(T);
}

/* ------------------------------------------------------------------ */
/* Camera -- Camera.cu:5-9 (double arithmetic rounded to f32),          */
/* Renderer.cpp:99                                                       */
/* ------------------------------------------------------------------ */
void ob_camera_reference(uint32_t w, uint32_t h, float cam[12]) {
    float aspect = (float)w / (float)h;
    float o[3] = {2.0f, 0.0f, -2.0f};
    cam[0] = o[0]; cam[1] = o[1]; cam[2] = o[2];
    cam[3] = (float)((double)o[0] - 2.0);
    cam[4] = (float)((double)o[1] - 1.0);
    cam[5] = (float)((double)o[2] + 1.0);
    cam[6] = (float)((double)aspect * 2.0); cam[7] = 0.0f; cam[8] = 0.0f;
    cam[9] = 0.0f; cam[10] = 2.0f; cam[11] = 0.0f;
}

/* ------------------------------------------------------------------ */
/* cuRAND XORWOW (curand_kernel.h of CUDA 12.0, restated; not vendored) */
/* used by InitRandGPU CUDAKernels.cu:450-459 and cudaRender :411-419    */
/* ------------------------------------------------------------------ */
static void xorwow_lin_step(uint32_t v[5]) {
    uint32_t t = v[0] ^ (v[0] >> 2);
    v[0] = v[1]; v[1] = v[2]; v[2] = v[3]; v[3] = v[4];
    v[4] = (v[4] ^ (v[4] << 4)) ^ (t ^ (t << 1));
}

/* 160x160 GF(2) matrices stored by column: col[b] = image of unit vector b */
typedef struct { uint32_t c[160][5]; } gf2m;

static void gf2_apply(const gf2m *A, uint32_t x[5]) {
    uint32_t r[5] = {0, 0, 0, 0, 0};
    for (int b = 0; b < 160; ++b)
        if ((x[b >> 5] >> (b & 31)) & 1u)
            for (int w = 0; w < 5; ++w) r[w] ^= A->c[b][w];
    memcpy(x, r, sizeof r);
}
static void gf2_mul(const gf2m *A, const gf2m *B, gf2m *C) {   /* C = A*B */
    for (int b = 0; b < 160; ++b) {
        uint32_t x[5]; memcpy(x, B->c[b], sizeof x);
        gf2_apply(A, x);
        memcpy(C->c[b], x, sizeof x);
    }
}

static gf2m g_step_pow[64];      /* M^(2^k)          */
static gf2m g_seq_pow[64];       /* M^(2^(67+k))     */
static int g_rng_ready = 0;

static void rng_tables_init(void) {
    if (__atomic_load_n(&g_rng_ready, __ATOMIC_ACQUIRE)) return;
#pragma omp critical(ob_rng_init)
    {
        if (!g_rng_ready) {
            static gf2m tmp;
            for (int b = 0; b < 160; ++b) {
                uint32_t x[5] = {0, 0, 0, 0, 0};
                x[b >> 5] = 1u << (b & 31);
                xorwow_lin_step(x);
                memcpy(g_step_pow[0].c[b], x, sizeof x);
            }
            for (int k = 1; k < 64; ++k) gf2_mul(&g_step_pow[k - 1], &g_step_pow[k - 1], &g_step_pow[k]);
            /* M^(2^67) = square M^(2^63) four more times */
            tmp = g_step_pow[63];
            for (int k = 0; k < 4; ++k) { gf2m sq; gf2_mul(&tmp, &tmp, &sq); tmp = sq; }
            g_seq_pow[0] = tmp;
            for (int k = 1; k < 64; ++k) gf2_mul(&g_seq_pow[k - 1], &g_seq_pow[k - 1], &g_seq_pow[k]);
            __atomic_store_n(&g_rng_ready, 1, __ATOMIC_RELEASE);
        }
    }
}

void ob_rng_state(uint64_t seed, uint64_t subsequence, uint64_t skip,
                  uint32_t v[5], uint32_t *d) {
    rng_tables_init();
    uint32_t s0 = (uint32_t)seed ^ 0xaad26b49u;
    uint32_t s1 = (uint32_t)(seed >> 32) ^ 0xf7dcefddu;
    uint32_t t0 = 1099087573u * s0;
    uint32_t t1 = 2591861531u * s1;
    *d = 6615241u + t1 + t0;
    v[0] = 123456789u + t0;
    v[1] = 362436069u ^ t0;
    v[2] = 521288629u + t1;
    v[3] = 88675123u ^ t1;
    v[4] = 5783321u + t0;
    for (int k = 0; subsequence; ++k, subsequence >>= 1)
        if (subsequence & 1) gf2_apply(&g_seq_pow[k], v);
    /* d unchanged by whole subsequences: 2^67 * 362437 == 0 mod 2^32 */
    uint64_t n = skip;
    for (int k = 0; n; ++k, n >>= 1)
        if (n & 1) gf2_apply(&g_step_pow[k], v);
    *d += (uint32_t)skip * 362437u;
}

uint32_t ob_rng_next(uint32_t v[5], uint32_t *d) {
    xorwow_lin_step(v);
    *d += 362437u;
    return v[4] + *d;
}

float ob_rng_uniform(uint32_t v[5], uint32_t *d) {
    /* _curand_uniform: x * CURAND_2POW32_INV + CURAND_2POW32_INV/2 */
    uint32_t x = ob_rng_next(v, d);
    return (float)x * 2.3283064e-10f + (2.3283064e-10f / 2.0f);
}

/* ------------------------------------------------------------------ */
/* Ray + MT -- Ray.cu:3-10, CUDAKernels.cu:17-50 (glm 0.9.9.4 order)    */
/* ------------------------------------------------------------------ */
typedef struct { float o[3], d[3], inv[3]; int sign[3]; } ray_t;

static inline void make_ray(const float o[3], const float d[3], ray_t *r) {
    for (int a = 0; a < 3; ++a) {
        r->o[a] = o[a]; r->d[a] = d[a];
        r->inv[a] = 1.0f / d[a];
        r->sign[a] = r->inv[a] < 0.0f;
    }
}

static inline float dot3(const float a[3], const float b[3]) {
    float x = a[0] * b[0], y = a[1] * b[1], z = a[2] * b[2];
    return (x + y) + z;                       /* func_geometric.inl:48-54 */
}
static inline void cross3(const float x[3], const float y[3], float r[3]) {
    r[0] = x[1] * y[2] - y[1] * x[2];         /* func_geometric.inl:68-78 */
    r[1] = x[2] * y[0] - y[2] * x[0];
    r[2] = x[0] * y[1] - y[0] * x[1];
}

static inline int mt_test(const float *tri, const ray_t *r, float *t_out) {
    float e1[3] = {tri[3] - tri[0], tri[4] - tri[1], tri[5] - tri[2]};
    float e2[3] = {tri[6] - tri[0], tri[7] - tri[1], tri[8] - tri[2]};
    float p[3]; cross3(r->d, e2, p);
    float det = dot3(e1, p);
    if ((double)det < 0.000001) return 0;     /* double compare, :28 */
    float inv = (float)(1.0 / (double)det);   /* :31 */
    float s[3] = {r->o[0] - tri[0], r->o[1] - tri[1], r->o[2] - tri[2]};
    float u = dot3(s, p) * inv;
    if (u < 0.0f || u > 1.0f) return 0;
    float q[3]; cross3(s, e1, q);
    float vv = dot3(r->d, q) * inv;
    if (vv < 0.0f || u + vv > 1.0f) return 0;
    *t_out = dot3(e2, q) * inv;
    return 1;
}

int ob_mt(const float tri[9], const float o[3], const float d[3], float *t_out) {
    ray_t r; make_ray(o, d, &r);
    return mt_test(tri, &r, t_out);
}

/* ------------------------------------------------------------------ */
/* Traversal                                                            */
/* ------------------------------------------------------------------ */
typedef struct { uint64_t nodes, leaves, tris; int max_stack; uint64_t push_at[33]; } cnt_t;
typedef struct { double t; int idx; } hit_t;   /* HitRecord, Tree.cuh:9-14 */

/* FindNearestTriangle, CUDAKernels.cu:206-224.  Returns 1 when anyhit and
 * a valid hit was recorded (early exit requested). */
static inline int find_nearest(const ob_tree *T, const ray_t *r, int leaf,
                               hit_t *rec, cnt_t *c, int anyhit) {
    c->leaves++;
    int32_t f = T->first_idx[leaf];
    int32_t e = f + (int32_t)T->dup_cnt[leaf];
    float t = FLT_MAX;
    for (int32_t i = f; i < e; ++i) {
        c->tris++;
        if (mt_test(T->tris + 9 * (size_t)T->tri_idx[i], r, &t)) {
            if (t > 0.0f && (double)t < rec->t) {
                rec->t = t; rec->idx = i;
                if (anyhit) return 1;
            }
        }
    }
    return 0;
}

/* C4 closest-hit rule over a leaf (see bih_oracle.h): min (t, i) with
 * t_lo < t < FLT_MAX; order-independent. */
static inline void find_closest(const ob_tree *T, const ray_t *r, int leaf, float t_lo,
                                float *bt, int32_t *bi, cnt_t *c) {
    c->leaves++;
    int32_t f = T->first_idx[leaf];
    int32_t e = f + (int32_t)T->dup_cnt[leaf];
    for (int32_t i = f; i < e; ++i) {
        float t;
        c->tris++;
        if (!mt_test(T->tris + 9 * (size_t)T->tri_idx[i], r, &t)) continue;
        if (!(t > t_lo && t < FLT_MAX)) continue;
        if (t < *bt || (t == *bt && i < *bi)) { *bt = t; *bi = i; }
    }
}

static int slab(const ob_tree *T, const ray_t *r, float *tmin_o, float *tmax_o) {
    /* CUDAKernels.cu:237-262 */
    const float *bb[2] = {T->scene_lo, T->scene_hi};
    float tmin = (bb[r->sign[0]][0] - r->o[0]) * r->inv[0];
    float tmax = (bb[1 - r->sign[0]][0] - r->o[0]) * r->inv[0];
    float tymin = (bb[r->sign[1]][1] - r->o[1]) * r->inv[1];
    float tymax = (bb[1 - r->sign[1]][1] - r->o[1]) * r->inv[1];
    if ((tmin > tymax) || (tymin > tmax)) return 0;
    if (tymin > tmin) tmin = tymin;
    if (tymax < tmax) tmax = tymax;
    float tzmin = (bb[r->sign[2]][2] - r->o[2]) * r->inv[2];
    float tzmax = (bb[1 - r->sign[2]][2] - r->o[2]) * r->inv[2];
    if ((tmin > tzmax) || (tzmin > tmax)) return 0;
    if (tzmin > tmin) tmin = tzmin;
    if (tzmax < tmax) tmax = tzmax;
    *tmin_o = tmin; *tmax_o = tmax;
    return 1;
}

typedef struct { int node; float tmin, tmax; } stk_t;   /* StackElement */

/* TraverseTree, CUDAKernels.cu:227-368.  Returns 1 on hit, -1 on slab miss. */
static int traverse_gpu_ref(const ob_tree *T, const ray_t *r, cnt_t *c, int anyhit) {
    hit_t rec = {(double)FLT_MAX, -1};
    float tMin, tMax;
    if (!slab(T, r, &tMin, &tMax)) return -1;
    int U = T->n_unique;
    if (U <= 0) return 0;
    if (U == 1) {   /* reference: UB (reads BIHTree[0] default node); defined here */
        find_nearest(T, r, 0, &rec, c, anyhit);
        return rec.idx >= 0;
    }
    stk_t stack[64];
    int sp = 0;
    stack[sp].node = -1; sp++;
    int cur = 0;
    while (cur != -1) {
        c->nodes++;
        int ax = T->axis[cur];
        float org = r->o[ax], inv = r->inv[ax];
        int nr = r->sign[ax], fr = 1 - nr;
        float t[2];
        t[0] = (T->clip[2 * cur] - org) * inv;
        t[1] = (T->clip[2 * cur + 1] - org) * inv;
        int A = tMin < t[nr];
        int B = tMax < t[fr];
        const int32_t *ch = T->children + 2 * cur;
        const uint8_t *lf = T->is_leaf + 2 * cur;
        int pop = 0;
        if (!A && B) {
            pop = 1;
        } else if (A && B) {
            if (lf[nr]) { if (find_nearest(T, r, ch[nr], &rec, c, anyhit)) return 1; pop = 1; }
            else { cur = ch[nr]; tMax = t[nr]; }
        } else if (!A && !B) {
            if (lf[fr]) { if (find_nearest(T, r, ch[fr], &rec, c, anyhit)) return 1; pop = 1; }
            else { cur = ch[fr]; tMin = t[fr]; }
        } else {
            if (lf[nr] && lf[fr]) {
                if (find_nearest(T, r, ch[nr], &rec, c, anyhit)) return 1;
                if (find_nearest(T, r, ch[fr], &rec, c, anyhit)) return 1;
                pop = 1;
            } else if (!lf[nr] && lf[fr]) {
                if (find_nearest(T, r, ch[fr], &rec, c, anyhit)) return 1;
                cur = ch[nr]; tMax = t[nr];
            } else if (lf[nr] && !lf[fr]) {
                if (find_nearest(T, r, ch[nr], &rec, c, anyhit)) return 1;
                cur = ch[fr]; tMin = t[fr];
            } else {
                stack[sp].node = ch[fr]; stack[sp].tmin = t[fr]; stack[sp].tmax = tMax;
                sp++;
                if (sp - 1 > c->max_stack) c->max_stack = sp - 1;
                c->push_at[sp - 1 < 32 ? sp - 1 : 32]++;   /* stack slot written */
                cur = ch[nr]; tMax = t[nr];
            }
        }
        if (pop) {
            sp--;
            cur = stack[sp].node; tMin = stack[sp].tmin; tMax = stack[sp].tmax;
        }
    }
    return rec.idx >= 0;
}

/* The reference walk (traverse_gpu_ref's decisions and order) with the C4
 * closest-hit rule at its leaves and front-to-back culling: before each node
 * a node entered beyond the best hit so far (tMin > best) is popped, and tMax
 * is clamped to the best hit (tMax = min(tMax, best), best = +inf until the
 * first hit, so the walk is the reference's until then).  A secondary ray
 * (t_lo > 0) starts inside the scene box: its walk interval starts at t_lo
 * (tMin = max(box entry, t_lo)) rather than at the box entry behind its
 * origin, where no accepted hit can lie (round 4; primary rays, t_lo = 0,
 * keep the reference's interval). */
static void traverse_closest(const ob_tree *T, const ray_t *r, float t_lo, float *bt, int32_t *bi,
                             cnt_t *c) {
    *bt = FLT_MAX; *bi = -1;
    float tMin, tMax;
    if (!slab(T, r, &tMin, &tMax)) return;
    if (t_lo > 0.0f && tMin < t_lo) tMin = t_lo;
    int U = T->n_unique;
    if (U <= 0) return;
    if (U == 1) { find_closest(T, r, 0, t_lo, bt, bi, c); return; }
    stk_t stack[64];
    int sp = 0;
    stack[sp].node = -1; sp++;
    int cur = 0;
    while (cur != -1) {
        const float best = *bi >= 0 ? *bt : INFINITY;
        if (tMin > best) {                       /* entered beyond the best hit: skip */
            sp--;
            cur = stack[sp].node; tMin = stack[sp].tmin; tMax = stack[sp].tmax;
            continue;
        }
        if (best < tMax) tMax = best;
        c->nodes++;
        int ax = T->axis[cur];
        float org = r->o[ax], inv = r->inv[ax];
        int nr = r->sign[ax], fr = 1 - nr;
        float t[2];
        t[0] = (T->clip[2 * cur] - org) * inv;
        t[1] = (T->clip[2 * cur + 1] - org) * inv;
        int A = tMin < t[nr];
        int B = tMax < t[fr];
        const int32_t *ch = T->children + 2 * cur;
        const uint8_t *lf = T->is_leaf + 2 * cur;
        int pop = 0;
        if (!A && B) {
            pop = 1;
        } else if (A && B) {
            if (lf[nr]) { find_closest(T, r, ch[nr], t_lo, bt, bi, c); pop = 1; }
            else { cur = ch[nr]; tMax = t[nr]; }
        } else if (!A && !B) {
            if (lf[fr]) { find_closest(T, r, ch[fr], t_lo, bt, bi, c); pop = 1; }
            else { cur = ch[fr]; tMin = t[fr]; }
        } else {
            if (lf[nr] && lf[fr]) {
                find_closest(T, r, ch[nr], t_lo, bt, bi, c);
                find_closest(T, r, ch[fr], t_lo, bt, bi, c);
                pop = 1;
            } else if (!lf[nr] && lf[fr]) {
                find_closest(T, r, ch[fr], t_lo, bt, bi, c);
                cur = ch[nr]; tMax = t[nr];
            } else if (lf[nr] && !lf[fr]) {
                find_closest(T, r, ch[nr], t_lo, bt, bi, c);
                cur = ch[fr]; tMin = t[fr];
            } else {
                stack[sp].node = ch[fr]; stack[sp].tmin = t[fr]; stack[sp].tmax = tMax;
                sp++;
                cur = ch[nr]; tMax = t[nr];
            }
        }
        if (pop) {
            sp--;
            cur = stack[sp].node; tMin = stack[sp].tmin; tMax = stack[sp].tmax;
        }
    }
}

int ob_closest(const ob_tree *T, const float o[3], const float d[3], float t_lo,
               float *t_out, int32_t *idx_out) {
    if (!T || !o || !d || !t_out || !idx_out) return -1;
    ray_t r; make_ray(o, d, &r);
    cnt_t c; memset(&c, 0, sizeof c);
    traverse_closest(T, &r, t_lo, t_out, idx_out, &c);
    return 0;
}

/* C4: hits along the mirror path of one primary ray, 0..OB_WHITTED_BOUNCES+1 */
static int whitted_path(const ob_tree *T, const float o0[3], const float d0[3], cnt_t *c,
                        uint64_t *rays) {
    float o[3] = {o0[0], o0[1], o0[2]}, d[3] = {d0[0], d0[1], d0[2]};
    int hits = 0;
    for (int depth = 0; depth <= OB_WHITTED_BOUNCES; ++depth) {
        ray_t r; make_ray(o, d, &r);
        float t; int32_t i;
        (*rays)++;
        traverse_closest(T, &r, depth ? 1e-4f : 0.0f, &t, &i, c);
        if (i < 0) break;
        hits++;
        if (depth == OB_WHITTED_BOUNCES) break;
        const float *v = T->tris + 9 * (size_t)T->tri_idx[i];
        float e1[3] = {v[3] - v[0], v[4] - v[1], v[5] - v[2]};
        float e2[3] = {v[6] - v[0], v[7] - v[1], v[8] - v[2]};
        float n[3]; cross3(e1, e2, n);
        float dn = dot3(d, n), nn = dot3(n, n);
        float k = (2.0f * dn) / nn;
        float p[3], rd[3];
        for (int a = 0; a < 3; ++a) {
            float td = t * d[a];
            p[a] = o[a] + td;
            float kn = k * n[a];
            rd[a] = d[a] - kn;
        }
        memcpy(o, p, sizeof p);
        memcpy(d, rd, sizeof rd);
    }
    return hits;
}

/* shade of a sample with h hits (bih_oracle.h), f32 */
static void whitted_shade(int h, float col[3]) {
    float c[3];
    if (h > OB_WHITTED_BOUNCES) { c[0] = 255.0f; c[1] = 255.0f; c[2] = 0.0f; h = OB_WHITTED_BOUNCES; }
    else { c[0] = 20.0f; c[1] = 20.0f; c[2] = 40.0f; }
    /* h hits at depths 0..h-1, each: 0.5*Y + 0.5*(deeper) */
    for (int d = h - 1; d >= 0; --d) {
        c[0] = 0.5f * 255.0f + 0.5f * c[0];
        c[1] = 0.5f * 255.0f + 0.5f * c[1];
        c[2] = 0.5f * 0.0f + 0.5f * c[2];
    }
    col[0] = c[0]; col[1] = c[1]; col[2] = c[2];
}

/* CPUTraverseTree, Renderer.cpp:202-349 (host debug semantics; the
 * debug-only ID==9 bookkeeping and printf are side effects, not restated). */
static int traverse_host_debug(const ob_tree *T, const ray_t *r, cnt_t *c) {
    hit_t rec = {(double)FLT_MAX, -1};
    float tMin, tMax;
    if (!slab(T, r, &tMin, &tMax)) return -1;
    int U = T->n_unique;
    if (U <= 0) return 0;
    if (U == 1) { find_nearest(T, r, 0, &rec, c, 0); return rec.idx >= 0; }
    stk_t stack[64];
    int sp = 0;
    stack[sp].node = -1; sp++;
    int cur = 0;
    while (cur != -1) {
        c->nodes++;
        int ax = T->axis[cur];
        float org = r->o[ax], inv = r->inv[ax];
        int nr = r->sign[ax], fr = 1 - nr;
        float t[2];
        t[0] = (T->clip[2 * cur] - org) * inv;
        t[1] = (T->clip[2 * cur + 1] - org) * inv;
        int A = tMin < t[nr];
        int B = tMax < t[fr];
        int noI = !A && B, nearI = A && B, bothI = A && !B;
        const int32_t *ch = T->children + 2 * cur;
        const uint8_t *lf = T->is_leaf + 2 * cur;
        if (lf[nr] || lf[fr]) {
            if (lf[nr] && !lf[fr]) { find_nearest(T, r, ch[nr], &rec, c, 0); cur = ch[fr]; }
            else if (lf[fr] && !lf[nr]) { find_nearest(T, r, ch[fr], &rec, c, 0); cur = ch[nr]; }
            else {
                find_nearest(T, r, ch[nr], &rec, c, 0);
                find_nearest(T, r, ch[fr], &rec, c, 0);
                sp--; cur = stack[sp].node; tMin = stack[sp].tmin; tMax = stack[sp].tmax;
            }
        } else if (noI) {
            sp--; cur = stack[sp].node; tMin = stack[sp].tmin; tMax = stack[sp].tmax;
        } else if (bothI) {
            if (sp >= 63) return rec.idx >= 0;   /* reference would overflow; bounded here */
            stack[sp].node = ch[fr]; stack[sp].tmin = tMin; stack[sp].tmax = tMax; sp++;
            if (sp - 1 > c->max_stack) c->max_stack = sp - 1;
            cur = ch[nr];
        } else {
            float tmn = nearI ? tMin : t[fr];
            float tmx = nearI ? t[nr] : tMax;
            cur = nearI ? ch[nr] : ch[fr];
            tMin = tmn; tMax = tmx;
        }
    }
    return rec.idx >= 0;
}

/* all-triangles closest hit (restates the intent of TraverseTriangles,
 * CUDAKernels.cu:157-202, over every leaf of the sorted order). */
static int traverse_brute(const ob_tree *T, const ray_t *r, cnt_t *c) {
    hit_t rec = {(double)FLT_MAX, -1};
    for (int32_t k = 0; k < T->n_unique; ++k) find_nearest(T, r, k, &rec, c, 0);
    return rec.idx >= 0;
}

static inline int trace_one(const ob_tree *T, const ray_t *r, int mode, cnt_t *c) {
    switch (mode) {
    case OB_MODE_GPU_REF: return traverse_gpu_ref(T, r, c, 0);
    case OB_MODE_GPU_ANYHIT: return traverse_gpu_ref(T, r, c, 1);
    case OB_MODE_HOST_DEBUG: return traverse_host_debug(T, r, c);
    default: return traverse_brute(T, r, c);
    }
}

/* clamp/rgbToInt, CUDAKernels.cu:74-88 */
static inline uint32_t rgb_to_int(float r, float g, float b) {
    r = fmaxf(0.0f, fminf(255.0f, r));
    g = fmaxf(0.0f, fminf(255.0f, g));
    b = fmaxf(0.0f, fminf(255.0f, b));
    return ((uint32_t)(int)b << 16) | ((uint32_t)(int)g << 8) | (uint32_t)(int)r;
}

static double now_s(void) {
    struct timespec ts; clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

static int render_impl(const ob_tree *T, const float cam[12], uint32_t w, uint32_t h,
                       uint32_t spp, uint32_t frame, uint64_t seed,
                       uint32_t row0, uint32_t nrows, uint32_t row_step,
                       uint32_t *out, int mode, int nthreads, ob_stats *stats,
                       uint32_t *ray_counts, int whitted, uint8_t *depth_out) {
    if (!T || !cam || !out || w == 0 || h == 0 || spp == 0 || row_step == 0) return -1;
    if ((uint64_t)row0 + (uint64_t)(nrows ? nrows - 1 : 0) * row_step >= h && nrows) return -1;
    rng_tables_init();
    /* per-pixel RNG states at the start of this frame (InitRandGPU + the
     * states cudaRender left behind after `frame` earlier frames) */
    size_t npix = (size_t)nrows * w;
    uint32_t *rv = (uint32_t *)malloc(npix * 6 * sizeof(uint32_t) + 4);
    if (!rv) return -4;
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#endif
#pragma omp parallel for schedule(dynamic, 1)
    for (int64_t k = 0; k < (int64_t)nrows; ++k) {
        uint32_t y = row0 + (uint32_t)k * row_step;
        uint32_t *s0 = rv + (size_t)k * w * 6;
        ob_rng_state(seed, (uint64_t)y * w, (uint64_t)2 * spp * frame, s0, s0 + 5);
        for (uint32_t x = 1; x < w; ++x) {   /* next subsequence = one more 2^67 jump */
            uint32_t *s = s0 + (size_t)x * 6;
            memcpy(s, s - 6, 6 * sizeof(uint32_t));
            gf2_apply(&g_seq_pow[0], s);
        }
    }
    uint64_t g_nodes = 0, g_leaves = 0, g_tris = 0, g_hit = 0, g_miss = 0;
    int g_max = 0, used = 1;
    uint64_t g_push[33];
    memset(g_push, 0, sizeof g_push);
    double t0 = now_s();
#pragma omp parallel reduction(+ : g_nodes, g_leaves, g_tris, g_hit, g_miss) reduction(max : g_max)
    {
#ifdef _OPENMP
#pragma omp single
        used = omp_get_num_threads();
#endif
#pragma omp for schedule(dynamic, 1)
        for (int64_t k = 0; k < (int64_t)nrows; ++k) {
            uint32_t j = row0 + (uint32_t)k * row_step;
            cnt_t c;
            memset(&c, 0, sizeof c);
            for (uint32_t i = 0; i < w; ++i) {
                uint32_t *s = rv + ((size_t)k * w + i) * 6;
                float col[3] = {0.0f, 0.0f, 0.0f};
                for (uint32_t sm = 0; sm < spp; ++sm) {
                    /* cudaRender, CUDAKernels.cu:413-418 */
                    float u = (float)((float)i + ob_rng_uniform(s, s + 5)) / (float)w;
                    float v = (float)((float)j + ob_rng_uniform(s, s + 5)) / (float)h;
                    float d[3];
                    for (int a = 0; a < 3; ++a) {   /* Camera::GetRay, Camera.cu:18-20 */
                        float hu = u * cam[6 + a];
                        float vv = v * cam[9 + a];
                        d[a] = ((cam[3 + a] + hu) + vv) - cam[a];
                    }
                    if (whitted) {
                        uint64_t nr = 0;
                        int hh = whitted_path(T, cam, d, &c, &nr);
                        if (depth_out) depth_out[((size_t)k * w + i) * spp + sm] = (uint8_t)hh;
                        g_hit += (uint64_t)(hh > 0);
                        g_miss += nr;      /* rays traced (primary + secondary) */
                        float sc[3];
                        whitted_shade(hh, sc);
                        col[0] += sc[0]; col[1] += sc[1]; col[2] += sc[2];
                        continue;
                    }
                    ray_t r; make_ray(cam, d, &r);
                    uint64_t n0 = c.nodes, l0 = c.leaves, t0r = c.tris;
                    int hit = trace_one(T, &r, mode, &c);
                    if (ray_counts) {
                        uint32_t *rc = ray_counts + 3 * (((size_t)k * w + i) * spp + sm);
                        rc[0] = (uint32_t)(c.nodes - n0);
                        rc[1] = (uint32_t)(c.leaves - l0);
                        rc[2] = (uint32_t)(c.tris - t0r);
                    }
                    if (hit < 0) { g_miss++; hit = 0; }
                    g_hit += (uint64_t)hit;
                    /* Color, CUDAKernels.cu:384-388 */
                    col[0] += hit ? 255.0f : 20.0f;
                    col[1] += hit ? 255.0f : 20.0f;
                    col[2] += hit ? 0.0f : 40.0f;
                }
                float fs = (float)spp;
                out[(size_t)k * w + i] = rgb_to_int(col[0] / fs, col[1] / fs, col[2] / fs);
            }
            g_nodes += c.nodes; g_leaves += c.leaves; g_tris += c.tris;
            if (c.max_stack > g_max) g_max = c.max_stack;
#pragma omp critical(ob_push_hist)
            for (int q = 0; q < 33; ++q) g_push[q] += c.push_at[q];
        }
    }
    double t1 = now_s();
    free(rv);
    if (stats) {
        stats->rays = (uint64_t)npix * spp;
        stats->rays_hit = g_hit;
        stats->node_visits = g_nodes;
        stats->leaf_visits = g_leaves;
        stats->tri_tests = g_tris;
        stats->slab_miss = g_miss;
        stats->max_stack = g_max;
        stats->threads = used;
        stats->render_seconds = t1 - t0;
        for (int q = 0; q < 33; ++q) stats->push_at[q] = g_push[q];
    }
    return 0;
}

int ob_render(const ob_tree *T, const float cam[12], uint32_t w, uint32_t h,
              uint32_t spp, uint32_t frame, uint64_t seed,
              uint32_t row0, uint32_t nrows, uint32_t row_step,
              uint32_t *out, int mode, int nthreads, ob_stats *stats,
              uint32_t *ray_counts) {
    return render_impl(T, cam, w, h, spp, frame, seed, row0, nrows, row_step, out, mode, nthreads,
                       stats, ray_counts, 0, NULL);
}

/* stats->slab_miss counts every ray traced (primary + secondary) here. */
int ob_render_whitted(const ob_tree *T, const float cam[12], uint32_t w, uint32_t h,
                      uint32_t spp, uint32_t frame, uint64_t seed,
                      uint32_t row0, uint32_t nrows, uint32_t row_step,
                      uint32_t *out, int nthreads, ob_stats *stats, uint8_t *depth_out) {
    return render_impl(T, cam, w, h, spp, frame, seed, row0, nrows, row_step, out, OB_MODE_GPU_REF,
                       nthreads, stats, NULL, 1, depth_out);
}

int ob_trace_rays(const ob_tree *T, const float *orig, const float *dir, int32_t n,
                  int mode, uint8_t *hit, uint32_t *nodes, uint32_t *tris) {
    if (!T || (n > 0 && (!orig || !dir || !hit))) return -1;
    for (int32_t i = 0; i < n; ++i) {
        ray_t r; make_ray(orig + 3 * (size_t)i, dir + 3 * (size_t)i, &r);
        cnt_t c;
        memset(&c, 0, sizeof c);
        int h = trace_one(T, &r, mode, &c);
        hit[i] = (uint8_t)(h > 0);
        if (nodes) nodes[i] = (uint32_t)c.nodes;
        if (tris) tris[i] = (uint32_t)c.tris;
    }
    return 0;
}
