// bih_render.hip -- primary-ray render kernel for gfx950 (MI355X).
//
// Replaces cudaRender (reference src/CUDAKernels.cu:391-423) and its callees
// Camera::GetRay (Camera.cu:18-20), Ray::Ray (Ray.cu:3-10), Color (:370-389),
// TraverseTree (:227-368), FindNearestTriangle (:206-224) and
// RayTriangleIntersection (:17-50); and InitRandGPU (:450-459).
//
// Numerics: every f32 operation is the reference's, in the reference's order
// (glm 0.9.9.4 dot = (x+y)+z, cross as func_geometric.inl:68-78), compiled
// with -ffp-contract=off and IEEE division, so results are bit-exact against
// the strict-IEEE oracle.  `det < 0.000001` (a double compare) is the f32
// compare det <= 0x1.0c6f7ap-20f; `1.0 / det` rounded to f32 is the correctly
// rounded f32 reciprocal (double rounding is innocuous for division).
#include <hip/hip_runtime.h>
#include <float.h>

#include <mutex>

#include "bih_internal.h"

namespace bih {
namespace {

constexpr int kThreads = 256;
constexpr float kDetEps = 9.99999997475242708e-07f;   // 0x358637bd: largest f32 < 1e-6
constexpr uint32_t kWeyl = 362437u;

// ---------------------------------------------------------------------------
// RNG init: v = M^skip * J^pixel * seed_state (J = M^(2^67)).
// ---------------------------------------------------------------------------
__device__ __forceinline__ void gf2_apply(const uint32_t *__restrict__ m, uint32_t x[5]) {
    uint32_t r0 = 0, r1 = 0, r2 = 0, r3 = 0, r4 = 0;
    for (int w = 0; w < 5; ++w) {
        uint32_t bits = x[w];
        while (bits) {
            int b = __ffs(bits) - 1;
            bits &= bits - 1;
            const uint32_t *c = m + (w * 32 + b) * 5;
            r0 ^= c[0]; r1 ^= c[1]; r2 ^= c[2]; r3 ^= c[3]; r4 ^= c[4];
        }
    }
    x[0] = r0; x[1] = r1; x[2] = r2; x[3] = r3; x[4] = r4;
}

__device__ __forceinline__ uint32_t global_row(uint32_t lr, uint32_t row0, uint32_t band_h,
                                               uint32_t band_step) {
    return row0 + (lr / band_h) * band_h * band_step + (lr % band_h);
}

__global__ void __launch_bounds__(kThreads) k_rng_init(uint32_t *__restrict__ rng, uint32_t w,
                                                       uint32_t row0, uint32_t nrows, uint32_t band_h,
                                                       uint32_t band_step, uint32_t s0, uint32_t s1,
                                                       uint32_t s2, uint32_t s3, uint32_t s4,
                                                       unsigned long long skip,
                                                       const uint32_t *__restrict__ tables) {
    const uint64_t P = (uint64_t)nrows * w;
    uint64_t lp = (uint64_t)blockIdx.x * kThreads + threadIdx.x;
    if (lp >= P) return;
    uint32_t lr = (uint32_t)(lp / w), x = (uint32_t)(lp % w);
    uint64_t pix = (uint64_t)global_row(lr, row0, band_h, band_step) * w + x;
    uint32_t v[5] = {s0, s1, s2, s3, s4};
    const uint32_t *seq = tables, *step = tables + 32 * 800;
    for (int k = 0; pix && k < 32; ++k, pix >>= 1)
        if (pix & 1) gf2_apply(seq + k * 800, v);
    for (int k = 0; skip && k < 64; ++k, skip >>= 1)
        if (skip & 1) gf2_apply(step + k * 800, v);
#pragma unroll
    for (int i = 0; i < 5; ++i) rng[(uint64_t)i * P + lp] = v[i];
}

// ---------------------------------------------------------------------------
// Traversal
// ---------------------------------------------------------------------------
struct Ray {
    float o[3], d[3], inv[3];
    uint32_t sgn[3];
};

__device__ __forceinline__ float pick3(const float v[3], uint32_t a) {
    return a == 0 ? v[0] : (a == 1 ? v[1] : v[2]);
}
__device__ __forceinline__ uint32_t pick3u(const uint32_t v[3], uint32_t a) {
    return a == 0 ? v[0] : (a == 1 ? v[1] : v[2]);
}

// RayTriangleIntersection + the t>0 && t<rec.t record test of
// FindNearestTriangle.  Returns true when the triangle sets rec.triangleIdx.
// With rec.t starting at FLT_MAX (Color, :380-382) "some triangle was
// recorded" == "some tested triangle has MT true and 0 < t < FLT_MAX".
__device__ __forceinline__ bool tri_hit(const float *__restrict__ tp, const Ray &r) {
    float v0x = tp[0], v0y = tp[1], v0z = tp[2];
    float e1x = tp[3], e1y = tp[4], e1z = tp[5];
    float e2x = tp[6], e2y = tp[7], e2z = tp[8];
    // pvec = cross(D, e2)
    float px = r.d[1] * e2z - e2y * r.d[2];
    float py = r.d[2] * e2x - e2z * r.d[0];
    float pz = r.d[0] * e2y - e2x * r.d[1];
    float det = (e1x * px + e1y * py) + e1z * pz;
    if (det <= kDetEps) return false;      // det < 0.000001 (double), NaN passes
    float inv = 1.0f / det;
    float sx = r.o[0] - v0x, sy = r.o[1] - v0y, sz = r.o[2] - v0z;
    float u = ((sx * px + sy * py) + sz * pz) * inv;
    if (u < 0.0f || u > 1.0f) return false;
    // qvec = cross(tvec, e1)
    float qx = sy * e1z - e1y * sz;
    float qy = sz * e1x - e1z * sx;
    float qz = sx * e1y - e1x * sy;
    float v = ((r.d[0] * qx + r.d[1] * qy) + r.d[2] * qz) * inv;
    if (v < 0.0f || u + v > 1.0f) return false;
    float t = ((e2x * qx + e2y * qy) + e2z * qz) * inv;
    return t > 0.0f && t < FLT_MAX;
}

// per-ray work counters (parity evidence + algorithmic bytes)
struct Cnt {
    uint32_t nodes, leaves, tris;
};

template <bool ANYHIT, bool STATS>
__device__ __forceinline__ bool leaf_test(const float *__restrict__ tris, uint32_t begin, uint32_t count,
                                          const Ray &r, Cnt &cnt) {
    bool hit = false;
    if (STATS) ++cnt.leaves;
    for (uint32_t i = 0; i < count; ++i) {
        if (STATS) ++cnt.tris;
        if (tri_hit(tris + 9ull * (begin + i), r)) {
            hit = true;
            if (ANYHIT) break;
        }
    }
    return hit;
}

template <bool ANYHIT, bool STATS>
__device__ bool trace(const RenderArgs &a, const Ray &r, const float slo[3], const float shi[3],
                      uint32_t U, uint32_t N, Cnt &cnt) {
    // scene AABB slab test, CUDAKernels.cu:237-262 (tMin may be negative)
    float tMin = ((r.sgn[0] ? shi[0] : slo[0]) - r.o[0]) * r.inv[0];
    float tMax = ((r.sgn[0] ? slo[0] : shi[0]) - r.o[0]) * r.inv[0];
    float tymin = ((r.sgn[1] ? shi[1] : slo[1]) - r.o[1]) * r.inv[1];
    float tymax = ((r.sgn[1] ? slo[1] : shi[1]) - r.o[1]) * r.inv[1];
    if ((tMin > tymax) || (tymin > tMax)) return false;
    if (tymin > tMin) tMin = tymin;
    if (tymax < tMax) tMax = tymax;
    float tzmin = ((r.sgn[2] ? shi[2] : slo[2]) - r.o[2]) * r.inv[2];
    float tzmax = ((r.sgn[2] ? slo[2] : shi[2]) - r.o[2]) * r.inv[2];
    if ((tMin > tzmax) || (tzmin > tMax)) return false;
    if (tzmin > tMin) tMin = tzmin;
    if (tzmax < tMax) tMax = tzmax;
    if (U == 0) return false;
    if (U == 1) return leaf_test<ANYHIT, STATS>(a.tris, 0, N, r, cnt);   // reference: UB

    uint32_t st_node[kStackDepth];
    float st_min[kStackDepth], st_max[kStackDepth];
    int sp = 0;
    uint32_t cur = 0;
    bool hit = false;
    for (;;) {
        if (STATS) ++cnt.nodes;
        const uint4 nd = a.nodes[cur];
        const uint32_t ax = (nd.z >> 27) & 3u;
        const float org = pick3(r.o, ax), inv = pick3(r.inv, ax);
        const uint32_t nr = pick3u(r.sgn, ax);
        const float t0 = (__uint_as_float(nd.x) - org) * inv;
        const float t1 = (__uint_as_float(nd.y) - org) * inv;
        const float tn = nr ? t1 : t0, tf = nr ? t0 : t1;
        const bool A = tMin < tn, B = tMax < tf;
        const uint32_t split = nd.z & kIdxMask, mid = nd.w & kIdxMask;
        const uint32_t leafL = (nd.z >> 29) & 1u, leafR = (nd.z >> 30) & 1u;
        const uint32_t leafN = nr ? leafR : leafL, leafF = nr ? leafL : leafR;
        const uint32_t idxN = split + nr, idxF = split + 1u - nr;
        // leaf ranges of the near / far child
        auto leaf_range = [&](uint32_t right, uint32_t &beg, uint32_t &cnt) {
            uint32_t code = right ? (nd.w >> 29) & 3u : (nd.w >> 27) & 3u;
            cnt = code ? code : a.dup_cnt[split + right];
            beg = right ? mid : mid - cnt;
        };
        bool pop = false;
        if (!A && B) {
            pop = true;
        } else if (A && B) {
            if (leafN) {
                uint32_t b, c; leaf_range(nr, b, c);
                hit |= leaf_test<ANYHIT, STATS>(a.tris, b, c, r, cnt);
                pop = true;
            } else { cur = idxN; tMax = tn; }
        } else if (!A && !B) {
            if (leafF) {
                uint32_t b, c; leaf_range(1u - nr, b, c);
                hit |= leaf_test<ANYHIT, STATS>(a.tris, b, c, r, cnt);
                pop = true;
            } else { cur = idxF; tMin = tf; }
        } else {
            if (leafN && leafF) {
                uint32_t b, c; leaf_range(nr, b, c);
                hit |= leaf_test<ANYHIT, STATS>(a.tris, b, c, r, cnt);
                if (!(ANYHIT && hit)) {
                    leaf_range(1u - nr, b, c);
                    hit |= leaf_test<ANYHIT, STATS>(a.tris, b, c, r, cnt);
                }
                pop = true;
            } else if (!leafN && leafF) {
                uint32_t b, c; leaf_range(1u - nr, b, c);
                hit |= leaf_test<ANYHIT, STATS>(a.tris, b, c, r, cnt);
                cur = idxN; tMax = tn;
            } else if (leafN && !leafF) {
                uint32_t b, c; leaf_range(nr, b, c);
                hit |= leaf_test<ANYHIT, STATS>(a.tris, b, c, r, cnt);
                cur = idxF; tMin = tf;
            } else {
                st_node[sp] = idxF; st_min[sp] = tf; st_max[sp] = tMax;
                ++sp;
                cur = idxN; tMax = tn;
            }
        }
        if (ANYHIT && hit) break;
        if (pop) {
            if (sp == 0) break;
            --sp;
            cur = st_node[sp]; tMin = st_min[sp]; tMax = st_max[sp];
        }
    }
    return hit;
}

__device__ __forceinline__ float xorwow_uniform(uint32_t v[5], uint32_t &d) {
    uint32_t t = v[0] ^ (v[0] >> 2);
    v[0] = v[1]; v[1] = v[2]; v[2] = v[3]; v[3] = v[4];
    v[4] = (v[4] ^ (v[4] << 4)) ^ (t ^ (t << 1));
    d += kWeyl;
    uint32_t x = v[4] + d;
    return (float)x * 2.3283064e-10f + (2.3283064e-10f / 2.0f);   // _curand_uniform
}

__device__ __forceinline__ uint32_t rgb_to_int(float r, float g, float b) {
    r = fmaxf(0.0f, fminf(255.0f, r));                             // clamp, :74-76
    g = fmaxf(0.0f, fminf(255.0f, g));
    b = fmaxf(0.0f, fminf(255.0f, b));
    return ((uint32_t)(int)b << 16) | ((uint32_t)(int)g << 8) | (uint32_t)(int)r;
}

// One wave = one 8x8 pixel tile (coherent primary rays share node fetches);
// one lane = one pixel, spp jittered samples in sequence (cudaRender order).
template <bool ANYHIT, bool STATS>
__global__ void __launch_bounds__(kThreads) k_render(const RenderArgs a) {
    const uint32_t tiles_x = (a.w + 7) >> 3;
    const uint32_t wv = blockIdx.x * (kThreads / 64) + (threadIdx.x >> 6);
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t x = (wv % tiles_x) * 8 + (lane & 7);
    const uint32_t lr = (wv / tiles_x) * 8 + (lane >> 3);
    if (x >= a.w || lr >= a.nrows) return;
    const uint32_t y = global_row(lr, a.row0, a.band_h, a.band_step);
    const uint64_t P = (uint64_t)a.nrows * a.w;
    const uint64_t lp = (uint64_t)lr * a.w + x;

    const float slo[3] = {a.hdr->scene_lo[0], a.hdr->scene_lo[1], a.hdr->scene_lo[2]};
    const float shi[3] = {a.hdr->scene_hi[0], a.hdr->scene_hi[1], a.hdr->scene_hi[2]};
    const uint32_t U = a.hdr->n_unique, N = a.hdr->n_tris;

    uint32_t v[5];
#pragma unroll
    for (int i = 0; i < 5; ++i) v[i] = a.rng[(uint64_t)i * P + lp];
    uint32_t d = a.d_base;

    float cr = 0.0f, cg = 0.0f, cb = 0.0f;
    for (uint32_t s = 0; s < a.spp; ++s) {
        const float ru = xorwow_uniform(v, d);
        const float rv = xorwow_uniform(v, d);
        const float u = ((float)x + ru) / (float)a.w;
        const float vv = ((float)y + rv) / (float)a.h;
        Ray r;
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            r.o[c] = a.cam[c];
            float hu = u * a.cam[6 + c];
            float vq = vv * a.cam[9 + c];
            r.d[c] = ((a.cam[3 + c] + hu) + vq) - a.cam[c];
            r.inv[c] = 1.0f / r.d[c];
            r.sgn[c] = r.inv[c] < 0.0f;
        }
        Cnt cnt = {0, 0, 0};
        const bool hit = trace<ANYHIT, STATS>(a, r, slo, shi, U, N, cnt);
        if (STATS) {
            uint64_t rid = lp * a.spp + s;
            a.ray_stats[3 * rid] = cnt.nodes;
            a.ray_stats[3 * rid + 1] = cnt.leaves;
            a.ray_stats[3 * rid + 2] = cnt.tris;
        }
        cr += hit ? 255.0f : 20.0f;
        cg += hit ? 255.0f : 20.0f;
        cb += hit ? 0.0f : 40.0f;
    }
#pragma unroll
    for (int i = 0; i < 5; ++i) a.rng[(uint64_t)i * P + lp] = v[i];
    const float fs = (float)a.spp;
    a.out[lp] = rgb_to_int(cr / fs, cg / fs, cb / fs);
}

std::mutex g_tab_mu;
uint32_t *g_tab_dev[64] = {nullptr};

}  // namespace

int upload_rng_tables(int device) {
    if (device < 0 || device >= 64) return (int)hipErrorInvalidDevice;
    std::lock_guard<std::mutex> lk(g_tab_mu);
    if (g_tab_dev[device]) return 0;
    const size_t bytes = (32 + 64) * 800 * sizeof(uint32_t);
    uint32_t *p = nullptr;
    hipError_t e = hipMalloc((void **)&p, bytes);
    if (e != hipSuccess) return (int)e;
    e = hipMemcpy(p, xorwow_tables_host(), bytes, hipMemcpyHostToDevice);
    if (e != hipSuccess) { (void)hipFree(p); return (int)e; }
    g_tab_dev[device] = p;
    return 0;
}

const uint32_t *rng_tables_device(int device) {
    std::lock_guard<std::mutex> lk(g_tab_mu);
    return (device >= 0 && device < 64) ? g_tab_dev[device] : nullptr;
}

int launch_rng_init(uint32_t *rng, uint32_t w, uint32_t row0, uint32_t nrows, uint32_t band_h,
                    uint32_t band_step, uint64_t seed, uint64_t skip, int device, void *stream) {
    const uint32_t *tab = rng_tables_device(device);
    if (!tab) return (int)hipErrorNotInitialized;
    uint32_t v[5], d;
    xorwow_seed(seed, v, &d);
    const uint64_t P = (uint64_t)nrows * w;
    if (P == 0) return 0;
    const uint32_t blocks = (uint32_t)((P + kThreads - 1) / kThreads);
    hipLaunchKernelGGL(k_rng_init, dim3(blocks), dim3(kThreads), 0, (hipStream_t)stream, rng, w, row0,
                       nrows, band_h, band_step, v[0], v[1], v[2], v[3], v[4],
                       (unsigned long long)skip, tab);
    return (int)hipGetLastError();
}

int launch_render(const RenderArgs &a, uint32_t traverse, void *stream) {
    const uint32_t tiles = ((a.w + 7) >> 3) * ((a.nrows + 7) >> 3);
    if (tiles == 0) return 0;
    const uint32_t blocks = (tiles + 3) / 4;
    hipStream_t st = (hipStream_t)stream;
    const bool stats = a.ray_stats != nullptr;
    if (traverse == 0) {
        if (stats) hipLaunchKernelGGL((k_render<true, true>), dim3(blocks), dim3(kThreads), 0, st, a);
        else hipLaunchKernelGGL((k_render<true, false>), dim3(blocks), dim3(kThreads), 0, st, a);
    } else {
        if (stats) hipLaunchKernelGGL((k_render<false, true>), dim3(blocks), dim3(kThreads), 0, st, a);
        else hipLaunchKernelGGL((k_render<false, false>), dim3(blocks), dim3(kThreads), 0, st, a);
    }
    return (int)hipGetLastError();
}

}  // namespace bih
