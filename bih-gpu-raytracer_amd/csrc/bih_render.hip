// bih_render.hip -- primary-ray render kernels for gfx950 (MI355X).
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
//
// Kernels
//   k_render_bins        any-hit default: the frustum-bin list walk,
//                        k_render_fallback finishes undecided packets.
//   k_render_packet_asm  the exact packet walk (TRAVERSE_REFERENCE, counters,
//                        renders without bins), hand-scheduled gfx950 asm.
//   k_render_packet2     the same packet walk in HIP: the asm walk's cross-check
//                        (BIH_RENDER_KERNEL=packet2, test_kernel_variants_agree).
//   k_render_packet      the packet walk over the canonical packed nodes: scenes
//                        past the camera-relative records' 2^26 triangles.
//   k_render_pixel       spp not a power of two: one lane per pixel, samples in
//                        sequence (cudaRender's own loop order).
// k_render_pixel's traversal core (Walker) makes the reference's 4-way
// decision per node in TraverseTree's order, so its per-ray counters equal
// the oracle's any-hit prefix.  Its stack keeps the first kLdsStack entries
// per lane in LDS ([entry][lane], conflict-free) and spills deeper ones to a
// per-lane HBM area.
#include <hip/hip_runtime.h>
#include <float.h>
#include <stdlib.h>
#include <string.h>

#include <mutex>
#include <stdio.h>
#include <vector>

#include "bih_internal.h"
#include "bih_bound.h"
#include "bih_packet_asm.h"
#include "bih_device.h"

namespace bih {
namespace {

using dev::camera_dir;
using dev::global_row;
using dev::kDetEps;
using dev::kWeyl;
using dev::rgb_to_int;
using dev::xorwow_uniform;

constexpr int kThreads = 256;
constexpr uint32_t kDone = 0xFFFFFFFFu;

#ifndef BIH_MT_EARLY_OUT
#define BIH_MT_EARLY_OUT 1      // return at the back-face test (else fully predicated MT)
#endif
#ifndef BIH_SPILL_NT
#define BIH_SPILL_NT 0          // non-temporal loads/stores for the HBM stack slots
#endif

// ---------------------------------------------------------------------------
// RNG: v = M^skip * J^pixel * seed_state (J = M^(2^67)), cuRAND XORWOW.
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

// Per-pixel curand_init(seed, pixel, 0) + skip (InitRandGPU,
// CUDAKernels.cu:450-459).  The host applied M^skip to the seed state
// (powers of M commute).  A wave seeds a segment of 64 x kRngRun consecutive
// pixels of one row: lane l's first pixel jumps to its subsequence with at
// most 4 byte-table applies (J^(b << 8k)), its next ones (64 pixels further
// each) are one J^64 step through the nibble table in LDS, and the 64 lanes
// store 64 consecutive words per plane (coalesced: a lane-per-run layout
// spread each store over 64 lines and was store-bound at 0.18 ms / 1080p).
#ifndef BIH_RNG_RUN
#define BIH_RNG_RUN 32
#endif
constexpr uint32_t kRngRun = BIH_RNG_RUN;
__device__ __forceinline__ void jump_lds(const uint32_t *__restrict__ nib, uint32_t x[5]) {
    uint32_t r0 = 0, r1 = 0, r2 = 0, r3 = 0, r4 = 0;
#pragma unroll
    for (int g = 0; g < 40; ++g) {
        const uint32_t n = (x[g >> 3] >> ((g & 7) * 4)) & 15u;
        const uint32_t *c = nib + (g * 16 + n) * 5;
        r0 ^= c[0]; r1 ^= c[1]; r2 ^= c[2]; r3 ^= c[3]; r4 ^= c[4];
    }
    x[0] = r0; x[1] = r1; x[2] = r2; x[3] = r3; x[4] = r4;
}

__global__ void __launch_bounds__(kThreads) k_rng_init(uint32_t *__restrict__ rng, uint32_t w,
                                                       uint32_t row0, uint32_t nrows, uint32_t band_h,
                                                       uint32_t band_step, uint32_t s0, uint32_t s1,
                                                       uint32_t s2, uint32_t s3, uint32_t s4,
                                                       const uint32_t *__restrict__ tables) {
    __shared__ uint32_t s_nib[40 * 16 * 5];
    const uint32_t *nib64 = tables + 4 * 256 * 800 + 40 * 16 * 5;   // J^64
    for (uint32_t k = threadIdx.x; k < 40 * 16 * 5; k += kThreads) s_nib[k] = nib64[k];
    __syncthreads();
    constexpr uint32_t kSeg = 64 * kRngRun;
    const uint32_t segs = (w + kSeg - 1) / kSeg;
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t wave = ((uint64_t)blockIdx.x * kThreads + threadIdx.x) >> 6;
    if (wave >= (uint64_t)nrows * segs) return;
    const uint32_t lr = (uint32_t)(wave / segs), x0 = (uint32_t)(wave % segs) * kSeg + lane;
    if (x0 >= w) return;
    const uint64_t pix = (uint64_t)global_row(lr, row0, band_h, band_step) * w + x0;
    uint32_t v[5] = {s0, s1, s2, s3, s4};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const uint32_t b = (uint32_t)(pix >> (8 * k)) & 255u;
        if (b) gf2_apply(tables + ((uint32_t)k * 256 + b) * 800, v);
    }
    const uint64_t P = (uint64_t)nrows * w, lp0 = (uint64_t)lr * w + x0;
    for (uint32_t i = 0; i < kRngRun && x0 + 64 * i < w; ++i) {
        if (i) jump_lds(s_nib, v);
#pragma unroll
        for (int j = 0; j < 5; ++j) rng[(uint64_t)j * P + lp0 + 64 * i] = v[j];
    }
}

// dst = every pixel's XORWOW xorshift state `steps` draws after src's (dst
// may be src).  2*spp*nframes steps: the state the launch after a render of
// nframes frames starts from (cudaRender's write-back, CUDAKernels.cu:419);
// more: a gap in the frame sequence.  The Weyl counter d is derived from the
// frame index, not stored.  Up to two of the powers 2^7 .. 2^13 of `steps`
// jump through their nibble tables in LDS (40 lookups each, against 128 ..
// 8192 steps; the frame-jump tables of k_rng_sync), the rest is stepped.
// The tables are re-laid in LDS as words 0-3 (one ds_read_b128) + word 4 of
// each entry; each thread loads its PPT pixels' states before it jumps any
// (their loads in flight together), PPT pixels a grid's width apart.
__device__ __forceinline__ void jump_lds4(const uint4 *__restrict__ a, const uint32_t *__restrict__ b, uint32_t x[5]) {
    uint32_t r0 = 0, r1 = 0, r2 = 0, r3 = 0, r4 = 0;
#pragma unroll
    for (int g = 0; g < 40; ++g) {
        const uint32_t e = g * 16 + ((x[g >> 3] >> ((g & 7) * 4)) & 15u);
        const uint4 c = a[e];
        r0 ^= c.x; r1 ^= c.y; r2 ^= c.z; r3 ^= c.w; r4 ^= b[e];
    }
    x[0] = r0; x[1] = r1; x[2] = r2; x[3] = r3; x[4] = r4;
}
template <int PPT>
__global__ void __launch_bounds__(kThreads) k_rng_advance(const uint32_t *src, uint32_t *dst, uint64_t P,
                                                          uint32_t steps, const uint32_t *__restrict__ jumps,
                                                          uint32_t k0, uint32_t k1) {
    __shared__ uint4 s_a[2][40 * 16];
    __shared__ uint32_t s_b[2][40 * 16];
    const uint32_t nj = (k0 < 7u) + (k1 < 7u);
    for (uint32_t t = 0; t < nj; ++t) {
        const uint32_t *tab = jumps + (t ? k1 : k0) * kRngNibWords;
        for (uint32_t e = threadIdx.x; e < 40 * 16; e += kThreads) {
            s_a[t][e] = make_uint4(tab[5 * e], tab[5 * e + 1], tab[5 * e + 2], tab[5 * e + 3]);
            s_b[t][e] = tab[5 * e + 4];
        }
    }
    if (nj) __syncthreads();
    const uint64_t stride = (uint64_t)gridDim.x * kThreads;
    for (uint64_t lp0 = (uint64_t)blockIdx.x * kThreads + threadIdx.x; lp0 < P; lp0 += stride * PPT) {
        uint32_t v[PPT][5];
#pragma unroll
        for (int j = 0; j < PPT; ++j) {
            const uint64_t lp = lp0 + j * stride;
            if (lp < P) {
#pragma unroll
                for (int i = 0; i < 5; ++i) v[j][i] = src[(uint64_t)i * P + lp];
            }
        }
#pragma unroll
        for (int j = 0; j < PPT; ++j) {
            for (uint32_t t = 0; t < nj; ++t) jump_lds4(s_a[t], s_b[t], v[j]);
#pragma unroll 8
            for (uint32_t k = 0; k < steps; ++k) {
                const uint32_t t = v[j][0] ^ (v[j][0] >> 2);
                v[j][0] = v[j][1]; v[j][1] = v[j][2]; v[j][2] = v[j][3]; v[j][3] = v[j][4];
                v[j][4] = (v[j][4] ^ (v[j][4] << 4)) ^ (t ^ (t << 1));
            }
        }
#pragma unroll
        for (int j = 0; j < PPT; ++j) {
            const uint64_t lp = lp0 + j * stride;
            if (lp < P) {
#pragma unroll
                for (int i = 0; i < 5; ++i) dst[(uint64_t)i * P + lp] = v[j][i];
            }
        }
    }
}

// Stamped state (RenderArgs::stamps): the frame and buffer a tile's state is
// read from in launch `seq` -- the stamp's prev when this launch already
// rewrote it, else its cur.
struct StampBase {
    uint32_t F, b;
};
__device__ __forceinline__ StampBase stamp_base(unsigned long long st, uint32_t seq) {
    const bool mine = (uint32_t)(st >> 54) == seq;
    const uint32_t w = mine ? (uint32_t)(st >> 27) & 0x7FFFFFFu : (uint32_t)st & 0x7FFFFFFu;
    return {w & kStampFrameMax, w >> kStampFrameBits};
}
__device__ __forceinline__ unsigned long long stamp_pack(uint32_t F, uint32_t b, StampBase prev, uint32_t seq) {
    return (unsigned long long)(F | (b << kStampFrameBits)) |
           ((unsigned long long)(prev.F | (prev.b << kStampFrameBits)) << 27) | ((unsigned long long)seq << 54);
}
__device__ __forceinline__ void xorwow_steps(uint32_t v[5], uint32_t n) {
#pragma unroll 4
    for (uint32_t k = 0; k < n; ++k) {
        const uint32_t t = v[0] ^ (v[0] >> 2);
        v[0] = v[1]; v[1] = v[2]; v[2] = v[3]; v[3] = v[4];
        v[4] = (v[4] ^ (v[4] << 4)) ^ (t ^ (t << 1));
    }
}

// Stamped state (RenderArgs::stamps): every tile at frame F in buffer 0.
__global__ void __launch_bounds__(kThreads) k_stamp_init(unsigned long long *__restrict__ stamps, uint32_t ntiles,
                                                         uint32_t frame) {
    const uint32_t t = blockIdx.x * kThreads + threadIdx.x;
    if (t < ntiles)
        stamps[t] = (unsigned long long)frame | ((unsigned long long)frame << 27);   // cur = prev = (F, 0), seq 0
}
// Every pixel's stamped state brought to frame `target` (2*spp draws per
// frame): into its tile's other buffer with the tile's new stamp (launch
// `seq`; the tile's first pixel writes it), or -- full != null -- into `full`
// for every pixel, leaving the stamps as they are (back to the ring).  Whole
// kStampJumpFrames runs jump through the nibble table of their matrix (40
// lookups against 64 * 2 * spp steps: background tiles lag by exactly that
// much between syncs), the rest is stepped.  Grid-stride, so that few blocks
// load the table into LDS.
__global__ void __launch_bounds__(kThreads) k_rng_sync(unsigned long long *__restrict__ stamps, uint32_t *buf0,
                                                       uint32_t *buf1, uint32_t *__restrict__ full, uint32_t w,
                                                       uint32_t nrows, uint32_t log2spp, uint32_t target,
                                                       uint32_t seq, const uint32_t *__restrict__ jump) {
    __shared__ uint32_t s_nib[kRngNibWords];
    for (uint32_t k = threadIdx.x; k < kRngNibWords; k += kThreads) s_nib[k] = jump[k];
    __syncthreads();
    const uint64_t P = (uint64_t)nrows * w;
    const uint32_t lpx = 6 - log2spp, tw = 1u << ((lpx + 1) / 2), th = 1u << (lpx / 2);
    const uint32_t tiles_x = (w + tw - 1) / tw;
    for (uint64_t lp = (uint64_t)blockIdx.x * kThreads + threadIdx.x; lp < P; lp += (uint64_t)gridDim.x * kThreads) {
        const uint32_t lr = (uint32_t)(lp / w), x = (uint32_t)(lp - (uint64_t)lr * w);
        const uint32_t t = (lr / th) * tiles_x + x / tw;
        const StampBase sb = stamp_base(stamps[t], seq);
        if (!full && sb.F >= target) continue;   // already at the frame
        const uint32_t *src = sb.b ? buf1 : buf0;
        uint32_t v[5];
#pragma unroll
        for (int i = 0; i < 5; ++i) v[i] = src[(uint64_t)i * P + lp];
        const uint32_t lag = target - sb.F;
        for (uint32_t q = 0; q < lag / kStampJumpFrames; ++q) jump_lds(s_nib, v);
        xorwow_steps(v, (lag % kStampJumpFrames) << (log2spp + 1));
        uint32_t *dst = full ? full : (sb.b ? buf0 : buf1);
#pragma unroll
        for (int i = 0; i < 5; ++i) dst[(uint64_t)i * P + lp] = v[i];
        if (!full && lr % th == 0 && x % tw == 0) stamps[t] = stamp_pack(target, sb.b ^ 1u, sb, seq);
    }
}

// Pixel of k hits out of spp samples.  Color() returns (255,255,0) or
// (20,20,40); the f32 sum of small integers is exact in any order, so the
// reference's col /= spp; rgbToInt(col) depends only on k (:412-422).
__device__ __forceinline__ uint32_t pixel_from_hits(uint32_t k, uint32_t spp) {
    const float fs = (float)spp;
    const float cr = (float)(255u * k + 20u * (spp - k));
    const float cb = (float)(40u * (spp - k));
    return rgb_to_int(cr / fs, cr / fs, cb / fs);
}

// ---------------------------------------------------------------------------
// Triangle test: RayTriangleIntersection + FindNearestTriangle's record test.
// With rec.t starting at FLT_MAX (Color, :380-382) "some triangle was
// recorded" == "some tested triangle has MT true and 0 < t < FLT_MAX".
// tp = {v0, e1 = v1-v0, e2 = v2-v0} (36 B, Morton order).
// ---------------------------------------------------------------------------
__device__ __forceinline__ bool tri_hit(const float *__restrict__ tp, float ox, float oy, float oz,
                                        float dx, float dy, float dz) {
    float v0x = tp[0], v0y = tp[1], v0z = tp[2];
    float e1x = tp[3], e1y = tp[4], e1z = tp[5];
    float e2x = tp[6], e2y = tp[7], e2z = tp[8];
    // one round trip for the whole record (hipcc would otherwise sink the v0
    // load behind the det test)
    asm volatile("" ::"v"(v0x), "v"(v0y), "v"(v0z), "v"(e1x), "v"(e1y), "v"(e1z), "v"(e2x),
                 "v"(e2y), "v"(e2z));
    float px = dy * e2z - e2y * dz;                  // pvec = cross(D, e2)
    float py = dz * e2x - e2z * dx;
    float pz = dx * e2y - e2x * dy;
    float det = (e1x * px + e1y * py) + e1z * pz;
#if BIH_MT_EARLY_OUT
    // Coherent rays see a triangle from the same side: the back-face test is
    // usually uniform across the wave, and then skips the rest entirely.
    if (det <= kDetEps) return false;                // det < 0.000001 (double); NaN passes
#endif
    float inv = 1.0f / det;
    float sx = ox - v0x, sy = oy - v0y, sz = oz - v0z;
    float u = ((sx * px + sy * py) + sz * pz) * inv;
#if BIH_MT_EARLY_OUT
    if (u < 0.0f || u > 1.0f) return false;
#endif
    float qx = sy * e1z - e1y * sz;                  // qvec = cross(tvec, e1)
    float qy = sz * e1x - e1z * sx;
    float qz = sx * e1y - e1x * sy;
    float v = ((dx * qx + dy * qy) + dz * qz) * inv;
#if BIH_MT_EARLY_OUT
    if (v < 0.0f || u + v > 1.0f) return false;
#endif
    float t = ((e2x * qx + e2y * qy) + e2z * qz) * inv;
    // det < 0.000001 (double compare) rejects; NaN det passes it
    const bool ok_det = !(det <= kDetEps);
    const bool ok_u = !(u < 0.0f || u > 1.0f);
    const bool ok_v = !(v < 0.0f || u + v > 1.0f);
    const bool ok_t = t > 0.0f && t < FLT_MAX;
    return ok_det & ok_u & ok_v & ok_t;
}

// v[ax] for ax in {0,1,2} with integer masks: written as a ?: chain, hipcc
// turns the three struct fields into an indexed scratch load.
__device__ __forceinline__ float sel3(uint32_t ax, float a, float b, float c) {
    const uint32_t m0 = 0u - (uint32_t)(ax == 0), m1 = 0u - (uint32_t)(ax == 1);
    const uint32_t m2 = ~(m0 | m1);
    return __uint_as_float((__float_as_uint(a) & m0) | (__float_as_uint(b) & m1) |
                           (__float_as_uint(c) & m2));
}

// per-ray work counters (parity evidence + algorithmic bytes)
struct Cnt {
    uint32_t nodes, leaves, tris;
};

// Uniform per-launch values.
struct SceneU {
    float ox, oy, oz;
    float slo0, slo1, slo2, shi0, shi1, shi2;
    uint32_t U, N;
    const uint4 *nodes;
    const float *tris;
    const uint32_t *dup_cnt;
};

__device__ __forceinline__ SceneU load_scene(const RenderArgs &a) {
    SceneU s;
    s.ox = a.cam[0]; s.oy = a.cam[1]; s.oz = a.cam[2];
    s.slo0 = a.hdr->scene_lo[0]; s.slo1 = a.hdr->scene_lo[1]; s.slo2 = a.hdr->scene_lo[2];
    s.shi0 = a.hdr->scene_hi[0]; s.shi1 = a.hdr->scene_hi[1]; s.shi2 = a.hdr->scene_hi[2];
    s.U = a.hdr->n_unique; s.N = a.hdr->n_tris;
    s.nodes = a.nodes; s.tris = a.tris; s.dup_cnt = a.dup_cnt;
    return s;
}

// Per-lane stack: slots [0, kLdsStack) in LDS, deeper slots in HBM.
struct Stack {
    uint32_t *node;      // LDS, [kLdsStack][kThreads]
    float *tmin, *tmax;
    uint32_t tid;
    uint32_t *spill;     // HBM, [(kStackDepth-kLdsStack)*3][gthreads]
    uint64_t gthreads, gtid;

    // The HBM slots sit behind a wave-uniform __any() test: written as one
    // if/else, hipcc merges both sides into FLAT loads (LDS through the
    // vector-memory path, waiting on vmcnt) on every pop.
    __device__ __forceinline__ void push(uint32_t sp, uint32_t n, float lo, float hi) const {
        const bool in_lds = sp < (uint32_t)kLdsStack;
        if (in_lds) {
            node[sp * kThreads + tid] = n;
            tmin[sp * kThreads + tid] = lo;
            tmax[sp * kThreads + tid] = hi;
        }
        if (__builtin_expect(__any(!in_lds), 0)) {
            if (!in_lds) {
                uint32_t *q = spill + (uint64_t)(sp - kLdsStack) * 3 * gthreads + gtid;
#if BIH_SPILL_NT
                __builtin_nontemporal_store(n, q);
                __builtin_nontemporal_store(__float_as_uint(lo), q + gthreads);
                __builtin_nontemporal_store(__float_as_uint(hi), q + 2 * gthreads);
#else
                q[0] = n;
                q[gthreads] = __float_as_uint(lo);
                q[2 * gthreads] = __float_as_uint(hi);
#endif
            }
        }
    }
    __device__ __forceinline__ void pop(uint32_t sp, uint32_t &n, float &lo, float &hi) const {
        const bool in_lds = sp < (uint32_t)kLdsStack;
        if (in_lds) {
            n = node[sp * kThreads + tid];
            lo = tmin[sp * kThreads + tid];
            hi = tmax[sp * kThreads + tid];
        }
        if (__builtin_expect(__any(!in_lds), 0)) {
            if (!in_lds) {
                const uint32_t *q = spill + (uint64_t)(sp - kLdsStack) * 3 * gthreads + gtid;
#if BIH_SPILL_NT
                n = __builtin_nontemporal_load(q);
                lo = __uint_as_float(__builtin_nontemporal_load(q + gthreads));
                hi = __uint_as_float(__builtin_nontemporal_load(q + 2 * gthreads));
#else
                n = q[0];
                lo = __uint_as_float(q[gthreads]);
                hi = __uint_as_float(q[2 * gthreads]);
#endif
            }
        }
    }
};

// One ray's walk (TraverseTree, CUDAKernels.cu:227-368).
template <bool ANYHIT, bool STATS>
struct Walker {
    float dx, dy, dz, ix, iy, iz;
    uint32_t sg;                       // sign bits of invDir (Ray::sign)
    float tMin, tMax;
    uint32_t cur, sp;
    uint32_t b0, e0, b1, e1;           // leaf queue: [b0,e0) then [b1,e1)
    bool alive, hit;
    Cnt cnt;

    // Ray::Ray + the scene-AABB slab test (:237-262); tMin may be negative.
    __device__ __forceinline__ void start(const SceneU &s, bool valid, float dx_, float dy_, float dz_) {
        dx = dx_; dy = dy_; dz = dz_;
        ix = 1.0f / dx; iy = 1.0f / dy; iz = 1.0f / dz;
        sg = (ix < 0.0f ? 1u : 0u) | (iy < 0.0f ? 2u : 0u) | (iz < 0.0f ? 4u : 0u);
        tMin = (((sg & 1) ? s.shi0 : s.slo0) - s.ox) * ix;
        tMax = (((sg & 1) ? s.slo0 : s.shi0) - s.ox) * ix;
        const float tymin = (((sg & 2) ? s.shi1 : s.slo1) - s.oy) * iy;
        const float tymax = (((sg & 2) ? s.slo1 : s.shi1) - s.oy) * iy;
        bool in = valid && !((tMin > tymax) || (tymin > tMax));
        if (tymin > tMin) tMin = tymin;
        if (tymax < tMax) tMax = tymax;
        const float tzmin = (((sg & 4) ? s.shi2 : s.slo2) - s.oz) * iz;
        const float tzmax = (((sg & 4) ? s.slo2 : s.shi2) - s.oz) * iz;
        in = in && !((tMin > tzmax) || (tzmin > tMax));
        if (tzmin > tMin) tMin = tzmin;
        if (tzmax < tMax) tMax = tzmax;
        cnt.nodes = cnt.leaves = cnt.tris = 0;
        hit = false;
        cur = 0; sp = 0;
        b0 = e0 = b1 = e1 = 0;
        alive = in && s.U > 0;
        if (alive && s.U == 1) {           // single leaf; reference: UB
            cur = kDone;
            e0 = s.N;
            if (STATS) cnt.leaves = 1;
        }
    }

    // One unit of work: a queued triangle, else one node.
    __device__ __forceinline__ void step(const SceneU &s, const Stack &st) {
        if (b0 < e0) {
            if (STATS) ++cnt.tris;
            const bool h = tri_hit(s.tris + 9ull * b0, s.ox, s.oy, s.oz, dx, dy, dz);
            hit |= h;
            ++b0;
            if (ANYHIT && h) {
                if (STATS && e1 > b1) --cnt.leaves;   // queued far leaf never visited
                alive = false;
                return;
            }
            if (b0 == e0) { b0 = b1; e0 = e1; b1 = e1 = 0; }
            if (b0 >= e0 && cur == kDone) alive = false;
            return;
        }
        if (STATS) ++cnt.nodes;
        const uint4 nd = s.nodes[cur];
        const uint32_t ax = (nd.z >> 27) & 3u;
        const float org = sel3(ax, s.ox, s.oy, s.oz);
        const float inv = sel3(ax, ix, iy, iz);
        const uint32_t nr = (sg >> ax) & 1u;
        const float t0 = (__uint_as_float(nd.x) - org) * inv;
        const float t1 = (__uint_as_float(nd.y) - org) * inv;
        const float tn = nr ? t1 : t0, tf = nr ? t0 : t1;
        const bool A = tMin < tn, B = tMax < tf;
        const uint32_t split = nd.z & kIdxMask, mid = nd.w & kIdxMask;
        const bool leafL = (nd.z >> 29) & 1u, leafR = (nd.z >> 30) & 1u;
        const bool leafN = nr ? leafR : leafL, leafF = nr ? leafL : leafR;
        // the reference's four cases, flattened
        const bool testN = A && leafN;                       // near leaf searched
        const bool testF = !B && leafF;                      // far leaf searched
        const bool goN = A && !leafN;                        // descend near
        const bool goF = !B && !leafF && (!A || leafN);      // descend far
        const bool push = goN && !B && !leafF;               // both internal: stack far
        // leaf ranges, computed unconditionally: left [mid-cL, mid), right [mid, mid+cR)
        uint32_t cL = (nd.w >> 27) & 3u, cR = (nd.w >> 29) & 3u;
        const bool escL = (testN | testF) ? (leafL && cL == 0) : false;   // count > 3
        const bool escR = (testN | testF) ? (leafR && cR == 0) : false;
        if (__builtin_expect(__any(escL | escR), 0)) {
            if (escL) cL = s.dup_cnt[split];
            if (escR) cR = s.dup_cnt[split + 1];
        }
        const uint32_t nb = nr ? mid : mid - cL, ne = nr ? mid + cR : mid;
        const uint32_t fb = nr ? mid - cL : mid, fe = nr ? mid : mid + cR;
        const bool two = testN && testF;
        b0 = testN ? nb : (testF ? fb : b0);
        e0 = testN ? ne : (testF ? fe : e0);
        b1 = two ? fb : b1;
        e1 = two ? fe : e1;
        if (STATS) cnt.leaves += (testN ? 1u : 0u) + (testF ? 1u : 0u);
        // stack: push the far child, or pop when no child is descended
        const bool pop = !goN && !goF && sp != 0;
        const uint32_t far = split + 1u - nr;
        uint32_t pn = kDone;
        float pmin = tMin, pmax = tMax;
        if (push) st.push(sp, far, tf, tMax);
        if (pop) st.pop(sp - 1u, pn, pmin, pmax);
        sp = sp + (push ? 1u : 0u) - (pop ? 1u : 0u);
        cur = goN ? split + nr : (goF ? far : pn);
        tMax = goN ? tn : pmax;
        tMin = goF ? tf : pmin;
        if (cur == kDone && b0 >= e0) alive = false;
    }
};

// Camera::GetRay(u, v) direction, Camera.cu:18-20 (glm order, no contraction).
template <int L>
struct TileShape {   // TW x TH pixels, TW*TH = 64 >> log2(spp)
    static constexpr uint32_t LP = 6 - L;
    static constexpr uint32_t TW = 1u << ((LP + 1) / 2);
    static constexpr uint32_t TH = 1u << (LP / 2);
};

// Ray id -> (local pixel, sample).  Ids run tile-major: 64 consecutive ids
// are one TW x TH pixel tile, pixel-major within the tile.
template <int LOG2SPP>
__device__ __forceinline__ void ray_coords(uint64_t rid, uint32_t tiles_x, uint32_t &x, uint32_t &lr,
                                           uint32_t &s) {
    constexpr uint32_t TW = TileShape<LOG2SPP>::TW, TH = TileShape<LOG2SPP>::TH;
    const uint32_t tile = (uint32_t)(rid >> 6);
    const uint32_t pix = ((uint32_t)rid & 63u) >> LOG2SPP;
    s = (uint32_t)rid & ((1u << LOG2SPP) - 1u);
    x = (tile % tiles_x) * TW + (pix % TW);
    lr = (tile / tiles_x) * TH + (pix / TW);
}

// RNG for sample s of pixel lp: draws 2s, 2s+1 of this frame (the pixel's
// state advanced 2s+2 steps).  The state the reference's cudaRender leaves
// behind (:419) is produced by k_rng_advance, not here: the render only reads
// its frame's state, so consecutive frames can be in flight together.
template <uint32_t SPP>
__device__ __forceinline__ void ray_jitter(const RenderArgs &a, uint64_t lp, uint32_t s, float &ru,
                                           float &rv, uint32_t fj = 0, uint32_t tile = 0) {
    const uint64_t P = (uint64_t)a.nrows * a.w;
    uint32_t v[5];
    // frame j of a multi-frame launch: its draws start 2*spp*j past rng_in's
    // (stamped state: past the tile's stamp frame)
    uint32_t pre = 2 * SPP * fj;
    const uint32_t *src = a.rng_in;
    if (a.stamps) {
        const StampBase sb = stamp_base(a.stamps[tile], a.st_seq);
        src = sb.b ? a.st_buf1 : a.st_buf0;
        pre = 2 * SPP * (a.st_f0 + fj - sb.F);
    }
#pragma unroll
    for (int i = 0; i < 5; ++i) v[i] = src[(uint64_t)i * P + lp];
    uint32_t d = a.d_base;
    xorwow_steps(v, pre);
    d += 2 * SPP * fj * kWeyl;
    for (uint32_t k = 0; k <= s; ++k) {
        ru = xorwow_uniform(v, d);
        rv = xorwow_uniform(v, d);
    }
}

// ---------------------------------------------------------------------------
// k_render_pixel: any spp; one lane per pixel, spp samples in sequence
// (cudaRender's own loop order).  One wave = one 8x8 pixel tile.
// ---------------------------------------------------------------------------
template <bool ANYHIT, bool STATS>
__global__ void __launch_bounds__(kThreads) k_render_pixel(const RenderArgs a) {
    __shared__ uint32_t s_node[kLdsStack * kThreads];
    __shared__ float s_min[kLdsStack * kThreads];
    __shared__ float s_max[kLdsStack * kThreads];
    const uint32_t tid = threadIdx.x, lane = tid & 63;
    const uint32_t tiles_x = (a.w + 7) >> 3;
    const uint32_t ntiles = tiles_x * ((a.nrows + 7) >> 3);
    const Stack st = {s_node, s_min, s_max, tid, a.spill, (uint64_t)gridDim.x * kThreads,
                      (uint64_t)blockIdx.x * kThreads + tid};
    const SceneU sc = load_scene(a);
    const uint64_t P = (uint64_t)a.nrows * a.w;
    // grid-stride over 8x8 tiles (the grid is capped at the spill area's size)
    for (uint32_t wv = blockIdx.x * (kThreads / 64) + (tid >> 6); wv < ntiles;
         wv += gridDim.x * (kThreads / 64)) {
        const uint32_t x = (wv % tiles_x) * 8 + (lane & 7);
        const uint32_t lr = (wv / tiles_x) * 8 + (lane >> 3);
        if (x >= a.w || lr >= a.nrows) continue;
        const uint32_t y = global_row(lr, a.row0, a.band_h, a.band_step);
        const uint64_t lp = (uint64_t)lr * a.w + x;
        uint32_t v[5];
#pragma unroll
        for (int i = 0; i < 5; ++i) v[i] = a.rng_in[(uint64_t)i * P + lp];
        uint32_t d = a.d_base;
        uint32_t k = 0;
        for (uint32_t s = 0; s < a.spp; ++s) {
            const float ru = xorwow_uniform(v, d);
            const float rv = xorwow_uniform(v, d);
            float dx, dy, dz;
            camera_dir(a, ((float)x + ru) / (float)a.w, ((float)y + rv) / (float)a.h, dx, dy, dz);
            Walker<ANYHIT, STATS> w;
            w.start(sc, true, dx, dy, dz);
            while (w.alive) w.step(sc, st);
            if (STATS) {
                const uint64_t rid = lp * a.spp + s;
                a.ray_stats[3 * rid] = w.cnt.nodes;
                a.ray_stats[3 * rid + 1] = w.cnt.leaves;
                a.ray_stats[3 * rid + 2] = w.cnt.tris;
            }
            k += w.hit ? 1u : 0u;
        }
        a.out[lp] = pixel_from_hits(k, a.spp);
    }
}

// ---------------------------------------------------------------------------
// k_render_packet: the wave walks the BIH as one packet of 64 rays.
//
// Every lane keeps its own interval [tMin, tMax] and makes the reference's
// own decision at each node: it visits the near child iff tMin < t[near]
// (interval [tMin, t[near]]) and the far child iff !(tMax < t[far])
// (interval [t[far], tMax]) -- the four cases of TraverseTree
// (CUDAKernels.cu:295-365) reduce to exactly that.  A lane's visited set and
// its intervals depend only on the path from the root, not on the order in
// which subtrees are walked, so the wave may walk the UNION of its lanes'
// sets in one order, with a 64-bit mask of the lanes that visit each node:
// every lane still tests exactly the leaves TraverseTree tests (reference
// walk), or a prefix of them in another order (any-hit walk, whose RGBA only
// needs "some tested triangle hit").
// Node index, masks and the triangle records are wave-uniform (scalar loads
// through the scalar cache); the per-lane intervals of the stack live in
// VGPRs indexed by the uniform stack pointer (s_set_gpr_idx), entries past
// kPacketRegs in a per-wave HBM area.
// ---------------------------------------------------------------------------
#ifndef BIH_PACKET_REGS
#define BIH_PACKET_REGS 16
#endif
constexpr int kPacketRegs = BIH_PACKET_REGS;
// child refs of the any-hit shortcut records (k_fast_refs)
constexpr uint32_t kFastLeaf = 0x80000000u, kFastDead = 0xffffffffu;

__device__ __forceinline__ unsigned long long lane_bit(uint32_t lane) { return 1ull << lane; }

// Scalar (SMEM) views of read-only tree data: a load through address space 4
// at a wave-uniform address is emitted as s_load_* (scalar cache) instead of
// a per-lane global_load.
typedef unsigned int su32x4 __attribute__((ext_vector_type(4)));
typedef float sf32x16 __attribute__((ext_vector_type(16)));
typedef __attribute__((address_space(4))) const su32x4 cnode_t;
typedef __attribute__((address_space(4))) const sf32x16 cprim_t;
typedef __attribute__((address_space(4))) const uint32_t cu32_t;

// MT for one primary-ray triangle record against this lane's ray.  The
// record holds the ray-independent parts for the camera origin O:
// {e1, e2, s = O - v0, q = cross(s, e1), tnum = dot(e2, q)} (k_tri_prim), so
// per lane only p = cross(D, e2), det, u, v and t = tnum * inv remain -- each
// the same f32 expression, in the same order, as RayTriangleIntersection
// (:18-47).  An early-out is taken only when no lane of the wave passes it
// (uniform branch); otherwise every lane evaluates the full predicate.
__device__ __forceinline__ bool prim_hit(const sf32x16 r, float dx, float dy, float dz) {
    const float px = dy * r[5] - r[4] * dz;          // pvec = cross(D, e2)
    const float py = dz * r[3] - r[5] * dx;
    const float pz = dx * r[4] - r[3] * dy;
    const float det = (r[0] * px + r[1] * py) + r[2] * pz;
    const bool ok_det = !(det <= kDetEps);           // det < 0.000001 (double); NaN passes
    if (!__any(ok_det)) return false;
    const float inv = 1.0f / det;
    const float u = ((r[6] * px + r[7] * py) + r[8] * pz) * inv;
    const bool ok_u = ok_det && !(u < 0.0f || u > 1.0f);
    if (!__any(ok_u)) return false;
    const float v = ((dx * r[9] + dy * r[10]) + dz * r[11]) * inv;
    const float t = r[12] * inv;
    return ok_u && !(v < 0.0f || u + v > 1.0f) && t > 0.0f && t < FLT_MAX;
}

// prim_hit with the record in this lane's registers (each lane its own
// triangle: the lane's hit in the previous frame of an item, k_render_bins'
// hit cache): the same f32 expressions in the same order, no wave-level
// early-outs.  r0..r2 = record words 0..11, t = word 12 (tnum).
__device__ __forceinline__ bool prim_hit_lane(const float4 r0, const float4 r1, const float4 r2, float tn, float dx,
                                              float dy, float dz) {
    const float e1x = r0.x, e1y = r0.y, e1z = r0.z, e2x = r0.w, e2y = r1.x, e2z = r1.y;
    const float px = dy * e2z - e2y * dz;            // pvec = cross(D, e2)
    const float py = dz * e2x - e2z * dx;
    const float pz = dx * e2y - e2x * dy;
    const float det = (e1x * px + e1y * py) + e1z * pz;
    const float inv = 1.0f / det;
    const float u = ((r1.z * px + r1.w * py) + r2.x * pz) * inv;
    const float v = ((dx * r2.y + dy * r2.z) + dz * r2.w) * inv;
    const float t = tn * inv;
    return !(det <= kDetEps) && !(u < 0.0f || u > 1.0f) && !(v < 0.0f || u + v > 1.0f) && t > 0.0f && t < FLT_MAX;
}

template <bool ANYHIT, bool STATS, int LOG2SPP>
__global__ void __launch_bounds__(kThreads) k_render_packet(const RenderArgs a) {
    constexpr uint32_t SPP = 1u << LOG2SPP;
    constexpr uint32_t TW = TileShape<LOG2SPP>::TW, TH = TileShape<LOG2SPP>::TH;
    constexpr int D = kPacketRegs;
    const uint32_t tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const unsigned long long me = lane_bit(lane);
    const uint64_t gwave = (uint64_t)blockIdx.x * (kThreads / 64) + wv;
    uint32_t *wspill = a.spill + gwave * (uint64_t)(kStackDepth - D) * 3 * 64;
    const SceneU sc = load_scene(a);
    const cnode_t *nodes = (const cnode_t *)(const void *)a.nodes;
    const cprim_t *prims = (const cprim_t *)(const void *)a.tri_prim;
    const cu32_t *dupc = (const cu32_t *)(const void *)a.dup_cnt;
    const uint32_t tiles_x = (a.w + TW - 1) / TW;
    const uint32_t ntiles = tiles_x * ((a.nrows + TH - 1) / TH);
    const float fw = (float)a.w, fh = (float)a.h;
    const uint32_t pix = lane >> LOG2SPP;

    for (;;) {
        uint32_t tile = 0;
        if (lane == 0) tile = atomicAdd(a.work, 1u);
        tile = __builtin_amdgcn_readfirstlane(tile);
        if (tile >= ntiles) break;
        uint32_t x, lr, s;
        ray_coords<LOG2SPP>((uint64_t)tile * 64 + lane, tiles_x, x, lr, s);
        const bool valid = x < a.w && lr < a.nrows;
        const uint64_t lp = (uint64_t)lr * a.w + x;
        float dx = 0.f, dy = 0.f, dz = 1.f;
        if (valid) {
            float ru = 0.f, rv = 0.f;
            ray_jitter<SPP>(a, lp, s, ru, rv);
            const uint32_t y = global_row(lr, a.row0, a.band_h, a.band_step);
            camera_dir(a, ((float)x + ru) / fw, ((float)y + rv) / fh, dx, dy, dz);
        }
        // Ray::Ray (Ray.cu:3-10) + scene-AABB slab test (CUDAKernels.cu:237-262)
        const float ix = 1.0f / dx, iy = 1.0f / dy, iz = 1.0f / dz;
        const uint32_t sg = (ix < 0.0f ? 1u : 0u) | (iy < 0.0f ? 2u : 0u) | (iz < 0.0f ? 4u : 0u);
        float tMin = (((sg & 1) ? sc.shi0 : sc.slo0) - sc.ox) * ix;
        float tMax = (((sg & 1) ? sc.slo0 : sc.shi0) - sc.ox) * ix;
        const float tymin = (((sg & 2) ? sc.shi1 : sc.slo1) - sc.oy) * iy;
        const float tymax = (((sg & 2) ? sc.slo1 : sc.shi1) - sc.oy) * iy;
        bool in_box = valid && !((tMin > tymax) || (tymin > tMax));
        if (tymin > tMin) tMin = tymin;
        if (tymax < tMax) tMax = tymax;
        const float tzmin = (((sg & 4) ? sc.shi2 : sc.slo2) - sc.oz) * iz;
        const float tzmax = (((sg & 4) ? sc.slo2 : sc.shi2) - sc.oz) * iz;
        in_box = in_box && !((tMin > tzmax) || (tzmin > tMax));
        if (tzmin > tMin) tMin = tzmin;
        if (tzmax < tMax) tMax = tzmax;
        bool hit = false;
        uint32_t c_nodes = 0, c_leaves = 0, c_tris = 0;
        // lanes whose ray is still searching
        unsigned long long live = sc.U > 0 ? __ballot(in_box) : 0ull;

        // test the triangles [b, b+n) for the lanes in m (every lane computes,
        // only the lanes of m record: no per-lane branch)
        auto test_leaf = [&](uint32_t b, uint32_t n, unsigned long long m) {
            if (STATS && (m & me)) ++c_leaves;
            for (uint32_t i = 0; i < n; ++i) {
                if (ANYHIT) {
                    m &= live;
                    if (!m) break;
                }
                const sf32x16 rec = prims[b + i];
                const bool in = (m & me) != 0ull;
                if (STATS) c_tris += in ? 1u : 0u;
                hit |= in && prim_hit(rec, dx, dy, dz);
                if (ANYHIT) live &= ~__ballot(hit);
            }
        };

        if (live && sc.U == 1) {                          // single leaf (reference: UB)
            test_leaf(0, sc.N, live);
        } else if (live) {
            float st[3 * D];   // per-lane entries {lo, hi, word} indexed by the uniform sp
            uint32_t cur = 0, sp = 0;
            unsigned long long act = live;
            for (;;) {
                if (STATS && (act & me)) ++c_nodes;
                const su32x4 nd = nodes[cur];
                const uint32_t ax = (nd.z >> 27) & 3u;
                const float org = ax == 0 ? sc.ox : (ax == 1 ? sc.oy : sc.oz);   // uniform
                const float inv = sel3(ax, ix, iy, iz);
                const bool nr = (sg >> ax) & 1u;
                const float t0 = (__uint_as_float(nd.x) - org) * inv;
                const float t1 = (__uint_as_float(nd.y) - org) * inv;
                const float tn = nr ? t1 : t0, tf = nr ? t0 : t1;
                const bool A = tMin < tn;                 // near child visited
                const bool nB = !(tMax < tf);             // far child visited
                // child intervals: near [tMin, tn], far [tf, tMax]
                const float lo_L = nr ? tf : tMin, hi_L = nr ? tMax : tn;
                const float lo_R = nr ? tMin : tf, hi_R = nr ? tn : tMax;
                const unsigned long long mN = __ballot(A) & act, mF = __ballot(nB) & act;
                const unsigned long long mnr = __ballot(nr);
                unsigned long long mL = (mN & ~mnr) | (mF & mnr);
                unsigned long long mR = (mN & mnr) | (mF & ~mnr);
                const uint32_t split = nd.z & kIdxMask, mid = nd.w & kIdxMask;
                const bool leafL = (nd.z >> 29) & 1u, leafR = (nd.z >> 30) & 1u;
                // near first for the majority of the packet
                const bool nearL = __popcll(act & mnr) * 2 <= (uint32_t)__popcll(act);
                if ((leafL && mL) || (leafR && mR)) {
                    uint32_t cL = (nd.w >> 27) & 3u, cR = (nd.w >> 29) & 3u;
                    if (leafL && cL == 0) cL = dupc[split];
                    if (leafR && cR == 0) cR = dupc[split + 1];
                    if (nearL) {
                        if (leafL && mL) test_leaf(mid - cL, cL, mL);
                        if (leafR && mR) test_leaf(mid, cR, mR);
                    } else {
                        if (leafR && mR) test_leaf(mid, cR, mR);
                        if (leafL && mL) test_leaf(mid - cL, cL, mL);
                    }
                }
                if (ANYHIT) {
                    mL &= live;
                    mR &= live;
                }
                const unsigned long long gL = leafL ? 0ull : mL, gR = leafR ? 0ull : mR;
                if (gL && gR) {
                    // descend near, stack far (node, mask, per-lane interval)
                    const uint32_t fnode = nearL ? split + 1 : split;
                    const unsigned long long fmask = nearL ? gR : gL;
                    const float flo = nearL ? lo_R : lo_L, fhi = nearL ? hi_R : hi_L;
                    // entry word: node index | this lane's mask bit << 31
                    const uint32_t word = fnode | (((fmask & me) != 0ull) ? 0x80000000u : 0u);
                    if (sp < (uint32_t)D) {
                        st[3 * sp] = flo;
                        st[3 * sp + 1] = fhi;
                        st[3 * sp + 2] = __uint_as_float(word);
                    } else {
                        uint32_t *q = wspill + ((sp - D) * 3) * 64 + lane;
                        q[0] = __float_as_uint(flo);
                        q[64] = __float_as_uint(fhi);
                        q[128] = word;
                    }
                    sp = __builtin_amdgcn_readfirstlane(sp + 1);
                    cur = nearL ? split : split + 1;
                    act = nearL ? gL : gR;
                    tMin = nearL ? lo_L : lo_R;
                    tMax = nearL ? hi_L : hi_R;
                } else if (gL) {
                    cur = split; act = gL; tMin = lo_L; tMax = hi_L;
                } else if (gR) {
                    cur = split + 1; act = gR; tMin = lo_R; tMax = hi_R;
                } else {
                    // pop until an entry still has a live lane
                    bool found = false;
                    while (sp > 0) {
                        sp = __builtin_amdgcn_readfirstlane(sp - 1);
                        uint32_t word;
                        float lo, hi;
                        if (sp < (uint32_t)D) {
                            lo = st[3 * sp];
                            hi = st[3 * sp + 1];
                            word = __float_as_uint(st[3 * sp + 2]);
                        } else {
                            const uint32_t *q = wspill + ((sp - D) * 3) * 64 + lane;
                            lo = __uint_as_float(q[0]);
                            hi = __uint_as_float(q[64]);
                            word = q[128];
                        }
                        unsigned long long m = __ballot(word >> 31);
                        if (ANYHIT) m &= live;
                        if (!m) continue;
                        cur = __builtin_amdgcn_readfirstlane(word & 0x7fffffffu);
                        act = m;
                        tMin = lo;
                        tMax = hi;
                        found = true;
                        break;
                    }
                    if (!found) break;
                }
            }
        }

        if (STATS && valid) {
            const uint64_t rid = lp * SPP + s;
            a.ray_stats[3 * rid] = c_nodes;
            a.ray_stats[3 * rid + 1] = c_leaves;
            a.ray_stats[3 * rid + 2] = c_tris;
        }
        const unsigned long long hb = __ballot(hit);
        if (valid && s == SPP - 1) {
            const unsigned long long m = (SPP == 64) ? ~0ull : ((1ull << SPP) - 1ull);
            a.out[lp] = pixel_from_hits(__popcll((hb >> (pix * SPP)) & m), SPP);
        }
    }
}

// ---------------------------------------------------------------------------
// k_render_packet2: the packet walk of k_render_packet, restructured so that
// the per-node work is mostly VALU and the wave-uniform control stays short:
//   * node records relative to the camera origin (k_node_prim): t = d * inv
//     with d = clip - O[axis] computed once per origin (same f32 subtraction
//     as the reference's (clip - origin[axis]), CUDAKernels.cu:300-301);
//   * no near/far swap: with s = sign of this lane's direction on the axis,
//       left  visited iff (t0 > (s ? tMax : tMin)) xor s,
//       right visited iff (t1 > (s ? tMin : tMax)) xnor s,
//     which is exactly tMin < t[near] (near) and !(tMax < t[far]) (far),
//     NaNs included (a NaN compare is false on both sides);
//   * hits kept as one wave-uniform mask; triangle early-outs on the lanes
//     that actually test the leaf;
//   * child order chosen once per packet and axis (majority direction).
// ---------------------------------------------------------------------------
__device__ __forceinline__ unsigned long long prim_hits(const sf32x16 r, float dx, float dy, float dz,
                                                       unsigned long long m,
                                                       uint32_t *cnt = nullptr) {
    const float px = dy * r[5] - r[4] * dz;          // pvec = cross(D, e2)
    const float py = dz * r[3] - r[5] * dx;
    const float pz = dx * r[4] - r[3] * dy;
    const float det = (r[0] * px + r[1] * py) + r[2] * pz;
#if BIH_PACKET_COUNTERS
    // wave-level outcome counters (debug builds): [0] tests, [1] all lanes
    // out at det, [2] at u, [3] reach v, [4] some hit, [5]/[6] division-free
    // filters on u / on u and v would drop every lane, [7] [6] but not [2]
    const bool lead = (threadIdx.x & 63) == 0;
    unsigned long long mf = 0;
    if (cnt) {
        if (lead) atomicAdd(cnt, 1u);
        const unsigned long long md = m & __ballot(!(det <= kDetEps));
        if (md) {
            const float un = (r[6] * px + r[7] * py) + r[8] * pz;
            const float vn = (dx * r[9] + dy * r[10]) + dz * r[11];
            const float lo = det * 0x1p-20f, hiu = det * (1.0f + 0x1p-20f);
            const float hiuv = det * (1.0f + 0x1p-18f);
            const unsigned long long fu = md & __ballot(!(un < -lo || un > hiu));
            const unsigned long long fuv = fu & __ballot(!(vn < -lo || un + vn > hiuv));
            if (lead && !fu) atomicAdd(cnt + 5, 1u);
            if (lead && !fuv) atomicAdd(cnt + 6, 1u);
            mf = fuv ? 1ull : 0ull;
        } else if (lead) {
            atomicAdd(cnt + 1, 1u);
        }
    }
#endif
    m &= __ballot(!(det <= kDetEps));                // det < 0.000001 (double); NaN passes
    if (!m) return 0ull;
    const float inv = 1.0f / det;
    const float u = ((r[6] * px + r[7] * py) + r[8] * pz) * inv;
    m &= __ballot(!(u < 0.0f || u > 1.0f));
#if BIH_PACKET_COUNTERS
    if (cnt && lead) {
        if (!m) atomicAdd(cnt + 2, 1u);
        else atomicAdd(cnt + 3, 1u);
        if (m && !mf) atomicAdd(cnt + 7, 1u);
    }
    if (cnt) {
        const float v = ((dx * r[9] + dy * r[10]) + dz * r[11]) * inv;
        const float t = r[12] * inv;
        const unsigned long long h = m & __ballot(!(v < 0.0f || u + v > 1.0f) && t > 0.0f && t < FLT_MAX);
        if (lead && h) atomicAdd(cnt + 4, 1u);
        if (h && !mf && lead) atomicAdd(cnt + 4, 0x10000u);   // a filter miss: must never happen
    }
#endif
    if (!m) return 0ull;
    const float v = ((dx * r[9] + dy * r[10]) + dz * r[11]) * inv;
    const float t = r[12] * inv;
    return m & __ballot(!(v < 0.0f || u + v > 1.0f) && t > 0.0f && t < FLT_MAX);
}



// The descend decision of one packet node step, wave-uniform: pickL = take
// the left child (nearL ? gL != 0 : gR == 0); the taken child gets mask gT,
// node cT and its lanes' intervals, the other (gO, cO, olo/ohi) is stacked
// when gO != 0.  Written as one SALU/VALU sequence (hipcc's own lowering of
// the same selects spends about twice the scalar instructions).
__device__ __forceinline__ void descend_pick(unsigned long long gL, unsigned long long gR,
                                             uint32_t nearL, uint32_t split, float loL, float hiL,
                                             float loR, float hiR, unsigned long long &gT,
                                             unsigned long long &gO, uint32_t &cT, uint32_t &cO,
                                             float &tlo, float &thi, float &olo, float &ohi) {
    uint32_t p, q;
    unsigned long long mk;
    asm volatile(
        "s_cmp_lg_u64 %[gL], 0\n\t"
        "s_cselect_b32 %[p], 1, 0\n\t"
        "s_cmp_eq_u64 %[gR], 0\n\t"
        "s_cselect_b32 %[q], 1, 0\n\t"
        "s_cmp_lg_u32 %[nearL], 0\n\t"
        "s_cselect_b32 %[p], %[p], %[q]\n\t"
        "s_cmp_lg_u32 %[p], 0\n\t"
        "s_cselect_b64 %[gT], %[gL], %[gR]\n\t"
        "s_cselect_b64 %[gO], %[gR], %[gL]\n\t"
        "s_cselect_b64 %[mk], -1, 0\n\t"
        "s_add_u32 %[cO], %[split], %[p]\n\t"
        "s_xor_b32 %[q], %[p], 1\n\t"
        "s_add_u32 %[cT], %[split], %[q]\n\t"
        "v_cndmask_b32_e64 %[tlo], %[loR], %[loL], %[mk]\n\t"
        "v_cndmask_b32_e64 %[thi], %[hiR], %[hiL], %[mk]\n\t"
        "v_cndmask_b32_e64 %[olo], %[loL], %[loR], %[mk]\n\t"
        "v_cndmask_b32_e64 %[ohi], %[hiL], %[hiR], %[mk]"
        : [p] "=&s"(p), [q] "=&s"(q), [mk] "=&s"(mk), [gT] "=&s"(gT), [gO] "=&s"(gO),
          [cT] "=&s"(cT), [cO] "=&s"(cO), [tlo] "=&v"(tlo), [thi] "=&v"(thi), [olo] "=&v"(olo),
          [ohi] "=&v"(ohi)
        : [gL] "s"(gL), [gR] "s"(gR), [nearL] "s"(nearL), [split] "s"(split), [loL] "v"(loL),
          [hiL] "v"(hiL), [loR] "v"(loR), [hiR] "v"(hiR)
        : "scc");
}

template <bool ANYHIT, bool STATS, int LOG2SPP>
__global__ void __launch_bounds__(kThreads) k_render_packet2(const RenderArgs a) {
    constexpr uint32_t SPP = 1u << LOG2SPP;
    constexpr uint32_t TW = TileShape<LOG2SPP>::TW, TH = TileShape<LOG2SPP>::TH;
    constexpr int D = kPacketRegs;
    const uint32_t tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const unsigned long long me = lane_bit(lane);
    const uint64_t gwave = (uint64_t)blockIdx.x * (kThreads / 64) + wv;
    uint32_t *wspill = a.spill + gwave * (uint64_t)(kStackDepth - D) * 3 * 64;
    const SceneU sc = load_scene(a);
    const cnode_t *nodes = (const cnode_t *)(const void *)(STATS ? a.node_prim : a.node_cull);
    const cprim_t *prims = (const cprim_t *)(const void *)a.tri_prim;
    const cu32_t *dupc = (const cu32_t *)(const void *)a.dup_cnt;
    const uint32_t tiles_x = (a.w + TW - 1) / TW;
    const uint32_t ntiles = tiles_x * ((a.nrows + TH - 1) / TH);
    const float fw = (float)a.w, fh = (float)a.h;
    const uint32_t pix = lane >> LOG2SPP;

    for (;;) {
        uint32_t tile = 0;
        if (lane == 0) tile = atomicAdd(a.work, 1u);
        tile = __builtin_amdgcn_readfirstlane(tile);
        if (tile >= ntiles) break;
        uint32_t x, lr, s;
        ray_coords<LOG2SPP>((uint64_t)tile * 64 + lane, tiles_x, x, lr, s);
        const bool valid = x < a.w && lr < a.nrows;
        const uint64_t lp = (uint64_t)lr * a.w + x;
        float dx = 0.f, dy = 0.f, dz = 1.f;
        if (valid) {
            float ru = 0.f, rv = 0.f;
            ray_jitter<SPP>(a, lp, s, ru, rv);
            const uint32_t y = global_row(lr, a.row0, a.band_h, a.band_step);
            camera_dir(a, ((float)x + ru) / fw, ((float)y + rv) / fh, dx, dy, dz);
        }
        // Ray::Ray (Ray.cu:3-10) + scene-AABB slab test (CUDAKernels.cu:237-262)
        const float ix = 1.0f / dx, iy = 1.0f / dy, iz = 1.0f / dz;
        const uint32_t sg = (ix < 0.0f ? 1u : 0u) | (iy < 0.0f ? 2u : 0u) | (iz < 0.0f ? 4u : 0u);
        float tMin = (((sg & 1) ? sc.shi0 : sc.slo0) - sc.ox) * ix;
        float tMax = (((sg & 1) ? sc.slo0 : sc.shi0) - sc.ox) * ix;
        const float tymin = (((sg & 2) ? sc.shi1 : sc.slo1) - sc.oy) * iy;
        const float tymax = (((sg & 2) ? sc.slo1 : sc.shi1) - sc.oy) * iy;
        bool in_box = valid && !((tMin > tymax) || (tymin > tMax));
        if (tymin > tMin) tMin = tymin;
        if (tymax < tMax) tMax = tymax;
        const float tzmin = (((sg & 4) ? sc.shi2 : sc.slo2) - sc.oz) * iz;
        const float tzmax = (((sg & 4) ? sc.slo2 : sc.shi2) - sc.oz) * iz;
        in_box = in_box && !((tMin > tzmax) || (tzmin > tMax));
        if (tzmin > tMin) tMin = tzmin;
        if (tzmax < tMax) tMax = tzmax;
        uint32_t c_nodes = 0, c_leaves = 0, c_tris = 0;
#if BIH_PACKET_COUNTERS
        uint32_t pk[8] = {1, 0, 0, 0, 0, 0, 0, 0};   // packet-level walk counters (debug builds)
#endif
        const unsigned long long live = sc.U > 0 ? __ballot(in_box) : 0ull;
        unsigned long long hits = 0ull;   // lanes whose ray hit some tested triangle
        // left child first on an axis when most of the packet runs +axis there
        uint32_t nearbits = 0;
#pragma unroll
        for (uint32_t k = 0; k < 3; ++k) {
            const unsigned long long neg = __ballot((sg >> k) & 1u) & live;
            if (__popcll(neg) * 2 <= __popcll(live)) nearbits |= 1u << k;
        }

        // test triangles [b, b+n) for the lanes of m
        auto test_leaf = [&](uint32_t b, uint32_t n, unsigned long long m) {
            if (STATS && (m & me)) ++c_leaves;
#if BIH_PACKET_COUNTERS
            ++pk[2];
#endif
            for (const uint32_t e = b + n; b < e; ++b) {
                if (ANYHIT) {
                    m &= ~hits;
                    if (!m) break;
                }
#if BIH_PACKET_COUNTERS
                ++pk[3];
                if (lane == 0) atomicAdd(a.work + kHistWord + 8 + (31 - __builtin_clz(__popcll(m))), 1u);
#endif
                if (STATS && (m & me)) ++c_tris;
#if BIH_PACKET_COUNTERS
                hits |= prim_hits(prims[b], dx, dy, dz, m, a.work + 56);
#else
                hits |= prim_hits(prims[b], dx, dy, dz, m);
#endif
            }
        };

        if (live && sc.U == 1) {                          // single leaf (reference: UB)
            test_leaf(0, sc.N, live);
        } else if (live) {
            // per-lane entries {lo, hi, node | this lane's mask bit << 31}, one
            // interleaved array (private memory: one dwordx3 access per push/pop)
            float st[3 * D];
            uint32_t cur = 0, sp = 0;
            unsigned long long act = live;
            for (;;) {
                if (STATS && (act & me)) ++c_nodes;
#if BIH_PACKET_COUNTERS
                ++pk[1];
                if (lane == 0) atomicAdd(a.work + kHistWord + (31 - __builtin_clz(__popcll(act))), 1u);
#endif
                const su32x4 nd = nodes[cur];
                const uint32_t ax = nd.z & 3u;          // prim record layout (k_node_prim)
                const float inv = ax == 2u ? iz : (ax == 1u ? iy : ix);
                const bool neg = (sg >> ax) & 1u;
                const float t0 = __uint_as_float(nd.x) * inv;
                const float t1 = __uint_as_float(nd.y) * inv;
                const unsigned long long mneg = __ballot(neg);
                unsigned long long gL = (__ballot(t0 > (neg ? tMax : tMin)) ^ mneg) & act;
                unsigned long long gR = ~(__ballot(t1 > (neg ? tMin : tMax)) ^ mneg) & act;
                const float lo_L = neg ? t0 : tMin, hi_L = neg ? tMax : t0;
                const float lo_R = neg ? tMin : t1, hi_R = neg ? t1 : tMax;
                const uint32_t split = nd.z >> 8, mid = nd.w & 0x3ffffffu;
                // bit 0: left is a leaf, bit 1: right (w' bits 26, 31)
                const uint32_t leaf = ((nd.w >> 26) & 1u) | ((nd.w >> 30) & 2u);
                const uint32_t nearL = (nearbits >> ax) & 1u;
                if (leaf) {
                    const unsigned long long tL = (leaf & 1u) ? gL : 0ull;
                    const unsigned long long tR = (leaf & 2u) ? gR : 0ull;
                    if (tL | tR) {
                        uint32_t cL = (nd.w >> 27) & 3u, cR = (nd.w >> 29) & 3u;
                        if (tL && cL == 0) cL = dupc[split];
                        if (tR && cR == 0) cR = dupc[split + 1];
                        if (nearL) {
                            if (tL) test_leaf(mid - cL, cL, tL);
                            if (tR) test_leaf(mid, cR, tR);
                        } else {
                            if (tR) test_leaf(mid, cR, tR);
                            if (tL) test_leaf(mid - cL, cL, tL);
                        }
                    }
                    if (leaf & 1u) gL = 0ull;
                    if (leaf & 2u) gR = 0ull;
                    if (ANYHIT) {
                        gL &= ~hits;
                        gR &= ~hits;
                    }
                }
                if (gL | gR) {
                    // take the near child (majority order) when both are
                    // visited, else the only one; stack the other if visited
                    unsigned long long gT, gO;
                    uint32_t cT, cO;
                    float tlo, thi, olo, ohi;
                    descend_pick(gL, gR, nearL, split, lo_L, hi_L, lo_R, hi_R, gT, gO, cT, cO, tlo,
                                 thi, olo, ohi);
                    if (gO) {
                        const uint32_t word = cO | ((uint32_t)((gO >> lane) & 1ull) << 31);
                        if (__builtin_expect(sp < (uint32_t)D, 1)) {
                            st[3 * sp] = olo;
                            st[3 * sp + 1] = ohi;
                            st[3 * sp + 2] = __uint_as_float(word);
                        } else {
                            uint32_t *q = wspill + ((sp - D) * 3) * 64 + lane;
                            q[0] = __float_as_uint(olo);
                            q[64] = __float_as_uint(ohi);
                            q[128] = word;
                        }
#if BIH_PACKET_COUNTERS
                        ++pk[4];
                        if (lane == 0) atomicAdd(a.work + 24 + (sp < 32 ? sp : 31), 1u);
                        pk[6] = sp + 1 > pk[6] ? sp + 1 : pk[6];
#endif
                        ++sp;
                    }
                    cur = cT;
                    act = gT;
                    tMin = tlo;
                    tMax = thi;
                    continue;
                }
                // pop until an entry still has a searching lane
                bool found = false;
                while (sp > 0) {
                    --sp;
#if BIH_PACKET_COUNTERS
                    ++pk[5];
#endif
                    uint32_t word;
                    float lo, hi;
                    if (sp < (uint32_t)D) {
                        lo = st[3 * sp];
                        hi = st[3 * sp + 1];
                        word = __float_as_uint(st[3 * sp + 2]);
                    } else {
                        const uint32_t *q = wspill + ((sp - D) * 3) * 64 + lane;
                        lo = __uint_as_float(q[0]);
                        hi = __uint_as_float(q[64]);
                        word = q[128];
                    }
                    unsigned long long m = __ballot(word >> 31);
                    if (ANYHIT) m &= ~hits;
                    if (!m) continue;
                    cur = __builtin_amdgcn_readfirstlane(word & 0x7fffffffu);
                    act = m;
                    tMin = lo;
                    tMax = hi;
                    found = true;
                    break;
                }
                if (!found) break;
            }
        }

#if BIH_PACKET_COUNTERS
        if (lane == 0) {
            for (int k = 0; k < 6; ++k) atomicAdd(a.work + 16 + k, pk[k]);
            atomicMax(a.work + 22, pk[6]);
            // packets by log2(node steps): count, node steps, triangle tests
            const uint32_t bin = pk[1] ? 31 - __builtin_clz(pk[1]) : 0;
            atomicAdd(a.work + kHistWord + 16 + bin, 1u);
            atomicAdd(a.work + kHistWord + 32 + bin, pk[1]);
            atomicAdd(a.work + kHistWord + 48 + bin, pk[3]);
        }
#endif
        if (STATS && valid) {
            const uint64_t rid = lp * SPP + s;
            a.ray_stats[3 * rid] = c_nodes;
            a.ray_stats[3 * rid + 1] = c_leaves;
            a.ray_stats[3 * rid + 2] = c_tris;
        }
        if (valid && s == SPP - 1) {
            const unsigned long long m = (SPP == 64) ? ~0ull : ((1ull << SPP) - 1ull);
            a.out[lp] = pixel_from_hits(__popcll((hits >> (pix * SPP)) & m), SPP);
        }
    }
}

// Tile scheduling of the persistent packet kernel, two levels:
//  * the image is cut into chunks of kChunkW x kChunkH tiles (a compact
//    block of pixels) and the chunks into kRegions bands of chunk rows, one
//    per XCD: an XCD drains its own band first (its L2 keeps that part of
//    the tree), then helps the others;
//  * all waves on one CU share one current chunk (per-CU slot, keyed by the
//    hardware CU id), so the ~28 packets in flight on a CU trace neighbouring
//    pixels and share the scalar cache's node and triangle lines.
// A slot is one 64-bit word {chunk + 1, next position}: a wave claims
// position p of the slot's chunk with one atomicAdd; the wave that draws
// p == chunk size (or the first one on an empty slot) refills it from the
// band counters; waves that overdraw wait (s_sleep) for the refill.
constexpr uint32_t kRegions = 8;
// 8 x 4 tiles (32 x 16 pixels).  With the any-hit shortcut (short packets):
// 8x4 0.632, 16x2 0.632, 8x2 0.649, 8x8 0.662, 4x4 0.668, 16x4 0.678, 4x2
// 0.86 ms per frame (3 in flight); with the exact walk 4x4 and 8x4 tied.
// Chunks of fewer tiles than half a CU's waves refill too often.
#ifndef BIH_CHUNK_W
#define BIH_CHUNK_W 8
#endif
#ifndef BIH_CHUNK_H
#define BIH_CHUNK_H 4
#endif
constexpr uint32_t kChunkW = BIH_CHUNK_W, kChunkH = BIH_CHUNK_H, kChunk = kChunkW * kChunkH;
constexpr uint32_t kSlotWord = 64;                     // work[64..): CU slots, kSlotStrideWords apart
constexpr unsigned long long kSlotDone = 0xFFFFFFFF00000000ull;

__device__ __forceinline__ uint32_t xcc_id() {
    uint32_t x;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
    return x & (kRegions - 1);
}

// (XCC, SE, SH, CU) -> 0..1023, unique per CU (tools/probe/hwid_probe.hip)
__device__ __forceinline__ uint32_t cu_key() {
    uint32_t h;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(h));
    return (xcc_id() << 7) | (((h >> 13) & 3u) << 5) | (((h >> 12) & 1u) << 4) | ((h >> 8) & 15u);
}

struct TileQueue {
    uint32_t *work;
    unsigned long long *slot;
    const uint32_t *order;             // chunk permutation (k_chunk_order) or null
    uint32_t tiles_x, tiles_y, chunks_x, nchunks;
    uint32_t band, left;
    uint32_t chunk;                    // chunk of the tile next() returned

    __device__ uint32_t band_begin(uint32_t b) const {
        const uint32_t rows = (nchunks / chunks_x);
        return (uint32_t)(((uint64_t)rows * b) / kRegions) * chunks_x;
    }

    // Next tile (global tile index t = ty * tiles_x + tx) for this wave.
    __device__ bool next(uint32_t lane, uint32_t &tile) {
        for (;;) {
            unsigned long long v = 0;
            if (lane == 0) v = atomicAdd(slot, 1ull);
            const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
            const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
            if (hi == 0xFFFFFFFFu) return false;
            if (hi != 0 && lo < kChunk) {
                const uint32_t g = hi - 1;
                const uint32_t tx = (g % chunks_x) * kChunkW + lo % kChunkW;
                const uint32_t ty = (g / chunks_x) * kChunkH + lo / kChunkW;
                if (tx < tiles_x && ty < tiles_y) {
                    tile = ty * tiles_x + tx;
                    chunk = g;
                    return true;
                }
                continue;                                // edge chunk: position off the image
            }
            if ((hi == 0 && lo == 0) || (hi != 0 && lo == kChunk)) {
                // this wave refills the slot with the next chunk of its band
                while (left) {
                    uint32_t c = 0;
                    if (lane == 0) c = atomicAdd(work + band, 1u);
                    c = __builtin_amdgcn_readfirstlane(c);
                    const uint32_t b0 = band_begin(band), b1 = band_begin(band + 1);
                    if (c < b1 - b0) {
                        const uint32_t g = order ? order[b0 + c] : b0 + c;
                        if (lane == 0) atomicExch(slot, ((unsigned long long)(g + 1) << 32) | 1ull);
                        tile = (g / chunks_x) * kChunkH * tiles_x + (g % chunks_x) * kChunkW;
                        chunk = g;
                        return true;                     // position 0: always on the image
                    }
                    band = (band + 1) & (kRegions - 1);
                    --left;
                }
                if (lane == 0) atomicExch(slot, kSlotDone);
                return false;
            }
            __builtin_amdgcn_s_sleep(4);                 // another wave is refilling
        }
    }
};

__device__ __forceinline__ TileQueue make_queue(const RenderArgs &a, uint32_t tiles_x,
                                                uint32_t tiles_y) {
    TileQueue q;
    q.work = a.work;
    q.slot = reinterpret_cast<unsigned long long *>(a.work + kSlotWord + kSlotStrideWords * cu_key());
    q.tiles_x = tiles_x;
    q.tiles_y = tiles_y;
    q.chunks_x = (tiles_x + kChunkW - 1) / kChunkW;
    q.nchunks = q.chunks_x * ((tiles_y + kChunkH - 1) / kChunkH);
    q.order = a.chunk_order;
    q.band = xcc_id();
    q.left = kRegions;
    q.chunk = 0;
    return q;
}

// ---------------------------------------------------------------------------
// Any-hit shortcut walk over one shortcut box set (k_fast_fit): the packet
// walks the boxes near-first and tests leaves with the exact intersector
// (prim_hits).  A lane stops at its first hit and keeps that leaf in `cand`.
// Returns the lanes with a candidate.  Nothing is decided here: a candidate
// stands only if fast_verify passes.
//   pass 1 (tight boxes, cons = false): finds the hits of most lanes fast;
//   pass 2 (miss-proof boxes, miss_box; cons = true): the whole line is
//     tested against every box, so a lane of `live` that ends with no
//     candidate has no triangle the exact intersector accepts: a reference
//     miss.  (The walk drops nothing: its stack cannot overflow, below.)
// Entry/exit parameters of the line O + t D against a camera-relative box,
// entry clamped below at cl.  Plain v_min/v_max (no NaN canonicalisation):
// no operand is NaN -- boxes are finite or +-inf, |1/D| >= 1/|D|max > 0 --
// and pass 2 only runs lanes with finite 1/D.
__device__ __forceinline__ void slab_t(float lx, float ly, float lz, float hx, float hy, float hz,
                                       float ix, float iy, float iz, float cl, float &tn,
                                       float &tf) {
    const float a0 = lx * ix, a1 = hx * ix, b0 = ly * iy, b1 = hy * iy;
    const float c0 = lz * iz, c1 = hz * iz;
    float n0, n1, n2, f0, f1, f2;
    asm("v_min_f32 %[n0], %[a0], %[a1]\n\t"
        "v_max_f32 %[f0], %[a0], %[a1]\n\t"
        "v_min_f32 %[n1], %[b0], %[b1]\n\t"
        "v_max_f32 %[f1], %[b0], %[b1]\n\t"
        "v_min_f32 %[n2], %[c0], %[c1]\n\t"
        "v_max_f32 %[f2], %[c0], %[c1]\n\t"
        "v_max3_f32 %[n0], %[n0], %[n1], %[n2]\n\t"
        "v_min3_f32 %[f0], %[f0], %[f1], %[f2]\n\t"
        "v_max_f32 %[n0], %[cl], %[n0]"
        : [n0] "=&v"(n0), [n1] "=&v"(n1), [n2] "=&v"(n2), [f0] "=&v"(f0), [f1] "=&v"(f1),
          [f2] "=&v"(f2)
        : [a0] "v"(a0), [a1] "v"(a1), [b0] "v"(b0), [b1] "v"(b1), [c0] "v"(c0), [c1] "v"(c1),
          [cl] "s"(cl));
    tn = n0;
    tf = f0;
}
// primary-ray triangle record i: one s_load with a 32-bit byte offset
__device__ __forceinline__ sf32x16 prim_rec(const cprim_t *prims, uint32_t i) {
    sf32x16 r;
    asm volatile("s_load_dwordx16 %0, %1, %2\n\t"
                 "s_waitcnt lgkmcnt(0)"
                 : "=s"(r)
                 : "s"(prims), "s"(i << 6)
                 : "memory");
    return r;
}
// shortcut records through the vector memory path (every lane the same
// address: one request per line) instead of scalar loads
#ifndef BIH_FAST_VLOAD
#define BIH_FAST_VLOAD 0
#endif
#ifndef BIH_FAST_NOEXACT
#define BIH_FAST_NOEXACT 0
#endif
#ifndef BIH_FAST_SINGLE
#define BIH_FAST_SINGLE 0
#endif
#ifndef BIH_FAST_MAJ
#define BIH_FAST_MAJ 0   // near order: majority of the lanes entering both (else the lowest)
#endif
#ifndef BIH_FAST_ASM_A
#define BIH_FAST_ASM_A 1   // child masks + near order as one asm sequence
#endif
__device__ __forceinline__ sf32x16 fast_rec(const float *boxes, uint32_t node) {
#if BIH_FAST_VLOAD
    float4 q0, q1, q2, q3;
    const float *p = boxes + 16ull * node;
    asm volatile("global_load_dwordx4 %0, %4, %5\n\t"
                 "global_load_dwordx4 %1, %4, %5 offset:16\n\t"
                 "global_load_dwordx4 %2, %4, %5 offset:32\n\t"
                 "global_load_dwordx4 %3, %4, %5 offset:48\n\t"
                 "s_waitcnt vmcnt(0)"
                 : "=&v"(q0), "=&v"(q1), "=&v"(q2), "=&v"(q3)
                 : "v"(0u), "s"(p)
                 : "memory");
    sf32x16 r;
    r[0] = q0.x; r[1] = q0.y; r[2] = q0.z; r[3] = q0.w;
    r[4] = q1.x; r[5] = q1.y; r[6] = q1.z; r[7] = q1.w;
    r[8] = q2.x; r[9] = q2.y; r[10] = q2.z; r[11] = q2.w;
    r[12] = __uint_as_float(__builtin_amdgcn_readfirstlane(__float_as_uint(q3.x)));
    r[13] = __uint_as_float(__builtin_amdgcn_readfirstlane(__float_as_uint(q3.y)));
    r[14] = __uint_as_float(__builtin_amdgcn_readfirstlane(__float_as_uint(q3.z)));
    r[15] = __uint_as_float(__builtin_amdgcn_readfirstlane(__float_as_uint(q3.w)));
    return r;
#else
    // one s_load with a 32-bit byte offset (no 64-bit address arithmetic);
    // loaded and waited for inside the statement
    sf32x16 r;
    asm volatile("s_load_dwordx16 %0, %1, %2\n\t"
                 "s_waitcnt lgkmcnt(0)"
                 : "=s"(r)
                 : "s"(boxes), "s"(node << 6)
                 : "memory");
    return r;
#endif
}
// BIH_FAST_COUNTERS builds: per-frame work of the shortcut passes in
// work[16..32) and their cycles in work[32..38) (printed by bih_sync)
#ifndef BIH_FAST_COUNTERS
#define BIH_FAST_COUNTERS 0
#endif
#if BIH_FAST_COUNTERS
#define BIH_FC(x) x
#else
#define BIH_FC(x)
#endif
__device__ __forceinline__ unsigned long long fast_walk(const float *boxes, bool cons,
                                                        const cprim_t *prims,
                                                        const cu32_t *dupc, float dx, float dy,
                                                        float dz, float ix, float iy, float iz,
                                                        unsigned long long live, uint32_t lane,
                                                        uint32_t &cand,
                                                        uint32_t &fc_steps, uint32_t &fc_tests) {
    const unsigned long long me = lane_bit(lane);
    unsigned long long found = 0ull;
    uint32_t node = 0;
    unsigned long long mask = live;
    int sp = 0;
    uint32_t st_node = 0, st_lo = 0, st_hi = 0;
    sf32x16 r = fast_rec(boxes, 0);
    while (true) {
        BIH_FC(++fc_steps);
        const uint32_t ref0 = __float_as_uint(r[12]), ref1 = __float_as_uint(r[13]);
        // slab test of both child boxes (camera-relative: t = box * inv); pass
        // 1 clamps the entry at t = 0 (the ray), pass 2 tests the whole line.
        // A dead child's box is NaN: never entered.
        const float cl = cons ? -INFINITY : 0.0f;
        float tn0, tf0, tn1, tf1;
        slab_t(r[0], r[1], r[2], r[3], r[4], r[5], ix, iy, iz, cl, tn0, tf0);
        slab_t(r[6], r[7], r[8], r[9], r[10], r[11], ix, iy, iz, cl, tn1, tf1);
        // child masks and the near child (as the lowest lane entering both
        // sees it), one SALU/VALU sequence (EXEC is the full wave here)
#if BIH_FAST_ASM_A
        unsigned long long m0, m1, lt, both;
        uint32_t first1, cnt_both;
        asm volatile("v_cmp_le_f32_e64 %[m0], %[tn0], %[tf0]\n\t"
                     "v_cmp_le_f32_e64 %[m1], %[tn1], %[tf1]\n\t"
                     "v_cmp_lt_f32_e64 %[lt], %[tn1], %[tn0]\n\t"
                     "s_and_b64 %[m0], %[m0], %[mask]\n\t"
                     "s_and_b64 %[m1], %[m1], %[mask]\n\t"
                     "s_and_b64 %[both], %[m0], %[m1]\n\t"
#if BIH_FAST_MAJ
                     "s_and_b64 %[lt], %[lt], %[both]\n\t"
                     "s_bcnt1_i32_b64 %[f1], %[lt]\n\t"
                     "s_bcnt1_i32_b64 %[c], %[both]\n\t"
                     "s_lshl_b32 %[f1], %[f1], 1\n\t"
                     "s_cmp_gt_u32 %[f1], %[c]\n\t"
#else
                     "s_ff1_i32_b64 %[f1], %[both]\n\t"
                     "s_bitcmp1_b64 %[lt], %[f1]\n\t"
#endif
                     "s_cselect_b32 %[f1], 1, 0"
                     : [m0] "=&s"(m0), [m1] "=&s"(m1), [lt] "=&s"(lt), [both] "=&s"(both),
                       [f1] "=&s"(first1), [c] "=&s"(cnt_both)
                     : [tn0] "v"(tn0), [tf0] "v"(tf0), [tn1] "v"(tn1), [tf1] "v"(tf1),
                       [mask] "s"(mask)
                     : "scc");
#else
        unsigned long long m0 = __ballot(tn0 <= tf0) & mask;
        unsigned long long m1 = __ballot(tn1 <= tf1) & mask;
        const unsigned long long both = m0 & m1;
        const uint32_t first1 = (__ballot(tn1 < tn0) & both & (0ull - both)) != 0ull ? 1u : 0u;
#endif
        if ((ref0 | ref1) & kFastLeaf) {
            // leaf children: test now (near one first)
#pragma unroll
            for (int q = 0; q < 2; ++q) {
                const int s = q ^ (first1 ? 1 : 0);
                const uint32_t ref = s ? ref1 : ref0;
                unsigned long long ms = (s ? m1 : m0) & ~found;
                if (!(ref & kFastLeaf) || !ms) continue;
                const uint32_t k = ref & ~kFastLeaf;
                const uint32_t fc = __float_as_uint(s ? r[15] : r[14]);
                const uint32_t b = fc & 0x3ffffffu;
                const uint32_t c = (fc >> 26) == 63u ? dupc[k] : (fc >> 26);
                for (uint32_t i = b; i < b + c && ms; ++i) {
                    const unsigned long long h = prim_hits(prim_rec(prims, i), dx, dy, dz, ms);
                    if (h & me) cand = k;
                    found |= h;
                    BIH_FC(++fc_tests);
                    ms &= ~h;
                }
            }
            if (ref0 & kFastLeaf) m0 = 0ull;
            if (ref1 & kFastLeaf) m1 = 0ull;
            m0 &= ~found;
            m1 &= ~found;
        }
        // descend: both children -> stack the far one (entry sp in lane sp of
        // st_node/st_lo/st_hi; sp < 31 always: at most one push per level and
        // the Karras tree of distinct 30-bit codes is at most 30 levels deep),
        // one child -> it, none -> pop
        uint32_t pop = 0;
        if (m0 && m1) {
            const uint32_t nf = first1 ? ref0 : ref1;
            const unsigned long long mf = first1 ? m0 : m1;
            uint32_t keep;   // M0 (the lane select) saved and restored
            asm volatile("s_mov_b32 %3, m0\n\t"
                         "s_mov_b32 m0, %7\n\t"
                         "s_nop 0\n\t"
                         "v_writelane_b32 %0, %4, m0\n\t"
                         "v_writelane_b32 %1, %5, m0\n\t"
                         "v_writelane_b32 %2, %6, m0\n\t"
                         "s_mov_b32 m0, %3"
                         : "+v"(st_node), "+v"(st_lo), "+v"(st_hi), "=&s"(keep)
                         : "s"(nf), "s"((uint32_t)mf), "s"((uint32_t)(mf >> 32)), "s"(sp));
            ++sp;
            node = first1 ? ref1 : ref0;
            mask = first1 ? m1 : m0;
        } else if (m0 | m1) {
            node = m0 ? ref0 : ref1;
            mask = m0 | m1;
        } else {
            pop = 1;
        }
        if (pop) {
            mask = 0ull;
            while (sp > 0) {
                --sp;
                mask = (((unsigned long long)__builtin_amdgcn_readlane(st_hi, sp) << 32) |
                        (uint32_t)__builtin_amdgcn_readlane(st_lo, sp)) & ~found;
                if (mask) {
                    node = __builtin_amdgcn_readlane(st_node, sp);
                    break;
                }
            }
            if (!mask) break;
        }
        r = fast_rec(boxes, node);
    }
    return found;
}

// Any-hit shortcut, pass 2: does the reference's own walk reach leaf `k`?
// Per lane, the exact BIH decisions of TraverseTree (CUDAKernels.cu:264-366)
// along the root path of leaf k (left iff k <= split: the Karras ranges),
// on the exact camera-relative records (k_node_prim): visit the near child
// iff tMin < t[near], the far child iff !(tMax < t[far]), intervals [tMin,
// t[near]] / [t[far], tMax] -- the same expressions as the packet walk's
// (BIH_NODE_DEC, BIH_DESCEND).  Every leaf the reference reaches is fully
// tested there, so a lane whose candidate triangle (an exact MT hit with
// 0 < t < FLT_MAX) lies in a reached leaf is a hit of the reference.
__device__ __forceinline__ bool fast_verify(const uint4 *__restrict__ rec, uint32_t k, float ix,
                                            float iy, float iz, float lo, float hi) {
    uint32_t n = 0;
    for (int d = 0; d < 64; ++d) {
        const uint4 r = rec[n];
        const uint32_t ax = r.z & 0xffu, split = r.z >> 8;
        const float inv = sel3(ax, ix, iy, iz);
        const bool neg = 0.0f > inv;
        const bool left = k <= split;
        bool g;
        float nlo, nhi;
        if (left) {
            const float t0 = __uint_as_float(r.x) * inv;
            const float sL = neg ? hi : lo;
            g = (t0 > sL) != neg;
            nlo = neg ? t0 : lo;
            nhi = neg ? hi : t0;
        } else {
            const float t1 = __uint_as_float(r.y) * inv;
            const float sR = neg ? lo : hi;
            g = (!(t1 > sR)) != neg;
            nlo = neg ? lo : t1;
            nhi = neg ? t1 : hi;
        }
        if (!g) return false;
        lo = nlo;
        hi = nhi;
        const uint32_t c = split + (left ? 0u : 1u);
        const bool leaf = left ? ((r.w >> 26) & 1u) : (r.w >> 31);
        if (leaf) return c == k;
        n = c;
    }
    return false;
}

// Exact MT of prim_hits with the division-free pre-test of the asm walk
// (BIH_MT, tests/test_mt_prefilter.py): lanes whose u numerator is certain to
// fail are dropped before the division.  Same f32 expressions, same result.
__device__ __forceinline__ unsigned long long prim_hits_pre(const sf32x16 r, float dx, float dy,
                                                           float dz, unsigned long long m) {
    const float px = dy * r[5] - r[4] * dz;          // pvec = cross(D, e2)
    const float py = dz * r[3] - r[5] * dx;
    const float pz = dx * r[4] - r[3] * dy;
    const float det = (r[0] * px + r[1] * py) + r[2] * pz;
    m &= __ballot(!(det <= kDetEps));                // det < 0.000001 (double); NaN passes
    if (!m) return 0ull;
    const float un = (r[6] * px + r[7] * py) + r[8] * pz;
    m &= __ballot(!(un < -(det * 0x1p-20f) || un > det * (1.0f + 0x1p-20f)));
    if (!m) return 0ull;
    const float inv = 1.0f / det;
    const float u = un * inv;
    m &= __ballot(!(u < 0.0f || u > 1.0f));
    if (!m) return 0ull;
    const float v = ((dx * r[9] + dy * r[10]) + dz * r[11]) * inv;
    const float t = r[12] * inv;
    return m & __ballot(!(v < 0.0f || u + v > 1.0f) && t > 0.0f && t < FLT_MAX);
}

// Frustum-bin walk (bih_bins.hip): the packet tests the triangles of its
// tile's list and then of the global list with the exact intersector until
// every lane of `live` has a hit.  Each 48-byte entry starts with the
// triangle's edge pre-test (three affine functions of the lane's f32 (u, v),
// each >= 0 whenever MT can accept): a lane failing one skips the triangle,
// and a triangle no remaining lane passes costs no MT.  A lane with a hit
// keeps the entry's leaf in `cand`; returns the lanes with a candidate.  A
// lane of `live` without one has tested every triangle the exact intersector
// could accept for its ray: a proven miss.
#ifndef BIH_BINS
#define BIH_BINS 1
#endif
// The list is streamed in chunks of 64 entries: lane j loads entry e + j
// (48 bytes, coalesced vector loads), the next chunk is requested
// before the current one is consumed, and each entry reaches the scalar unit
// by v_readlane -- one memory round trip per 64 entries instead of one per
// entry.
#ifndef BIH_SKIP_TRACE
#define BIH_SKIP_TRACE 0
#endif
#ifndef BIH_NO_VERIFY
#define BIH_NO_VERIFY 0
#endif
#ifndef BIH_BIN_PREFETCH_AT
#define BIH_BIN_PREFETCH_AT 16
#endif
#ifndef BIH_BIN_PREFETCH
#define BIH_BIN_PREFETCH 1
#endif
#ifndef BIH_BIN_SETBITS
#define BIH_BIN_SETBITS 1   // 0: the per-entry mask check (v_readlane + scalar test per entry)
#endif
#ifndef BIH_HIT_CACHE
#define BIH_HIT_CACHE 1   // 0: every frame of an item walks the tile's list from its start (A/B)
#endif
constexpr uint32_t kNoCache = 0xFFFFFFFFu;
#ifndef BIH_ENT_LDS
#define BIH_ENT_LDS 1   // bin_walk's pre-tests read their entry from LDS (broadcast), not by v_readlane
#endif
#ifndef BIH_ENT_KEEP
#define BIH_ENT_KEEP BIH_ENT_LDS   // the tile list's first chunk stays in LDS across an item's frames
#endif
#if BIH_ENT_KEEP && !(BIH_ENT_LDS && BIH_BIN_PREFETCH)
#error "BIH_ENT_KEEP needs BIH_ENT_LDS and BIH_BIN_PREFETCH"
#endif
#if BIH_ENT_LDS && !BIH_BIN_SETBITS
#error "BIH_ENT_LDS writes the chunk where the set-bits walk ballots it"
#endif
#ifndef BIH_HC_EARLY
#define BIH_HC_EARLY 0   // loads ahead of use: 1 stamp and entry together, 2 the record before the ray (A/B r06r-s: within noise)
#endif
#ifndef BIH_CACHE_MINLEN
#define BIH_CACHE_MINLEN 16   // list entries from which a tile's items use the hit cache
#endif
#ifndef BIH_PATHV_SKIP
#define BIH_PATHV_SKIP 0
#endif
#ifndef BIH_BIN_LOOP2
#define BIH_BIN_LOOP2 1   // 0: the entry loop tests todo && rem every entry (A/B)
#endif
#ifndef BIH_REC_LDS
#define BIH_REC_LDS 0   // multi-frame items: the records of the tile's first 64 entries in LDS
#endif
#ifndef BIH_REC_PREFETCH
#define BIH_REC_PREFETCH 0   // 1: neutral to slightly slower (0.0964 vs 0.094 ms/frame)
#endif
__device__ __forceinline__ float lane_f(float v, uint32_t j) {
    return __uint_as_float(__builtin_amdgcn_readlane(__float_as_uint(v), j));
}
__device__ __forceinline__ void bin_chunk_load(const float4 *ents, uint32_t e, uint32_t end,
                                               uint32_t lane, float4 &c0, float4 &c1, float4 &c2) {
    const uint32_t k = e + lane;
    if (k < end) {
        const float4 *p = ents + (uint64_t)kBinEntryF4 * k;
        c0 = p[0];
        c1 = p[1];
        c2 = p[2];
    }
}
// 16-bit mask of the pixels (4 lanes each, spp 4) that still have a lane in m
__device__ __forceinline__ uint32_t pixels_of(unsigned long long m) {
    m = (m | (m >> 1) | (m >> 2) | (m >> 3)) & 0x1111111111111111ull;
    m = (m | (m >> 3)) & 0x0303030303030303ull;
    m = (m | (m >> 6)) & 0x000F000F000F000Full;
    m = (m | (m >> 12)) & 0x000000FF000000FFull;
    return (uint32_t)((m | (m >> 24)) & 0xFFFFull);
}
// COUNT: count the entries pre-tested and the intersector calls into fc_ent /
// fc_mt (the work a launch that measures tile costs records)
template <bool PMASK, bool COUNT = false>
__device__ __forceinline__ unsigned long long bin_walk(const RenderArgs &a, const cprim_t *prims,
                                                      uint32_t bin, float uf, float vf, float dx,
                                                      float dy, float dz, unsigned long long live,
                                                      uint32_t lane, uint32_t &cand, uint32_t &cmeta,
                                                      uint32_t &cent, uint32_t &fc_ent,
                                                      uint32_t &fc_mt, uint32_t &pf,
                                                      const float4 *lrec = nullptr, uint32_t lrec_n = 0,
                                                      float4 *lent = nullptr, uint32_t *ltag = nullptr) {
    const cu32_t *off = (const cu32_t *)(const void *)a.bin_off;
    const float4 *ents = reinterpret_cast<const float4 *>(a.bin_list);
    uint32_t e = off[bin], end = off[bin + 1];
    const uint32_t e_first = e;
    unsigned long long rem = live;
    const unsigned long long me = lane_bit(lane);
    // spp 4: an entry whose pixel mask (word 11 >> 16, bih_bins.hip
    // pixel_mask) misses every pixel that still has a lane is skipped
    // before its pre-test
    uint32_t rpix = PMASK ? pixels_of(rem) : 0xFFFFu;
    for (int part = 0; part < 2; ++part) {
#if BIH_ENT_KEEP
        // the tile list's first chunk is still in the wave's LDS slots from
        // the previous frame of this tile (*ltag: the bin it belongs to)
        bool kept = part == 0 && *ltag == bin;
#else
        constexpr bool kept = false;
#endif
#if BIH_BIN_PREFETCH
        float4 c0 = make_float4(0.f, 0.f, 0.f, 0.f), c1 = c0, c2 = c0;
        if (e < end && !kept) bin_chunk_load(ents, e, end, lane, c0, c1, c2);
#endif
        while (e < end && rem) {
#if BIH_BIN_PREFETCH
            // the next chunk is requested once this one is a quarter done
            const float4 d0 = c0, d1 = c1, d2 = c2;
#else
            float4 d0 = make_float4(0.f, 0.f, 0.f, 0.f), d1 = d0, d2 = d0;
            bin_chunk_load(ents, e, end, lane, d0, d1, d2);
#endif
            const uint32_t n = end - e < 64u ? end - e : 64u;
#if BIH_REC_PREFETCH
            // touch every listed triangle's intersector record now (lane j:
            // entry j's), so that the scalar loads below hit L2 instead of
            // each paying a miss in turn; the value is folded into pf, which
            // the caller consumes after the walk (keeps the load alive)
            if (e + lane < end)
                pf ^= *reinterpret_cast<const volatile uint32_t *>(
                    reinterpret_cast<const uint32_t *>(a.tri_prim) + 16ull * __float_as_uint(d2.y));
#endif
#if BIH_BIN_SETBITS
            // the chunk's entries whose pixel mask meets a pixel that still
            // has a lane, as one ballot (lane j: entry j), walked in order by
            // find-first-set; a hit shrinks rpix and re-filters the rest --
            // the entries the per-entry mask check below would pre-test
#if BIH_ENT_KEEP
            const uint32_t pm =
                (kept ? reinterpret_cast<const uint32_t *>(lent + 3 * lane + 2)[3] : __float_as_uint(d2.w)) >> 16;
#else
            const uint32_t pm = __float_as_uint(d2.w) >> 16;
#endif
            unsigned long long todo = __ballot(lane < n && (!PMASK || (pm & rpix)));
#if BIH_ENT_LDS
            // the chunk's entries in the wave's LDS slots (lane j: entry j):
            // each pre-test then reads its entry's 9 plane words as one
            // broadcast instead of 9 v_readlane (12 fewer VALU per entry)
            if (!kept) {
                lent[3 * lane] = d0;
                lent[3 * lane + 1] = d1;
                lent[3 * lane + 2] = d2;
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#if BIH_ENT_KEEP
                *ltag = (part == 0 && e == e_first) ? bin : ~0u;
#endif
            }
#endif
#if BIH_BIN_PREFETCH
            if (e + 64u < end) bin_chunk_load(ents, e + 64u, end, lane, c0, c1, c2);
#endif
#if BIH_BIN_LOOP2
            // (the loop tests `todo` alone -- `rem` only after a hit, where it
            // can change -- and clears bit j with one s_bitset0: 6 scalar
            // instructions per rejected entry instead of 14)
            while (todo) {
                const uint32_t j = (uint32_t)__builtin_ctzll(todo);
                asm volatile("s_bitset0_b64 %0, %1" : "+s"(todo) : "s"(j));
#else
            while (todo && rem) {
                const uint32_t j = (uint32_t)__builtin_ctzll(todo);
                todo &= todo - 1ull;
#endif
#else
            for (uint32_t j = 0; j < n && rem; ++j) {
#if BIH_BIN_PREFETCH
                if (j == BIH_BIN_PREFETCH_AT && e + 64u < end)
                    bin_chunk_load(ents, e + 64u, end, lane, c0, c1, c2);
#endif
                if (PMASK && !((__builtin_amdgcn_readlane(__float_as_uint(d2.w), j) >> 16) & rpix)) continue;
#endif
#if BIH_ENT_LDS
                const float4 q0 = lent[3 * j], q1 = lent[3 * j + 1];
                const float q2x = reinterpret_cast<const float *>(lent + 3 * j + 2)[0];
                const float f0 = __builtin_fmaf(q0.z, vf, __builtin_fmaf(q0.y, uf, q0.x));
                const float f1 = __builtin_fmaf(q1.y, vf, __builtin_fmaf(q1.x, uf, q0.w));
                const float f2 = __builtin_fmaf(q2x, vf, __builtin_fmaf(q1.w, uf, q1.z));
#else
                const float f0 = __builtin_fmaf(lane_f(d0.z, j), vf,
                                                __builtin_fmaf(lane_f(d0.y, j), uf, lane_f(d0.x, j)));
                const float f1 = __builtin_fmaf(lane_f(d1.y, j), vf,
                                                __builtin_fmaf(lane_f(d1.x, j), uf, lane_f(d0.w, j)));
                const float f2 = __builtin_fmaf(lane_f(d2.x, j), vf,
                                                __builtin_fmaf(lane_f(d1.w, j), uf, lane_f(d1.z, j)));
#endif
                const unsigned long long in =
                    rem & __ballot(!(f0 < 0.0f) && !(f1 < 0.0f) && !(f2 < 0.0f));
                BIH_FC(++fc_ent);
                if (COUNT && !BIH_FAST_COUNTERS) ++fc_ent;
                if (!in) continue;
                BIH_FC(++fc_mt);
                if (COUNT && !BIH_FAST_COUNTERS) ++fc_mt;
#if BIH_ENT_LDS
                // the entry's words 9-11 (triangle, leaf, plan | pixel mask), broadcast
                const float4 q2 = lent[3 * j + 2];
                const uint32_t ti = (a.dbg & 1024u) ? 0u : __builtin_amdgcn_readfirstlane(__float_as_uint(q2.y));
#else
                const uint32_t ti = (a.dbg & 1024u) ? 0u : __builtin_amdgcn_readlane(__float_as_uint(d2.y), j);
#endif
                sf32x16 r;
                const uint32_t rel = e + j - e_first;          // (part 0: the tile's list)
                if (BIH_REC_LDS && part == 0 && rel < lrec_n) {
                    // the item's copy of the record in LDS (bin_rec_fill): an
                    // LDS round trip instead of a scalar load from L2/MALL
                    // one 16-byte read at a time straight into SGPRs (four
                    // VGPRs live, not 13: the walk is at its register peak)
#pragma unroll
                    for (int k = 0; k < 4; ++k) {
                        const float4 q = lrec[4 * rel + k];
                        r[4 * k] = __uint_as_float(__builtin_amdgcn_readfirstlane(__float_as_uint(q.x)));
                        if (k < 3) {
                            r[4 * k + 1] = __uint_as_float(__builtin_amdgcn_readfirstlane(__float_as_uint(q.y)));
                            r[4 * k + 2] = __uint_as_float(__builtin_amdgcn_readfirstlane(__float_as_uint(q.z)));
                            r[4 * k + 3] = __uint_as_float(__builtin_amdgcn_readfirstlane(__float_as_uint(q.w)));
                        }
                        asm volatile("" ::: "memory");
                    }
                } else {
                    r = prim_rec(prims, ti);
                }
                const unsigned long long h = prim_hits_pre(r, dx, dy, dz, in);
                if (h & me) {
#if BIH_ENT_LDS
                    cand = __float_as_uint(q2.z);
                    cmeta = __float_as_uint(q2.w);
#else
                    cand = __builtin_amdgcn_readlane(__float_as_uint(d2.z), j);
                    cmeta = __builtin_amdgcn_readlane(__float_as_uint(d2.w), j);
#endif
                    cent = ti;
                }
                rem &= ~h;
                if (PMASK && h) {
                    rpix = pixels_of(rem);
#if BIH_BIN_SETBITS
                    todo &= __ballot((pm & rpix) != 0u);
#endif
                }
#if BIH_BIN_SETBITS && BIH_BIN_LOOP2
                // (no lane left: the loop ends on todo -- with PMASK rpix is then
                // 0 and the ballot above already cleared it; one exit keeps the
                // loop free of the structurizer's break flags)
                if (!PMASK && !rem) todo = 0ull;
#endif
            }
            e += 64u;
#if BIH_ENT_KEEP
            kept = false;
#endif
        }
        if (!rem) break;
        ents = reinterpret_cast<const float4 *>(a.bin_glist);
        e = 0;
        end = *a.bin_gstat;   // the global list's length (the bins are usable here)
    }
    return live & ~rem;
}

// fast_verify over the leaf's root path from the per-camera path table
// (bih_bins.hip: 32 steps {clip - O[axis] of the side taken, axis | side << 2}
// root-first, end 8, 16 = never verified): the same decisions and intervals,
// with every load's address known up front (no dependent chain).
__device__ __forceinline__ bool path_step(uint32_t val, uint32_t meta, float ix, float iy, float iz,
                                          float &lo, float &hi, bool &done, bool &ok) {
    if (meta & 8u) {
        done = true;
        ok = (meta & 16u) == 0u;
        return false;
    }
    const float inv = sel3(meta & 3u, ix, iy, iz);
    const bool neg = 0.0f > inv;
    const float t = __uint_as_float(val) * inv;
    bool g;
    float nlo, nhi;
    if (!(meta & 4u)) {                       // left child
        const float sL = neg ? hi : lo;
        g = (t > sL) != neg;
        nlo = neg ? t : lo;
        nhi = neg ? hi : t;
    } else {                                  // right child
        const float sR = neg ? lo : hi;
        g = (!(t > sR)) != neg;
        nlo = neg ? lo : t;
        nhi = neg ? t : hi;
    }
    if (!g) {
        done = true;
        ok = false;
        return false;
    }
    lo = nlo;
    hi = nhi;
    return true;
}
// The first 24 steps are requested at once (one round trip for most
// leaves), the last 8 only by lanes whose path is longer.
#ifndef BIH_PATH_BATCH
#define BIH_PATH_BATCH 8
#endif
#ifndef BIH_PATH_FLAT
#define BIH_PATH_FLAT 1
#endif
#if BIH_PATH_FLAT
// path_step without control flow: the same decisions and intervals for a
// lane still walking (live); the compare bound and the updated end coincide
// (left: neg ? hi : lo, right: neg ? lo : hi -- the bound compared is the
// one the child keeps, the other becomes t)
__device__ __forceinline__ void path_step_flat(uint32_t val, uint32_t meta, float ix, float iy, float iz,
                                               float &lo, float &hi, bool &live, bool &ok) {
    const bool end = (meta & 8u) != 0u;
    const float inv = sel3(meta & 3u, ix, iy, iz);
    const bool neg = 0.0f > inv;
    const float t = __uint_as_float(val) * inv;
    const bool right = (meta & 4u) != 0u;
    const bool use_hi = neg != right;
    const bool gt = t > (use_hi ? hi : lo);
    const bool g = (right ? !gt : gt) != neg;
    ok = ok || (live && end && (meta & 16u) == 0u);
    live = live && !end && g;
    lo = (live && use_hi) ? t : lo;
    hi = (live && !use_hi) ? t : hi;
}
__device__ __forceinline__ bool path_verify(const uint2 *__restrict__ path, uint32_t k, float ix,
                                            float iy, float iz, float lo, float hi) {
    const uint4 *p = reinterpret_cast<const uint4 *>(path + 32ull * k);
    bool live = true, ok = false;
#pragma unroll
    for (int g = 0; g < 24 / BIH_PATH_BATCH; ++g) {
        // BIH_PATH_BATCH steps per round trip (8: 3 rounds, 16 VGPRs of
        // steps live instead of 48 -- that was k_render_bins' register peak:
        // 98 VGPRs and 4 waves per SIMD, now 79 and 6)
        uint4 q[BIH_PATH_BATCH / 2];
#pragma unroll
        for (int j = 0; j < BIH_PATH_BATCH / 2; ++j) q[j] = p[g * (BIH_PATH_BATCH / 2) + j];
#pragma unroll
        for (int j = 0; j < BIH_PATH_BATCH; ++j) {
            const uint4 w = q[j >> 1];
            path_step_flat((j & 1) ? w.z : w.x, (j & 1) ? w.w : w.y, ix, iy, iz, lo, hi, live, ok);
        }
    }
    if (__ballot(live)) {
        uint4 q[4];
        if (live) {
#pragma unroll
            for (int j = 0; j < 4; ++j) q[j] = p[12 + j];
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const uint4 w = q[j >> 1];
            path_step_flat((j & 1) ? w.z : w.x, (j & 1) ? w.w : w.y, ix, iy, iz, lo, hi, live, ok);
        }
    }
    return ok;
}
#else
__device__ __forceinline__ bool path_verify(const uint2 *__restrict__ path, uint32_t k, float ix,
                                            float iy, float iz, float lo, float hi) {
    const uint4 *p = reinterpret_cast<const uint4 *>(path + 32ull * k);
    bool done = false, ok = false;
    {
        uint4 q[12];
#pragma unroll
        for (int j = 0; j < 12; ++j) q[j] = p[j];
#pragma unroll
        for (int j = 0; j < 24; ++j) {
            const uint4 w = q[j >> 1];
            if (!path_step((j & 1) ? w.z : w.x, (j & 1) ? w.w : w.y, ix, iy, iz, lo, hi, done, ok))
                return ok;
        }
    }
    uint4 q[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) q[j] = p[12 + j];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const uint4 w = q[j >> 1];
        if (!path_step((j & 1) ? w.z : w.x, (j & 1) ? w.w : w.y, ix, iy, iz, lo, hi, done, ok))
            return ok;
    }
    return false;
}
#endif

// Ray::Ray (Ray.cu:3-10) + the scene-AABB slab test (CUDAKernels.cu:237-262):
// the ray's inverse direction and [tMin, tMax]; true when the ray meets the box
__device__ __forceinline__ bool scene_slab(const SceneU &sc, float dx, float dy, float dz, float &ix,
                                           float &iy, float &iz, float &tMin, float &tMax) {
    ix = 1.0f / dx;
    iy = 1.0f / dy;
    iz = 1.0f / dz;
    const uint32_t sg = (ix < 0.0f ? 1u : 0u) | (iy < 0.0f ? 2u : 0u) | (iz < 0.0f ? 4u : 0u);
    tMin = (((sg & 1) ? sc.shi0 : sc.slo0) - sc.ox) * ix;
    tMax = (((sg & 1) ? sc.slo0 : sc.shi0) - sc.ox) * ix;
    const float tymin = (((sg & 2) ? sc.shi1 : sc.slo1) - sc.oy) * iy;
    const float tymax = (((sg & 2) ? sc.slo1 : sc.shi1) - sc.oy) * iy;
    bool in_box = !((tMin > tymax) || (tymin > tMax));
    if (tymin > tMin) tMin = tymin;
    if (tymax < tMax) tMax = tymax;
    const float tzmin = (((sg & 4) ? sc.shi2 : sc.slo2) - sc.oz) * iz;
    const float tzmax = (((sg & 4) ? sc.slo2 : sc.shi2) - sc.oz) * iz;
    in_box = in_box && !((tMin > tzmax) || (tzmin > tMax));
    if (tzmin > tMin) tMin = tzmin;
    if (tzmax < tMax) tMax = tzmax;
    return in_box;
}
#ifndef BIH_SLAB_AGAIN
#define BIH_SLAB_AGAIN 0   // 1: 72 VGPRs, 7 waves, but 0.0420 vs 0.0413 ms per frame (A/B r04n)
#endif

// A plan's 1-2 critical comparisons (meta & 3 of them) on its values v
__device__ __forceinline__ bool plan_values_check(uint32_t meta, const float4 v, float ix, float iy, float iz,
                                                  float tMin, float tMax) {
    const uint32_t n = meta & 3u;
    bool ok = true;
#pragma unroll
    for (uint32_t c = 0; c < 2; ++c) {
        if (c >= n) break;
        const uint32_t m = meta >> (2 + 6 * c);
        const float vk = c ? v.z : v.x, vp = c ? v.w : v.y;
        const float tk = vk * sel3(m & 3u, ix, iy, iz);
        const bool is_exit = (m & 4u) != 0u;
        const float tp = (m & 32u) ? (is_exit ? tMin : tMax) : vp * sel3((m >> 3) & 3u, ix, iy, iz);
        ok = ok && (is_exit ? (tk > tp) : !(tk > tp));
    }
    return ok;
}

// The candidate's verification plan (triangle_plan, bih_bins.hip): the
// entry's leaf carries bit 31 when every decision on its root path is
// proven; otherwise meta & 3 = 1-2 critical comparisons, each t_k against
// t_p (another plane on the path, or the slab test's tMin / tMax), whose
// operands sit in the entry's last 16 bytes; 3 = the full root-path check.
__device__ __forceinline__ bool plan_verify(const RenderArgs &a, uint32_t cand, uint32_t meta,
                                            uint32_t cent, float ix, float iy, float iz, float tMin,
                                            float tMax) {
    if (cand >> 31) return true;
    meta &= 0xFFFFu;                   // (bits 16-31: the entry's pixel mask)
    const uint32_t n = meta & 3u;
#if BIH_PATHV_SKIP
    if (n == 3u) return true;   // timing experiment only: wrong pixels
#endif
    if (n == 3u) return path_verify(a.bin_path, cand, ix, iy, iz, tMin, tMax);
    // the triangle's plan values (its k_bin_fp record; the same in every list)
    return plan_values_check(meta, reinterpret_cast<const float4 *>(a.bin_rec)[4ull * cent + 3], ix, iy, iz,
                             tMin, tMax);
}

// plan_verify with the plan values already loaded (the hit cache's
// candidate: loaded before the frame's ray is made)
__device__ __forceinline__ bool plan_verify_v(const RenderArgs &a, uint32_t cand, uint32_t meta, const float4 v,
                                              float ix, float iy, float iz, float tMin, float tMax) {
    if (cand >> 31) return true;
    meta &= 0xFFFFu;
#if BIH_PATHV_SKIP
    if ((meta & 3u) == 3u) return true;
#endif
    if ((meta & 3u) == 3u) return path_verify(a.bin_path, cand, ix, iy, iz, tMin, tMax);
    return plan_values_check(meta, v, ix, iy, iz, tMin, tMax);
}

// ---------------------------------------------------------------------------
// k_render_bins: the any-hit render through the frustum bins alone (no BIH
// walk in this kernel).  Persistent waves draw items from the launch's tile
// queue (launch_bin_queue, bih_bins.hip): a wave starts in its XCD's band of
// tile rows and moves on to the others when that band is drained.  An item is
// a live tile -- one 64-ray packet: jitter, camera ray, scene slab test,
// bin_walk over the tile's list, plan_verify of each lane's candidate -- or
// 64 background tiles (one per lane), which no triangle's footprint touches.
// A packet whose lanes all end as a verified hit or a proven miss writes its
// pixels; a packet with a lane left undecided (a candidate the plan or the
// root-path check rejects, or a single-leaf scene) appends {tile, undecided,
// hits} to the slot's fallback list, and k_render_fallback finishes it with
// the exact walk.  Registers stay those of the list walk (no BIH walk state).
// Queue state (a "head set", kBinSetWords, zero at launch; the launch zeroes
// the slot's other set for its next launch): 8 band heads and the fallback
// count, then per-CU slots like TileQueue's -- a wave claims a position of
// its CU's current batch of kBinBatch consecutive items with one atomicAdd
// on the CU's own 128-byte line, and the wave that drains a batch refills
// the slot from a band head.  One device-wide atomic per batch instead of
// one per item: a single head word saturates near 90 dequeues per us.
// ---------------------------------------------------------------------------
#ifndef BIH_BINS_TIMELINE
#define BIH_BINS_TIMELINE 0   // diagnostic builds: per-item records of k_render_bins (bins_timeline_dump)
#endif
#if BIH_BINS_TIMELINE
// {wave | xcc << 24 | kind << 28, start, duration, list length} per queue
// item (s_memrealtime, 100 MHz); kind 0 live item, 1 background or advance
// item (length 1), 2 wave start, 3 wave exit.  Each wave appends to its own
// run of kTlPerWave records (no shared counter: a single atomic word would
// serialise the items, ~90 per us); g_tl_n[wave] counts them.
constexpr uint32_t kTlWaves = 1u << 14, kTlPerWave = 62;
__device__ uint32_t g_tl_n[kTlWaves];
__device__ uint4 g_tl_rec[kTlWaves * kTlPerWave];
__device__ __forceinline__ void tl_rec(uint32_t lane, uint32_t kind, uint64_t t0, uint64_t t1, uint32_t len) {
    const uint32_t wv = blockIdx.x * (kThreads / 64) + (threadIdx.x >> 6);
    if (lane == 0 && wv < kTlWaves) {
        const uint32_t k = g_tl_n[wv]++;
        if (k < kTlPerWave)
            g_tl_rec[wv * kTlPerWave + k] = make_uint4(wv | (xcc_id() << 24) | (kind << 28), (uint32_t)t0,
                                                       (uint32_t)(t1 - t0), len);
    }
}
#endif
#ifndef BIH_BINS_WAVES_PER_EU
#define BIH_BINS_WAVES_PER_EU 0   // 0: the compiler's choice (97 VGPRs, 4 waves: 0.048 vs 0.050 ms/frame forced to 5)
#endif
#if BIH_BINS_WAVES_PER_EU
#define BIH_BINS_OCC __attribute__((amdgpu_waves_per_eu(BIH_BINS_WAVES_PER_EU, BIH_BINS_WAVES_PER_EU)))
#else
#define BIH_BINS_OCC
#endif
constexpr uint32_t kFbWords = 8;   // fallback record: tile, undecided lo/hi, hits lo/hi, pad
#ifndef BIH_BIN_BATCH
#define BIH_BIN_BATCH 8   // A/B (16 frames per call): 8 0.0464 ms per frame, 16 0.0471, 32 0.0482
#endif
#ifndef BIH_PHASES
#define BIH_PHASES BIH_FAST_COUNTERS   // per-phase wave cycles (bih_sync prints them)
#endif
#ifndef BIH_QUEUE_STATIC
#define BIH_QUEUE_STATIC 0
#endif
#ifndef BIH_QUEUE_AHEAD
#define BIH_QUEUE_AHEAD 0   // 1: slower (0.112 vs 0.095 ms/frame): waves wait on refills held by busy waves
#endif
constexpr uint32_t kBinBatch = BIH_BIN_BATCH;
constexpr uint32_t kBinSlot0 = 16 * 32;   // words: heads at b * 32, fallback count at 8 * 32
struct BinQueue {
    const uint4 *hdr;                  // per band {start, live, bg, items}
    uint32_t *set;
    unsigned long long *slot;
    uint32_t band, left;
    uint4 hb;                          // header of the band of the item next() returned
    unsigned long long pending;        // a position claimed ahead (claim()), lane 0
    bool has_pending;
    // items per live tile: ns (RenderArgs::nsplit, frame ranges of a.fpi
    // frames); the band's first heavy[b] tiles take hs each instead
    // (RenderArgs::hsplit); a background item covers 64 tiles in every
    // frame.  hv = the heavy count of the band of the item next() returned
    // (the heavy counts follow the 8 band headers: launch_bin_queue's kQHeavy)
    uint32_t ns, hs, hv;
    __device__ __forceinline__ uint32_t extra(uint32_t b) const {
        return hs != ns ? reinterpret_cast<const uint32_t *>(hdr + 8)[b] : 0u;
    }
    __device__ __forceinline__ uint32_t band_items(const uint4 &h, uint32_t x) const {
        return x * hs + (h.y - x) * ns + (h.w - h.y);
    }
    // Start-up without atomics: each wave's first `rounds` items are static
    // -- in round r, block k's waves take items r * W(b) + (k >> 3) * 4 + w
    // of band b = k & 7, W(b) the band's waves (blocks are dealt round-robin
    // over the XCDs, so that is mostly the XCD's own band; only the speed
    // depends on it) -- and the band heads hand out the items after those:
    // stat(b) per band.  (Every wave starting in the per-CU slot made the 24
    // waves of a CU wait for three serial refills: 5.6 us median to a wave's
    // first item in a one-frame launch, 12 us at q90.)  rounds = 0 with a
    // shared grid, whose heads then hand out every item.
    uint32_t rounds, round;
    __device__ __forceinline__ uint32_t band_waves(uint32_t b) const {
        return gridDim.x > b ? ((gridDim.x - b + 7u) >> 3) * (kThreads / 64) : 0u;
    }
    __device__ __forceinline__ uint32_t stat(uint32_t b) const { return rounds * band_waves(b); }

    // Claims the slot position next() will use, so that its round trip
    // overlaps the current item's loads (BIH_QUEUE_AHEAD).
    __device__ void claim(uint32_t lane) {
        pending = 0;
        if (lane == 0) pending = atomicAdd(slot, 1ull);
        has_pending = true;
    }

    // next item: band (this->hb / band) and index within the band
    __device__ bool next(uint32_t lane, uint32_t &item) {
        if (round < rounds) {
            const uint32_t b = blockIdx.x & 7u;
            const uint32_t idx = round * band_waves(b) + (blockIdx.x >> 3) * (kThreads / 64) +
                                 __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
            ++round;
            const uint4 h = hdr[b];
            const uint32_t x = extra(b);
            if (idx < band_items(h, x)) {
                hb = h;
                hv = x;
                item = idx;
                return true;
            }
            round = rounds;   // (the band's items end before this wave's next round)
        }
        for (;;) {
            unsigned long long v = 0;
            if (has_pending) {
                v = pending;
                has_pending = false;
            } else if (lane == 0) {
                v = atomicAdd(slot, 1ull);
            }
            const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
            const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
            if (hi == 0xFFFFFFFFu) return false;
            if (hi != 0 && lo < kBinBatch) {
                const uint32_t b = (hi - 1u) >> 24, start = ((hi - 1u) & 0xFFFFFFu) * kBinBatch + stat(b);
                hb = hdr[b];
                hv = extra(b);
                if (start + lo < band_items(hb, hv)) {
                    item = start + lo;
                    band = b;
                    return true;
                }
                continue;                                // past the band's end
            }
            if ((hi == 0 && lo == 0) || (hi != 0 && lo == kBinBatch)) {
                while (left) {
                    const uint4 h = hdr[band];
                    const uint32_t x = extra(band);
                    uint32_t c = 0;
                    if (lane == 0) c = atomicAdd(set + band * 32, kBinBatch);
                    c = __builtin_amdgcn_readfirstlane(c);
                    if (c + stat(band) < band_items(h, x)) {
                        if (lane == 0)
                            atomicExch(slot, ((unsigned long long)(((band << 24) | (c / kBinBatch)) + 1u) << 32) | 1ull);
                        hb = h;
                        hv = x;
                        item = c + stat(band);
                        return true;
                    }
                    band = (band + 1u) & 7u;
                    --left;
                }
                if (lane == 0) atomicExch(slot, kSlotDone);
                return false;
            }
            __builtin_amdgcn_s_sleep(2);                 // another wave is refilling
        }
    }
};
// MODE 1: also write the per-tile hit masks (RenderArgs::hit_mask; the C4
// primary pass); MODE 2: also record each live tile's cycles per frame
// (RenderArgs::bin_cost; the launch after which the queue is ordered by
// measured cost); | kBinsStamped: the XORWOW state per tile
// (RenderArgs::stamps) -- separate instantiations, so the headline kernel
// keeps its registers
constexpr int kBinsStamped = 4;
#ifndef BIH_STAMPED_WAVES
#define BIH_STAMPED_WAVES 1   // 6: the stamped instance held to 6 waves per SIMD (scratch spills; one-frame calls 0.093 against 0.082 ms at its own 5)
#endif
// SGPR cap of k_render_bins (0: the compiler's choice, 106 + spills): below
// ~100 a wave's SGPR block leaves room in each SIMD's file beside 6 render
// waves for the waves of a concurrently dispatched kernel (the next call's
// XORWOW advance), and the stamped instance fits 6 waves' VGPRs
#ifndef BIH_BINS_SGPR
#define BIH_BINS_SGPR 0
#endif
#if BIH_BINS_SGPR
#define BIH_BINS_SGPR_ATTR __attribute__((amdgpu_num_sgpr(BIH_BINS_SGPR)))
#else
#define BIH_BINS_SGPR_ATTR
#endif
template <int LOG2SPP, int MODE = 0>
__global__ void __launch_bounds__(kThreads, (MODE & kBinsStamped) ? BIH_STAMPED_WAVES : 1) BIH_BINS_OCC
BIH_BINS_SGPR_ATTR k_render_bins(const RenderArgs a) {
    constexpr bool MASK = (MODE & 3) == 1, COST = (MODE & 3) == 2, STAMP = (MODE & kBinsStamped) != 0;
    constexpr uint32_t SPP = 1u << LOG2SPP;
    constexpr uint32_t TW = TileShape<LOG2SPP>::TW, TH = TileShape<LOG2SPP>::TH;
    const uint32_t tid = threadIdx.x, lane = tid & 63;
    __shared__ uint32_t s_rs[5][kThreads];   // each lane's XORWOW state between the frames of an item
#if BIH_HIT_CACHE
    __shared__ uint32_t s_hc[3][kThreads];   // each lane's hit of the item's previous frame: {record, leaf, plan}
#endif
#if BIH_ENT_LDS
    __shared__ float4 s_ent[kThreads / 64][64 * 3];   // per wave: the list chunk bin_walk pre-tests
    float4 *const lent = s_ent[tid >> 6];
#else
    float4 *const lent = nullptr;
#endif
    uint32_t ltag = ~0u;   // the bin whose list's first chunk is in lent (BIH_ENT_KEEP)
#if BIH_REC_LDS
    // per wave: the intersector records (tri_prim, 13 of 16 words) of its
    // item's first 64 list entries, loaded once and read by every frame of
    // the item (a multi-frame item walks the same list each frame; each
    // record's scalar load was a dependent round trip to L2/MALL per frame)
    __shared__ float4 s_rec[kThreads / 64][64 * 4];
    const float4 *lrec = s_rec[tid >> 6];
#else
    const float4 *lrec = nullptr;
#endif
    // the slot's next launch starts from a zeroed set: every one of the 1024
    // per-CU slot lines (cu_key() spans 0..1023 sparsely, whatever the grid)
    if (tid == 0)
        for (uint32_t k = blockIdx.x; k < 1024u; k += gridDim.x)
            *reinterpret_cast<unsigned long long *>(a.bin_heads_next + kBinSlot0 + k * 32) = 0ull;
    if (tid == 0)
        for (uint32_t k = blockIdx.x; k < 9u; k += gridDim.x) a.bin_heads_next[k * 32] = 0u;
    const SceneU sc = load_scene(a);
    const cprim_t *prims = (const cprim_t *)(const void *)a.tri_prim;
    const uint32_t tiles_x = (a.w + TW - 1) / TW;
    const float fw = (float)a.w, fh = (float)a.h;
    const uint32_t pix = lane >> LOG2SPP;
    const uint32_t bgpix = pixel_from_hits(0u, SPP);
    BinQueue q;
    q.hdr = reinterpret_cast<const uint4 *>(a.bin_qhdr);
    q.set = a.bin_heads;
    q.slot = reinterpret_cast<unsigned long long *>(a.bin_heads + kBinSlot0 + cu_key() * 32);
    q.band = xcc_id();
    q.left = 8;
    // (not while another render holds CU slots: this launch's blocks then
    // start as that one's waves exit, and a late block's static item -- the
    // band's costliest first -- would start late)
    q.rounds = a.shared_grid ? 0u : a.static_rounds;
    q.round = 0;
    q.has_pending = false;
    q.ns = a.nsplit;   // an item covers a tile in a.fpi consecutive frames of the launch
    q.hs = a.hsplit;
    q.hv = 0;
    uint32_t fpi = a.fpi;
    if (a.live_items && a.nframes > 1u) {
        // items per live tile from the queue's live count (the same in every
        // wave): a launch over few live tiles -- a small mesh, a rank's bands
        // -- splits its tiles' frames so that the items still outnumber the
        // waves; one over many keeps every frame of a tile in one item
        uint32_t live = 0;
        for (uint32_t b = 0; b < 8u; ++b) live += q.hdr[b].y;
        const uint32_t target = a.live_items & 0x7FFFFFFFu;
        uint32_t ns = live ? (target + live / 2u) / live : a.nframes;
        ns = ns < 1u ? 1u : (ns > a.nframes ? a.nframes : ns);
        fpi = (a.nframes + ns - 1u) / ns;
        ns = (a.nframes + fpi - 1u) / fpi;
        const uint32_t hx = ns * (a.nframes >= 8u ? 4u : 2u);
        q.ns = ns;
        q.hs = (a.live_items >> 31) ? (hx < a.nframes ? hx : a.nframes) : ns;
        if (q.hs < ns) q.hs = ns;
    }
    const uint32_t fhv = (a.nframes + q.hs - 1u) / q.hs;   // frames per item of a heavy tile
    uint32_t it = 0;
#if BIH_QUEUE_STATIC
    // timing experiment: items dealt round-robin over the waves (no atomics)
    const uint32_t nwv = gridDim.x * (kThreads / 64);
    uint32_t g_next = blockIdx.x * (kThreads / 64) + (threadIdx.x >> 6);
    g_next = __builtin_amdgcn_readfirstlane(g_next);
#endif
#if BIH_PHASES
    // per-phase wave cycles (s_memtime), summed over waves into work[64..75]
    unsigned long long ph[6] = {0, 0, 0, 0, 0, 0};   // queue, background, setup, walk, verify, write
    uint64_t tq = __builtin_amdgcn_s_memtime();
#define BIH_PH(k) do { const uint64_t t_ = __builtin_amdgcn_s_memtime(); ph[k] += t_ - tq; tq = t_; } while (0)
#else
#define BIH_PH(k) do { } while (0)
#endif
#if BIH_QUEUE_STATIC
    for (;;) {
        {
            uint32_t g = g_next, b = 0;
            g_next += nwv;
            uint4 h = q.hdr[0];
            while (b < 8u && g >= h.w) {
                g -= h.w;
                if (++b < 8u) h = q.hdr[b];
            }
            if (b >= 8u) break;
            q.hb = h;
            it = g;
        }
#else
#if BIH_BINS_TIMELINE
    const uint64_t tl_w0 = __builtin_amdgcn_s_memrealtime();
    tl_rec(lane, 2u, tl_w0, tl_w0, 0u);
#endif
    while (q.next(lane, it)) {
#endif
        BIH_PH(0);
#if BIH_BINS_TIMELINE
        const uint64_t tl_t0 = __builtin_amdgcn_s_memrealtime();
#endif
        const uint4 hb = q.hb;
        // an item covers its tile in frames [f0, nf) of the launch: the
        // band's first hv tiles (measured cost >= kHeavyFactor x the mean)
        // hs items each, frames [sp * fhv, (sp + 1) * fhv), so that no tile's
        // frames run for most of the launch on one wave; the other live tiles
        // ns items of a.fpi frames each -- tile-major, so the queue's LPT
        // order holds for the items; then the background items (`it` past
        // hb.y: 64 tiles each, every frame)
        uint32_t f0 = 0, nf = a.nframes;
        if (q.ns > 1u || q.hv) {   // (one item per tile: `it` is the tile's position already)
            const uint32_t hx = q.hv * q.hs;
            if (it < hx) {
                const uint32_t j = it / q.hs, sp = it - j * q.hs;
                it = j;
                f0 = sp * fhv;
                nf = f0 + fhv < a.nframes ? f0 + fhv : a.nframes;
            } else {
                const uint32_t k = it - hx, nx = (hb.y - q.hv) * q.ns;
                if (k < nx) {
                    const uint32_t j = k / q.ns, sp = k - j * q.ns;
                    it = q.hv + j;
                    f0 = sp * fpi;
                    nf = f0 + fpi < a.nframes ? f0 + fpi : a.nframes;
                } else {
                    it = hb.y + (k - nx);
                }
            }
        }
        if (it >= hb.y) {
            // background: every sample misses (Color's background), whatever its jitter
            const uint32_t k = (it - hb.y) * 64u + lane;
            if (k < hb.z && !(a.dbg & 1u)) {
                const uint32_t t = a.bin_queue[hb.x + hb.y + k];
                if (MASK) a.hit_mask[t] = 0ull;      // (one-frame launches)
                const uint32_t ty = t / tiles_x, tx = t - ty * tiles_x;
                const uint32_t x0 = tx * TW;
                for (uint32_t fj = f0; fj < nf; ++fj) {
                    uint32_t *const fout = a.out + (uint64_t)fj * a.out_stride;
                    for (uint32_t r = 0; r < TH; ++r) {
                        const uint32_t lr = ty * TH + r;
                        if (lr >= a.nrows) break;
                        uint32_t *o = fout + (uint64_t)lr * a.w + x0;
                        if (TW == 4 && x0 + 4 <= a.w && ((uintptr_t)o & 15u) == 0) {
                            *reinterpret_cast<uint4 *>(o) = make_uint4(bgpix, bgpix, bgpix, bgpix);
                        } else {
                            for (uint32_t c = 0; c < TW && x0 + c < a.w; ++c) o[c] = bgpix;
                        }
                    }
                }
            }
            BIH_PH(1);
#if BIH_BINS_TIMELINE
            tl_rec(lane, 1u, tl_t0, __builtin_amdgcn_s_memrealtime(), 0u);
#endif
            continue;
        }
        if (a.dbg & 2u) continue;
        const uint32_t tile = a.bin_queue[hb.x + it];
        uint32_t x, lr, s;
        ray_coords<LOG2SPP>((uint64_t)tile * 64 + lane, tiles_x, x, lr, s);
        const bool valid = x < a.w && lr < a.nrows;
        const uint64_t lp = (uint64_t)lr * a.w + x;
        const uint32_t ty = tile / tiles_x, tx = tile - ty * tiles_x;
        const uint32_t bin = (global_row(ty * TH, a.row0, a.band_h, a.band_step) / TH) * a.bins_x + tx;
        const uint32_t y = global_row(lr, a.row0, a.band_h, a.band_step);
        // the pixel's XORWOW state at the start of the launch's first frame;
        // each frame takes 2*SPP draws (cudaRender), sample s the draws
        // 2s+1 and 2s+2 of its frame
        // (kept in LDS between frames: registers stay those of the list walk)
        uint32_t dfr = a.d_base + f0 * (2u * SPP * kWeyl);   // Weyl counter at the start of frame fj
        if (valid) {
            // frame f0's state: the launch's first frame's stepped 2*SPP*f0
            // draws on (a later item split or a heavy tile's later frame
            // range: at most ~100 steps, against the frames the item renders)
            const uint64_t P = (uint64_t)a.nrows * a.w;
            const uint32_t *src = a.rng_in;
            uint32_t pre = 2u * SPP * f0;
            if (STAMP) {
                // the tile's stamped state, stepped to frame st_f0 + f0
                const StampBase sb = stamp_base(a.stamps[tile], a.st_seq);
                src = sb.b ? a.st_buf1 : a.st_buf0;
                pre = 2u * SPP * (a.st_f0 + f0 - sb.F);
            }
            uint32_t v[5];
#pragma unroll
            for (int i = 0; i < 5; ++i) v[i] = src[(uint64_t)i * P + lp];
            xorwow_steps(v, pre);
#pragma unroll
            for (int i = 0; i < 5; ++i) s_rs[i][tid] = v[i];
        }
#if BIH_HIT_CACHE
        s_hc[0][tid] = kNoCache;
        // (tiles with short lists: the walk finds a lane's triangle about as
        // fast as the cache test would -- a record gather and a full
        // intersector call per lane -- so they walk every frame)
        const bool use_cache = ((const uint32_t *)a.bin_off)[bin + 1] - ((const uint32_t *)a.bin_off)[bin] >=
                               BIH_CACHE_MINLEN;
        // the lane's hit of the tile's last item (an earlier launch of this
        // camera set's current queue, RenderArgs::hcache): valid while the
        // tile's stamp is the queue's sequence number; the triangle's leaf
        // word and plan come from its record (the words every list entry of
        // the triangle carries)
#if BIH_HC_EARLY & 1
        // (stamp and entry read together, the entry discarded unless the
        // stamp matches: one round trip, not two)
        if (use_cache && a.hcache && valid) {
            const uint32_t st = a.hstamp[tile];
            const uint32_t ti0 = a.hcache[(uint64_t)tile * 64 + lane];
            const uint32_t ti = st == a.hseq ? ti0 : kNoCache;
#else
        if (use_cache && a.hcache && valid && a.hstamp[tile] == a.hseq) {
            const uint32_t ti = a.hcache[(uint64_t)tile * 64 + lane];
#endif
            if (ti < a.hdr_n_tris) {
                const float4 m = reinterpret_cast<const float4 *>(a.bin_rec)[4ull * ti + 2];
                s_hc[0][tid] = ti;
                s_hc[1][tid] = __float_as_uint(m.z);
                s_hc[2][tid] = __float_as_uint(m.w);
            }
        }
#endif
        uint32_t lrec_n = 0;
#if BIH_REC_LDS
        if (nf - f0 >= 2u) {
            const uint32_t e0 = ((const uint32_t *)a.bin_off)[bin];
            const uint32_t len = ((const uint32_t *)a.bin_off)[bin + 1] - e0;
            lrec_n = len < 64u ? len : 64u;
            if (lane < lrec_n) {
                const uint32_t ti = __float_as_uint(
                    reinterpret_cast<const float4 *>(a.bin_list)[(uint64_t)kBinEntryF4 * (e0 + lane) + 2].y);
                const float4 *src = reinterpret_cast<const float4 *>(a.tri_prim) + 4ull * ti;
                const float4 q0 = src[0], q1 = src[1], q2 = src[2], q3 = src[3];
                float4 *dst = s_rec[tid >> 6] + 4 * lane;
                dst[0] = q0;
                dst[1] = q1;
                dst[2] = q2;
                dst[3] = q3;
            }
            // the wave's own LDS writes before its reads (lanes read other lanes' slots)
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        }
#endif
        // (measuring launches) the item's work: entries pre-tested + 4 x
        // intersector calls -- each call a dependent scalar load of the
        // record, which is what makes a tile slow; wall time on a SIMD shared
        // with five other waves orders the tiles worse
        uint32_t work = 0;
#if BIH_BINS_TIMELINE
        uint32_t tl_ent = 0, tl_mt = 0, tl_pv = 0, tl_pl = 0;   // per item: entries, intersector calls, lanes
                                                               // through the path table / a plan
#endif
        for (uint32_t fj = f0; fj < nf; ++fj, dfr += 2u * SPP * kWeyl) {
            uint32_t *const fout = a.out + (uint64_t)fj * a.out_stride;
            float dx = 0.f, dy = 0.f, dz = 1.f, uf = 0.f, vf = 0.f;
#if BIH_HIT_CACHE && (BIH_HC_EARLY & 2)
            // the cached candidate's intersector record and plan values,
            // requested before the ray is made (they depend on the lane's
            // last hit only), so that their round trip overlaps the jitter
            uint32_t cti = kNoCache;
            float4 cr0 = make_float4(0.f, 0.f, 0.f, 0.f), cr1 = cr0, cr2 = cr0, cv = cr0;
            float ctn = 0.f;
            if (use_cache && valid) {
                cti = s_hc[0][tid];
                if (cti != kNoCache) {
                    const float4 *rp = reinterpret_cast<const float4 *>(a.tri_prim) + 4ull * cti;
                    cr0 = rp[0];
                    cr1 = rp[1];
                    cr2 = rp[2];
                    ctn = reinterpret_cast<const float *>(rp)[12];
                    cv = reinterpret_cast<const float4 *>(a.bin_rec)[4ull * cti + 3];
                }
            }
#endif
            if (valid) {
                // the frame's 2*SPP draws on every lane (uniform control
                // flow); rs ends at the next frame's state
                // (the two words this sample takes are converted to floats,
                // not all 2*SPP: curand_uniform of the same words)
                uint32_t xu = 0u, xv = 0u;
                uint32_t d = dfr, rs[5];
#pragma unroll
                for (int i = 0; i < 5; ++i) rs[i] = s_rs[i][tid];
#pragma unroll 8
                for (uint32_t k = 0; k < 2u * SPP; ++k) {
                    const uint32_t x = dev::xorwow_next(rs, d);
                    if (k == 2u * s) xu = x;
                    if (k == 2u * s + 1u) xv = x;
                }
                const float ru = dev::xorwow_to_uniform(xu), rv = dev::xorwow_to_uniform(xv);
                if (fj + 1u < nf) {
#pragma unroll
                    for (int i = 0; i < 5; ++i) s_rs[i][tid] = rs[i];
                } else if (STAMP && nf == a.nframes && s == 0u) {
                    // stamped: the state after the launch's last frame
                    // (cudaRender's write-back, CUDAKernels.cu:419) into the
                    // tile's other buffer; other items of the tile read the
                    // base buffer, which nobody writes in this launch
                    const StampBase sb = stamp_base(a.stamps[tile], a.st_seq);
                    uint32_t *dst = sb.b ? a.st_buf0 : a.st_buf1;
                    const uint64_t P = (uint64_t)a.nrows * a.w;
#pragma unroll
                    for (int i = 0; i < 5; ++i) dst[(uint64_t)i * P + lp] = rs[i];
                }
                uf = ((float)x + ru) / fw;       // CUDAKernels.cu:414-415
                vf = ((float)y + rv) / fh;
                camera_dir(a, uf, vf, dx, dy, dz);
            }
            // Ray::Ray (Ray.cu:3-10) + scene-AABB slab test (CUDAKernels.cu:237-262)
            float ix, iy, iz, tMin, tMax;
            const bool in_box = valid && scene_slab(sc, dx, dy, dz, ix, iy, iz, tMin, tMax);
            const unsigned long long live = sc.U > 0 ? __ballot(in_box) : 0ull;
            unsigned long long hits = 0ull, undecided = 0ull;
            BIH_PH(2);
            // bins_ok: the lists were built (k_bin_status); else the exact walk decides
            const bool bins_ok = *a.bin_gstat != kBinsUnusable;
            if (live && sc.U > 1 && bins_ok && !(a.dbg & 8u)) {
                uint32_t cand = 0, cmeta = 0, cent = 0, fc_ent = 0, fc_mt = 0, pf = 0;
                // Hit cache (frames after an item's first): a lane first tests
                // the triangle it hit in the item's previous frame -- the exact
                // intersector on the new ray, then that candidate's verification
                // plan.  Any verified candidate proves the hit Color() needs
                // (a lane of the reference walk that reaches an accepting
                // triangle), whatever the order the candidates are tried in; a
                // lane it does not prove walks the list as before, and only a
                // full walk proves a miss.  The jitter moves a sample within its
                // pixel, so most lanes hit the same small triangle again.
                unsigned long long chit = 0ull;
#if BIH_HIT_CACHE
                if (use_cache && !(a.dbg & 20u)) {
#if BIH_HC_EARLY & 2
                    const bool okc = in_box && cti != kNoCache && prim_hit_lane(cr0, cr1, cr2, ctn, dx, dy, dz) &&
                                     plan_verify_v(a, s_hc[1][tid], s_hc[2][tid], cv, ix, iy, iz, tMin, tMax);
#else
                    const uint32_t cti = s_hc[0][tid];
                    bool okc = false;
                    if (in_box && cti != kNoCache) {
                        const float4 *rp = reinterpret_cast<const float4 *>(a.tri_prim) + 4ull * cti;
                        const float4 r0 = rp[0], r1 = rp[1], r2 = rp[2];
                        const float tn = reinterpret_cast<const float *>(rp)[12];
                        okc = prim_hit_lane(r0, r1, r2, tn, dx, dy, dz) &&
                              plan_verify(a, s_hc[1][tid], s_hc[2][tid], cti, ix, iy, iz, tMin, tMax);
                    }
#endif
                    chit = __ballot(okc);
                }
#endif
                const unsigned long long wlive = live & ~chit;
                const unsigned long long found = wlive ? bin_walk<LOG2SPP == 2, COST || BIH_BINS_TIMELINE>(
                    a, prims, bin, uf, vf, dx, dy, dz, wlive, lane, cand, cmeta, cent, fc_ent, fc_mt, pf, lrec,
                    lrec_n, lent, &ltag) : 0ull;
                if (COST) work += fc_ent + 4u * fc_mt;
#if BIH_BINS_TIMELINE
                tl_ent += fc_ent;
                tl_mt += fc_mt;
                tl_pv += (uint32_t)__popcll(__ballot(((found >> lane) & 1ull) && !(cand >> 31) && (cmeta & 3u) == 3u));
                tl_pl += (uint32_t)__popcll(__ballot(((found >> lane) & 1ull) && !(cand >> 31) && (cmeta & 3u) != 3u));
#endif
                if (pf == 0x7f7f7f7fu && a.dbg == 0xdeadbeefu) a.out[0] = pf;   // (never: keeps the touches)
                BIH_PH(3);
#if BIH_SLAB_AGAIN
                // the slab test's values again for the verification, not kept
                // live across the walk (the walk's register peak)
                {
                    float ex = dx, ey = dy, ez = dz;
                    asm volatile("" : "+v"(ex), "+v"(ey), "+v"(ez));
                    scene_slab(sc, ex, ey, ez, ix, iy, iz, tMin, tMax);
                }
#endif
                const bool ok = ((found >> lane) & 1ull) &&
                                ((a.dbg & 16u) || plan_verify(a, cand, cmeta, cent, ix, iy, iz, tMin, tMax));
                hits = __ballot(ok) | chit;
                undecided = wlive & found & ~hits;
#if BIH_HIT_CACHE
                // the next frame of the item tries this one first (also a hit
                // among the list's first entries: every lane the cache settles
                // leaves the walk, whose pixel masks then skip more entries --
                // caching only hits past the 4th / 12th entry was slower, r06l)
                if (use_cache && ok) {
                    s_hc[0][tid] = cent;
                    s_hc[1][tid] = cand;
                    s_hc[2][tid] = cmeta;
                }
#endif
                BIH_PH(4);
#if BIH_FAST_COUNTERS
                {   // bin counters (bih_sync prints them): candidates decided by a
                    // plan, and plans that disagree with the root-path check (0)
                    const bool fnd = ((found >> lane) & 1ull) != 0ull;
                    const bool planned = fnd && ((cand >> 31) || (cmeta & 3u) != 3u);
                    const bool pv = fnd && path_verify(a.bin_path, cand & 0x7fffffffu, ix, iy, iz, tMin, tMax);
                    const unsigned long long rb = __ballot(planned), bad = __ballot(planned && (pv != ok));
                    if (lane == 0) {
                        atomicAdd(a.work + 38, (uint32_t)__popcll(bad));
                        atomicAdd(a.work + 39, (uint32_t)__popcll(rb));
                        atomicAdd(a.work + 40, 1u);
                        atomicAdd(a.work + 41, (uint32_t)__popcll(live));
                        atomicAdd(a.work + 42, fc_ent);
                        atomicAdd(a.work + 43, fc_mt);
                        atomicAdd(a.work + 44, (uint32_t)__popcll(found));
                        atomicAdd(a.work + 45, (uint32_t)__popcll(hits));
                        atomicAdd(a.work + 46, (uint32_t)__popcll(undecided));
                        atomicAdd(a.work + 47, found != wlive ? 1u : 0u);
                        atomicAdd(a.work + 52, (uint32_t)__popcll(chit));
                    }
                }
#endif
                if (a.dbg & 4u) {              // tests: every live lane to the fallback
                    hits = 0ull;
                    undecided = live;
                }
            } else if (live) {
                undecided = live;              // one leaf (U == 1) or no lists: the exact walk decides
            }
            if (undecided) {
                uint32_t r = 0;
                if (lane == 0) r = atomicAdd(a.bin_heads + 8 * 32, 1u);
                r = __builtin_amdgcn_readfirstlane(r);
                if (lane < 6) {
                    const uint32_t v[6] = {tile, (uint32_t)undecided, (uint32_t)(undecided >> 32), (uint32_t)hits,
                                           (uint32_t)(hits >> 32), fj};
                    a.bin_fb[(uint64_t)r * kFbWords + lane] = v[lane];
                }
                continue;
            }
            if (valid && s == SPP - 1) {
                const unsigned long long m = (SPP == 64) ? ~0ull : ((1ull << SPP) - 1ull);
                fout[lp] = pixel_from_hits(__popcll((hits >> (pix * SPP)) & m), SPP);
            }
            if (MASK && lane == 0) a.hit_mask[tile] = hits;
            BIH_PH(5);
        }
        if (COST && lane == 0) a.bin_cost[bin] = (work << 8) / (nf - f0);
#if BIH_HIT_CACHE
        if (use_cache && a.hcache) {   // for the tile's next item (a later launch)
            if (valid) a.hcache[(uint64_t)tile * 64 + lane] = s_hc[0][tid];
            if (lane == 0) a.hstamp[tile] = a.hseq;
        }
#endif
        if (STAMP && nf == a.nframes && lane == 0) {
            // (the item ending at the launch's last frame) the tile's new stamp
            const StampBase sb = stamp_base(a.stamps[tile], a.st_seq);
            a.stamps[tile] = stamp_pack(a.st_f0 + a.nframes, sb.b ^ 1u, sb, a.st_seq);
        }
#if BIH_BINS_TIMELINE
        tl_rec(lane, 0u, tl_t0, __builtin_amdgcn_s_memrealtime(),
               (((const uint32_t *)a.bin_off)[bin + 1] - ((const uint32_t *)a.bin_off)[bin]) | ((nf - f0) << 24));
        tl_rec(lane, 4u, tl_ent, tl_ent + tl_mt, tl_pv | (tl_pl << 16));   // {ent, mt, pv | pl << 16}
#endif
    }
#if BIH_BINS_TIMELINE
    {
        const uint64_t t = __builtin_amdgcn_s_memrealtime();
        tl_rec(lane, 3u, t, t, 0u);
    }
#endif
#if BIH_PHASES
    if (lane == 0)
        for (int k = 0; k < 6; ++k)
            atomicAdd(reinterpret_cast<unsigned long long *>(a.work + 64) + k, ph[k]);
#endif
#undef BIH_PH
}

// The packets k_render_bins left undecided: the undecided lanes take the
// exact any-hit walk (Walker: TraverseTree as the reference runs it, per
// lane, LDS stack), then the tile's pixels are written.  Launched after every
// k_render_bins on the same stream; with no fallback record it only reads
// the count.
template <int LOG2SPP>
__global__ void __launch_bounds__(kThreads) k_render_fallback(const RenderArgs a) {
    constexpr uint32_t SPP = 1u << LOG2SPP;
    constexpr uint32_t TW = TileShape<LOG2SPP>::TW;
    __shared__ uint32_t s_node[kLdsStack * kThreads];
    __shared__ float s_min[kLdsStack * kThreads];
    __shared__ float s_max[kLdsStack * kThreads];
    const uint32_t tid = threadIdx.x, lane = tid & 63;
    const uint32_t n = *(volatile const uint32_t *)(a.bin_heads + 8 * 32);
    const uint64_t gwave = (uint64_t)blockIdx.x * (kThreads / 64) + (tid >> 6);
    const uint64_t nwaves = (uint64_t)gridDim.x * (kThreads / 64);
    if (gwave >= n) return;
    const Stack st = {s_node, s_min, s_max, tid, a.spill, (uint64_t)gridDim.x * kThreads,
                      (uint64_t)blockIdx.x * kThreads + tid};
    const SceneU sc = load_scene(a);
    const uint32_t tiles_x = (a.w + TW - 1) / TW;
    const float fw = (float)a.w, fh = (float)a.h;
    const uint32_t pix = lane >> LOG2SPP;
    for (uint64_t r = gwave; r < n; r += nwaves) {
        const uint32_t *rec = a.bin_fb + r * kFbWords;
        const uint32_t tile = rec[0];
        const unsigned long long und = ((unsigned long long)rec[2] << 32) | rec[1];
        unsigned long long hits = ((unsigned long long)rec[4] << 32) | rec[3];
        const uint32_t fj = rec[5];                      // frame of a multi-frame launch
        uint32_t *const fout = a.out + (uint64_t)fj * a.out_stride;
        uint32_t x, lr, s;
        ray_coords<LOG2SPP>((uint64_t)tile * 64 + lane, tiles_x, x, lr, s);
        const bool valid = x < a.w && lr < a.nrows;
        const uint64_t lp = (uint64_t)lr * a.w + x;
        const bool mine = valid && ((und >> lane) & 1ull);
        float dx = 0.f, dy = 0.f, dz = 1.f;
        if (mine) {
            float ru = 0.f, rv = 0.f;
            ray_jitter<SPP>(a, lp, s, ru, rv, fj, tile);
            const uint32_t y = global_row(lr, a.row0, a.band_h, a.band_step);
            camera_dir(a, ((float)x + ru) / fw, ((float)y + rv) / fh, dx, dy, dz);
        }
        Walker<true, false> w;
        w.start(sc, mine, dx, dy, dz);
        while (w.alive) w.step(sc, st);
        hits |= __ballot(mine && w.hit);
        if (valid && s == SPP - 1) {
            const unsigned long long m = (SPP == 64) ? ~0ull : ((1ull << SPP) - 1ull);
            fout[lp] = pixel_from_hits(__popcll((hits >> (pix * SPP)) & m), SPP);
        }
        if (a.hit_mask && lane == 0) a.hit_mask[tile] = hits;
    }
}

// k_render_packet_asm: k_render_packet2 with the walk as one hand-scheduled
// loop (bih_packet_asm.h); ray setup and writeback stay in HIP.  Triangle
// offsets are 32-bit in the loop: used for scenes of < 2^26 triangles.
// ---------------------------------------------------------------------------
#ifndef BIH_ASM_WAVES_PER_EU
#define BIH_ASM_WAVES_PER_EU 7
#endif
template <bool ANYHIT, bool STATS, int LOG2SPP>
__global__ void __launch_bounds__(kThreads)
__attribute__((amdgpu_waves_per_eu(BIH_ASM_WAVES_PER_EU, BIH_ASM_WAVES_PER_EU)))
k_render_packet_asm(const RenderArgs a) {
    constexpr uint32_t SPP = 1u << LOG2SPP;
    constexpr uint32_t TW = TileShape<LOG2SPP>::TW, TH = TileShape<LOG2SPP>::TH;
    const uint32_t tid = threadIdx.x, lane = tid & 63;
    const uint32_t wv = __builtin_amdgcn_readfirstlane(tid >> 6);
    const uint64_t gwave = (uint64_t)blockIdx.x * (kThreads / 64) + wv;
    const uint32_t *wspill = a.spill + gwave * (uint64_t)(kStackDepth - kPacketRegs) * 3 * 64;
    const SceneU sc = load_scene(a);
    const cprim_t *prims = (const cprim_t *)(const void *)a.tri_prim;
    const void *nodes = (const void *)(STATS ? a.node_prim : a.node_cull);
    const void *dupc = (const void *)a.dup_cnt;
    const uint32_t tiles_x = (a.w + TW - 1) / TW;
    const uint32_t ntiles = tiles_x * ((a.nrows + TH - 1) / TH);
    const float fw = (float)a.w, fh = (float)a.h;
    const uint32_t pix = lane >> LOG2SPP;
    const uint32_t lane4 = lane * 4u;
    const uint32_t snan = 0x7f800001u;
    const uint32_t eps = __float_as_uint(kDetEps), fmax = __float_as_uint(FLT_MAX);

    TileQueue queue = make_queue(a, tiles_x, (a.nrows + TH - 1) / TH);
    uint32_t tile = 0;
    (void)ntiles;
#if BIH_WAVE_TIMELINE
    const uint64_t tl_begin = __builtin_amdgcn_s_memrealtime();
    uint64_t tl_last = tl_begin;
    uint32_t tl_packets = 0, tl_live = 0, tl_max = 0;
    uint64_t tl_max_at = tl_begin, tl_pk = tl_begin;
#endif
    while (queue.next(lane, tile)) {
        const uint64_t t_start = __builtin_amdgcn_s_memtime();
        uint32_t x, lr, s;
        ray_coords<LOG2SPP>((uint64_t)tile * 64 + lane, tiles_x, x, lr, s);
        const bool valid = x < a.w && lr < a.nrows;
        const uint64_t lp = (uint64_t)lr * a.w + x;
        float dx = 0.f, dy = 0.f, dz = 1.f, uf = 0.f, vf = 0.f;
        if (valid) {
            float ru = 0.f, rv = 0.f;
            ray_jitter<SPP>(a, lp, s, ru, rv);
            const uint32_t y = global_row(lr, a.row0, a.band_h, a.band_step);
            uf = ((float)x + ru) / fw;
            vf = ((float)y + rv) / fh;
            camera_dir(a, uf, vf, dx, dy, dz);
        }
        // Ray::Ray (Ray.cu:3-10) + scene-AABB slab test (CUDAKernels.cu:237-262)
        const float ix = 1.0f / dx, iy = 1.0f / dy, iz = 1.0f / dz;
        const uint32_t sg = (ix < 0.0f ? 1u : 0u) | (iy < 0.0f ? 2u : 0u) | (iz < 0.0f ? 4u : 0u);
        float tMin = (((sg & 1) ? sc.shi0 : sc.slo0) - sc.ox) * ix;
        float tMax = (((sg & 1) ? sc.slo0 : sc.shi0) - sc.ox) * ix;
        const float tymin = (((sg & 2) ? sc.shi1 : sc.slo1) - sc.oy) * iy;
        const float tymax = (((sg & 2) ? sc.slo1 : sc.shi1) - sc.oy) * iy;
        bool in_box = valid && !((tMin > tymax) || (tymin > tMax));
        if (tymin > tMin) tMin = tymin;
        if (tymax < tMax) tMax = tymax;
        const float tzmin = (((sg & 4) ? sc.shi2 : sc.slo2) - sc.oz) * iz;
        const float tzmax = (((sg & 4) ? sc.slo2 : sc.shi2) - sc.oz) * iz;
        in_box = in_box && !((tMin > tzmax) || (tzmin > tMax));
        if (tzmin > tMin) tMin = tzmin;
        if (tzmax < tMax) tMax = tzmax;
        uint32_t c_nodes = 0, c_leaves = 0, c_tris = 0;
#if BIH_SKIP_TRACE   // timing experiments only: the kernel without any traversal
        unsigned long long live = 0ull;
        (void)in_box;
#else
        unsigned long long live = sc.U > 0 ? __ballot(in_box) : 0ull;
#endif
        unsigned long long hits = 0ull, shortcut = 0ull;
#if BIH_FAST_COUNTERS
        uint64_t fc_walk0 = __builtin_amdgcn_s_memtime();
#endif
        if (ANYHIT && !STATS && a.fast && live && sc.U > 1) {
            // any-hit shortcut: lanes whose shortcut hit the reference's walk
            // provably reaches are done; the others take the exact walk below
            uint32_t cand = 0, s1 = 0, n1 = 0, s2 = 0, n2 = 0;
            (void)s1, (void)n1, (void)s2, (void)n2;
            BIH_FC(const uint64_t fc_t0 = __builtin_amdgcn_s_memtime());
            const unsigned long long fin =
                __ballot(__builtin_isfinite(ix) && __builtin_isfinite(iy) && __builtin_isfinite(iz));
#if BIH_FAST_SINGLE
            // one conservative pass: hits and miss proofs together
            const bool single = a.fast2 != nullptr;
#else
            const bool single = false;
#endif
            const unsigned long long m1 = single ? live & fin : live;
            const unsigned long long found =
                fast_walk(single ? a.fast2 : a.fast, single, prims, (const cu32_t *)dupc, dx, dy,
                          dz, ix, iy, iz, m1, lane, cand, s1, n1);
            BIH_FC(const uint64_t fc_tw = __builtin_amdgcn_s_memtime());
            const bool ok = ((found >> lane) & 1ull) &&
                            fast_verify(a.node_prim, cand, ix, iy, iz, tMin, tMax);
            shortcut = __ballot(ok);
            BIH_FC(const unsigned long long fc_live0 = live);
            BIH_FC(const uint32_t fc_v1 = (uint32_t)__popcll(shortcut));
            live &= ~shortcut;
            if (single) live &= ~(m1 & ~found);   // proven misses
            BIH_FC(const uint64_t fc_t1 = __builtin_amdgcn_s_memtime());
            // miss proof for the rest (lanes with an infinite 1/D component
            // keep the exact walk: 0 * inf in a slab test)
            const unsigned long long m2 = a.fast2 && !single ? live & fin : 0ull;
            if (m2) {
                const unsigned long long found2 =
                    fast_walk(a.fast2, true, prims, (const cu32_t *)dupc, dx, dy, dz, ix, iy, iz,
                              m2, lane, cand, s2, n2);
                const bool ok2 = ((found2 >> lane) & 1ull) &&
                                 fast_verify(a.node_prim, cand, ix, iy, iz, tMin, tMax);
                const unsigned long long hit2 = __ballot(ok2);
                shortcut |= hit2;
                live &= ~(hit2 | (m2 & ~found2));   // proven misses are done too
                BIH_FC(if (lane == 0) {
                    atomicAdd(a.work + 22, 1u);
                    atomicAdd(a.work + 23, s2);
                    atomicAdd(a.work + 24, n2);
                    atomicAdd(a.work + 25, (uint32_t)__popcll(hit2));
                    atomicAdd(a.work + 26, (uint32_t)__popcll(m2 & ~found2));
                })
            }
#if BIH_FAST_COUNTERS
            const uint64_t fc_t2 = __builtin_amdgcn_s_memtime();
            if (lane == 0) {
                unsigned long long *cy = reinterpret_cast<unsigned long long *>(a.work + 32);
                atomicAdd(a.work + 16, 1u);
                atomicAdd(a.work + 17, (uint32_t)__popcll(fc_live0));
                atomicAdd(a.work + 18, s1);
                atomicAdd(a.work + 19, n1);
                atomicAdd(a.work + 20, (uint32_t)__popcll(found));
                atomicAdd(a.work + 21, fc_v1);
                atomicAdd(a.work + 28, live ? 1u : 0u);
                atomicAdd(a.work + 29, (uint32_t)__popcll(live));
                atomicAdd(cy, (unsigned long long)(fc_t1 - fc_t0));
                atomicAdd(cy + 1, (unsigned long long)(fc_t2 - fc_t1));
                atomicAdd(cy + 3, (unsigned long long)(fc_tw - fc_t0));
            }
            fc_walk0 = __builtin_amdgcn_s_memtime();
#endif
        }
        uint32_t nearbits = 0;
#pragma unroll
        for (uint32_t k = 0; k < 3; ++k) {
            const unsigned long long neg = __ballot((sg >> k) & 1u) & live;
            if (__popcll(neg) * 2 <= __popcll(live)) nearbits |= 1u << k;
        }
        nearbits = __builtin_amdgcn_readfirstlane(nearbits);
        if (live && sc.U == 1) {                          // single leaf (reference: UB)
            unsigned long long m = live;
            if (STATS && (m & lane_bit(lane))) ++c_leaves;
            for (uint32_t b = 0; b < sc.N; ++b) {
                if (ANYHIT) {
                    m &= ~hits;
                    if (!m) break;
                }
                if (STATS && (m & lane_bit(lane))) ++c_tris;
                hits |= prim_hits(prims[b], dx, dy, dz, m);
            }
        } else if (live) {
            if constexpr (ANYHIT && !STATS) {
#if BIH_FAST_NOEXACT
                // timing experiments only (wrong for unresolved lanes)
#else
                asm volatile(BIH_PACKET_WALK(BIH_ANY_ON, BIH_CLR_ON,
                                             BIH_POP_ANY,
                                             "", "", "", "", "")
                             : [hits] "=&s"(hits), [tmin] "+v"(tMin), [tmax] "+v"(tMax)
                             : [nodes] "s"(nodes), [prims] "s"(prims), [dupc] "s"(dupc),
                               [spill] "s"(wspill), [live] "s"(live), [near] "s"(nearbits),
                               [eps] "s"(eps), [fmax] "s"(fmax), [snan] "v"(snan),
                               [lane4] "v"(lane4), [dx] "v"(dx), [dy] "v"(dy), [dz] "v"(dz),
                               [ix] "v"(ix), [iy] "v"(iy), [iz] "v"(iz), [sgn] "v"(sg)
                             : BIH_PACKET_CLOBBERS);
#endif
            } else if constexpr (ANYHIT && STATS) {
                asm volatile(BIH_PACKET_WALK(BIH_ANY_ON, BIH_CLR_ON,
                                             BIH_POP_ANY,
                                             BIH_CNT_NODE, BIH_CNT_LEAF_L, BIH_CNT_LEAF_R,
                                             BIH_CNT_TRI_L, BIH_CNT_TRI_R)
                             : [hits] "=&s"(hits), [tmin] "+v"(tMin), [tmax] "+v"(tMax),
                               [cn] "+v"(c_nodes), [cl] "+v"(c_leaves), [ct] "+v"(c_tris)
                             : [nodes] "s"(nodes), [prims] "s"(prims), [dupc] "s"(dupc),
                               [spill] "s"(wspill), [live] "s"(live), [near] "s"(nearbits),
                               [eps] "s"(eps), [fmax] "s"(fmax), [snan] "v"(snan),
                               [lane4] "v"(lane4), [dx] "v"(dx), [dy] "v"(dy), [dz] "v"(dz),
                               [ix] "v"(ix), [iy] "v"(iy), [iz] "v"(iz), [sgn] "v"(sg)
                             : BIH_PACKET_CLOBBERS);
            } else if constexpr (!ANYHIT && !STATS) {
                asm volatile(BIH_PACKET_WALK(BIH_ANY_OFF, BIH_CLR_OFF, "", "", "", "", "", "")
                             : [hits] "=&s"(hits), [tmin] "+v"(tMin), [tmax] "+v"(tMax)
                             : [nodes] "s"(nodes), [prims] "s"(prims), [dupc] "s"(dupc),
                               [spill] "s"(wspill), [live] "s"(live), [near] "s"(nearbits),
                               [eps] "s"(eps), [fmax] "s"(fmax), [snan] "v"(snan),
                               [lane4] "v"(lane4), [dx] "v"(dx), [dy] "v"(dy), [dz] "v"(dz),
                               [ix] "v"(ix), [iy] "v"(iy), [iz] "v"(iz), [sgn] "v"(sg)
                             : BIH_PACKET_CLOBBERS);
            } else {
                asm volatile(BIH_PACKET_WALK(BIH_ANY_OFF, BIH_CLR_OFF, "",
                                             BIH_CNT_NODE, BIH_CNT_LEAF_L, BIH_CNT_LEAF_R,
                                             BIH_CNT_TRI_L, BIH_CNT_TRI_R)
                             : [hits] "=&s"(hits), [tmin] "+v"(tMin), [tmax] "+v"(tMax),
                               [cn] "+v"(c_nodes), [cl] "+v"(c_leaves), [ct] "+v"(c_tris)
                             : [nodes] "s"(nodes), [prims] "s"(prims), [dupc] "s"(dupc),
                               [spill] "s"(wspill), [live] "s"(live), [near] "s"(nearbits),
                               [eps] "s"(eps), [fmax] "s"(fmax), [snan] "v"(snan),
                               [lane4] "v"(lane4), [dx] "v"(dx), [dy] "v"(dy), [dz] "v"(dz),
                               [ix] "v"(ix), [iy] "v"(iy), [iz] "v"(iz), [sgn] "v"(sg)
                             : BIH_PACKET_CLOBBERS);
            }
        }
        hits |= shortcut;
#if BIH_FAST_COUNTERS
        if (lane == 0 && live)
            atomicAdd(reinterpret_cast<unsigned long long *>(a.work + 32) + 2,
                      (unsigned long long)(__builtin_amdgcn_s_memtime() - fc_walk0));
#endif

        if (STATS && valid) {
            const uint64_t rid = lp * SPP + s;
            a.ray_stats[3 * rid] = c_nodes;
            a.ray_stats[3 * rid + 1] = c_leaves;
            a.ray_stats[3 * rid + 2] = c_tris;
        }
        if (valid && s == SPP - 1) {
            const unsigned long long m = (SPP == 64) ? ~0ull : ((1ull << SPP) - 1ull);
            a.out[lp] = pixel_from_hits(__popcll((hits >> (pix * SPP)) & m), SPP);
        }
        // the longest packet of a chunk (cycles) orders the chunk in the next
        // frames (k_chunk_order): a chunk's packets run side by side on one
        // CU, so its longest packet is what has to start early
        if (a.chunk_cost && lane == 0)
            atomicMax(a.chunk_cost + queue.chunk,
                      (uint32_t)(__builtin_amdgcn_s_memtime() - t_start));
#if BIH_WAVE_TIMELINE
        {
            // 100 MHz real-time clock (one time base for every XCD)
            const uint64_t now = __builtin_amdgcn_s_memrealtime();
            const uint32_t dt = (uint32_t)(now - tl_pk);
            const uint64_t t_start = tl_pk;
            tl_pk = now;
            tl_last = t_start;
            ++tl_packets;
            tl_live += live ? 1u : 0u;
            if (dt > tl_max) {
                tl_max = dt;
                tl_max_at = t_start;
            }
        }
#endif
    }
#if BIH_WAVE_TIMELINE
    // debug builds: {begin, end, last packet start} u64, packets, live packets,
    // longest packet (cycles) at the wave's spill base (bih_sync prints them)
    if (lane == 0) {
        uint32_t *r = const_cast<uint32_t *>(wspill);
        const uint64_t tl_end = __builtin_amdgcn_s_memrealtime();
        const uint64_t v[3] = {tl_begin, tl_end, tl_last};
        for (int k = 0; k < 3; ++k) {
            r[2 * k] = (uint32_t)v[k];
            r[2 * k + 1] = (uint32_t)(v[k] >> 32);
        }
        r[6] = tl_packets;
        r[7] = tl_live;
        r[8] = tl_max;
        r[9] = xcc_id();
        r[10] = (uint32_t)tl_max_at;
        r[11] = (uint32_t)(tl_max_at >> 32);
    }
#endif
}

// Chunk order of the persistent packet kernel: within each of the kRegions
// bands (TileQueue::band_begin), chunks by descending cost (the cycles their
// longest packet took in an earlier frame of the same geometry), ties by index, so
// that the slow chunks start first and the frame does not end on one long
// packet (longest-processing-time-first).  One block per band sorts the
// band's keys (~cost << 32 | index: descending cost, ascending index; padded
// to a power of two with all-ones keys) bitonically in LDS.  Bands of more
// than kOrderMax chunks keep the identity order.  Only the order of the work
// changes, never a pixel.
constexpr uint32_t kOrderMax = 4096;
__global__ void __launch_bounds__(kThreads) k_chunk_order(const uint32_t *__restrict__ cost,
                                                          uint32_t chunks_x, uint32_t nchunks,
                                                          uint32_t *__restrict__ order) {
    __shared__ unsigned long long key[kOrderMax];
    const uint32_t rows = nchunks / chunks_x, b = blockIdx.x;
    const uint32_t b0 = (uint32_t)(((uint64_t)rows * b) / kRegions) * chunks_x;
    const uint32_t b1 = (uint32_t)(((uint64_t)rows * (b + 1)) / kRegions) * chunks_x;
    const uint32_t n = b1 - b0;
    if (n > kOrderMax) {
        for (uint32_t i = threadIdx.x; i < n; i += kThreads) order[b0 + i] = b0 + i;
        return;
    }
    uint32_t np = 1;
    while (np < n) np <<= 1;
    for (uint32_t i = threadIdx.x; i < np; i += kThreads)
        key[i] = i < n ? ((unsigned long long)(~cost[b0 + i]) << 32) | i : ~0ull;
    __syncthreads();
    for (uint32_t k = 2; k <= np; k <<= 1)
        for (uint32_t jj = k >> 1; jj > 0; jj >>= 1) {
            for (uint32_t i = threadIdx.x; i < np; i += kThreads) {
                const uint32_t l = i ^ jj;
                if (l > i) {
                    const unsigned long long x = key[i], y = key[l];
                    const bool up = (i & k) == 0;
                    if ((x > y) == up) {
                        key[i] = y;
                        key[l] = x;
                    }
                }
            }
            __syncthreads();
        }
    for (uint32_t i = threadIdx.x; i < n; i += kThreads) order[b0 + i] = b0 + (uint32_t)key[i];
}

// A primary ray from O can hit triangle k only if its tnum = dot(e2, q) (the
// ray-independent numerator of t, k_tri_prim) is a positive finite f32:
// t = tnum * (1/det) with 1/det > 0 finite for every lane that passes the
// det test (CUDAKernels.cu:33-47), so tnum <= 0, +inf or NaN gives t <= 0,
// inf or NaN, and the t > 0 && t < FLT_MAX test fails for every ray.
__device__ __forceinline__ bool tri_alive(const float *prim, uint32_t k) {
    return dev::tnum_alive(prim[16ull * k + 12]);
}

// Leaf k can produce a hit only if one of its triangles [first[k],
// first[k] + cnt[k]) is alive; long duplicate runs count as alive unscanned.
__global__ void __launch_bounds__(kThreads) k_leaf_alive(const float *__restrict__ prim,
                                                         const int32_t *__restrict__ first,
                                                         const uint32_t *__restrict__ cnt,
                                                         uint32_t U, uint8_t *__restrict__ alive) {
    const uint32_t k = blockIdx.x * kThreads + threadIdx.x;
    if (k >= U) return;
    const uint32_t b = (uint32_t)first[k], c = cnt[k];
    bool a = c > 64u;
    for (uint32_t i = 0; !a && i < c; ++i) a = tri_alive(prim, b + i);
    alive[k] = a ? 1 : 0;
}

// Internal node p is alive if a child is (leaf: leaf_alive; internal: this
// array).  Starts all-alive and only ever clears entries whose children are
// both dead, so any number of passes (run in place, in any order) leaves a
// conservative answer; dead subtrees of height h need h passes.
__global__ void __launch_bounds__(kThreads) k_node_alive(const uint4 *__restrict__ nodes, uint32_t m,
                                                         const uint8_t *__restrict__ leaf_alive,
                                                         uint8_t *__restrict__ node_alive) {
    const uint32_t p = blockIdx.x * kThreads + threadIdx.x;
    if (p >= m || !node_alive[p]) return;
    const uint4 nd = nodes[p];
    const uint32_t split = nd.z & 0x7ffffffu;
    const bool aL = ((nd.z >> 29) & 1u) ? leaf_alive[split] : node_alive[split];
    const bool aR = ((nd.z >> 30) & 1u) ? leaf_alive[split + 1] : node_alive[split + 1];
    if (!aL && !aR) node_alive[p] = 0;
}

// Camera-relative node records {clip0 - O[axis], clip1 - O[axis], z', w'} with
// z' = split << 8 | axis (z' >> 4: the byte offset of the children's record
// pair; the low byte is the axis alone, an s_set_gpr_idx_on index) and w' =
// the packed w (mid | cntL << 27 | cntR << 29) | leafL << 26 | leafR << 31 --
// for split < 2^24 and mid < 2^26, the scenes the packet kernels take
// (packet_records_fit) -- and the
// same records with every child subtree that no primary ray from O can
// hit (all its triangles dead, tri_alive) cut off: clip0 - O = -inf (left) /
// clip1 - O = +inf (right) make t0 = -inf*inv / t1 = +inf*inv fail the
// child's visit test (tMin < t[near], !(tMax < t[far])) for either ray
// direction, so the walk never enters it.  Only which dead subtrees are
// visited changes, so the hit set -- and the image -- is the same; the
// per-ray counters are not, and STATS launches use the exact records.
__global__ void __launch_bounds__(kThreads) k_node_prim(const uint4 *__restrict__ nodes, uint32_t m,
                                                        float ox, float oy, float oz,
                                                        const uint8_t *__restrict__ leaf_alive,
                                                        const uint8_t *__restrict__ node_alive,
                                                        uint4 *__restrict__ out,
                                                        uint4 *__restrict__ out_cull) {
    const uint32_t i = blockIdx.x * kThreads + threadIdx.x;
    if (i >= m) return;
    const uint4 nd = nodes[i];
    const uint32_t ax = (nd.z >> 27) & 3u;
    const float org = sel3(ax, ox, oy, oz);
    const uint32_t split = nd.z & 0x7ffffffu;
    const uint32_t z = (split << 8) | ax;
    const uint32_t w = nd.w | (((nd.z >> 29) & 1u) << 26) | (((nd.z >> 30) & 1u) << 31);
    uint4 r = make_uint4(__float_as_uint(__uint_as_float(nd.x) - org),
                         __float_as_uint(__uint_as_float(nd.y) - org), z, w);
    out[i] = r;
    if (!out_cull) return;   // records only (launch_prim); the culled set follows in launch_prim_cull
    const bool aL = ((nd.z >> 29) & 1u) ? leaf_alive[split] : node_alive[split];
    const bool aR = ((nd.z >> 30) & 1u) ? leaf_alive[split + 1] : node_alive[split + 1];
    if (!aL) r.x = 0xff800000u;   // -inf
    if (!aR) r.y = 0x7f800000u;   // +inf
    out_cull[i] = r;
}

// Primary-ray triangle records for the camera origin O (every primary ray of
// a frame starts at O, Camera.cu:18-20): dev::tri_prim_record per
// Morton-ordered triangle.  (Renders through the frustum bins get the same
// records from k_cam_tris, bih_bins.hip.)
__global__ void __launch_bounds__(kThreads) k_tri_prim(const float *__restrict__ tris, uint32_t n,
                                                       float ox, float oy, float oz,
                                                       float *__restrict__ prim) {
    const uint32_t i = blockIdx.x * kThreads + threadIdx.x;
    if (i >= n) return;
    (void)dev::tri_prim_record(tris + 9ull * i, ox, oy, oz, prim + 16ull * i);
}

// ---------------------------------------------------------------------------
// Shortcut boxes (the any-hit walk's shortcut passes, k_render_packet_asm):
// per internal node p a 64-byte record {box of child 0 (lo xyz, hi xyz), box
// of child 1, ref 0, ref 1, leaf 0, leaf 1}, camera-relative (box - O), each
// box an AABB of the child subtree's ALIVE triangles (tri_alive: the only
// ones that can produce a hit from O) -- set 1 tight, set 2 the miss-proof
// boxes (miss_box).  ref = internal node index, or kFastLeaf | leaf index,
// or kFastDead (no alive triangle below); leaf s = first | min(count, 63) << 26
// for a leaf child (63: read dup_cnt).  The topology is the BIH's own
// (children {split, split+1}); only the culling geometry differs.  Nothing
// here decides a pixel by itself: a hit found through these boxes is kept
// only after the exact BIH decisions are replayed along the leaf's root path
// (fast_verify); a miss only when the miss-proof walk finds no triangle the
// exact intersector accepts; every other lane runs the exact walk.
// ---------------------------------------------------------------------------
__device__ __forceinline__ void fbox_put(float *slot, const float lo[3], const float hi[3]) {
    int32_t acc = 0;
    int32_t *s = reinterpret_cast<int32_t *>(slot);
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        acc ^= atomicExch(s + c, __float_as_int(lo[c]));
        acc ^= atomicExch(s + 3 + c, __float_as_int(hi[c]));
    }
    asm volatile("" ::"v"(acc) : "memory");
}
__device__ __forceinline__ void fbox_get(float *slot, float lo[3], float hi[3]) {
    int32_t *s = reinterpret_cast<int32_t *>(slot);
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        lo[c] = __int_as_float(atomicOr(s + c, 0));
        hi[c] = __int_as_float(atomicOr(s + 3 + c, 0));
    }
}

// Miss-proof box of one alive triangle (camera-relative), from its primary-ray
// record r and dmax[] (miss_bary, bih_bound.h): the AABB of the inflated
// triangle of barycentric corners (-a, -b), (1+b+c, -b), (-a, 1+a+c), padded
// by 1e-5 + 1e-6|x| (far more than the slab test's own rounding).  If the
// exact intersector returns a hit for direction D, the line O + t D passes
// through this box.  No bound gives the unbounded box.
__device__ __forceinline__ void miss_box(const float *r, const float *dmax, float lo[3],
                                         float hi[3]) {
    const float e1[3] = {r[0], r[1], r[2]}, e2[3] = {r[3], r[4], r[5]};
    const float sv[3] = {r[6], r[7], r[8]};
    float a, bb, c;
    bool ok = miss_bary(r, dmax, a, bb, c);
    const float cu[3] = {-a, 1.0f + bb + c, -a}, cv[3] = {-bb, -bb, 1.0f + a + c};
#pragma unroll
    for (int ax = 0; ax < 3; ++ax) {
        float l = INFINITY, h = -INFINITY;
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            const float x = (cu[j] * e1[ax] + cv[j] * e2[ax]) - sv[ax];
            l = fminf(l, x);
            h = fmaxf(h, x);
        }
        lo[ax] = l - (1e-5f + 1e-6f * fabsf(l));
        hi[ax] = h + (1e-5f + 1e-6f * fabsf(h));
        ok = ok && lo[ax] > -1e30f && hi[ax] < 1e30f;
    }
    if (!ok) {
#pragma unroll
        for (int ax = 0; ax < 3; ++ax) { lo[ax] = -INFINITY; hi[ax] = INFINITY; }
    }
}

// One thread per leaf: the leaf's box of alive triangles (empty: lo = +inf,
// hi = -inf), then up the parent chain; the second arriver at a node unions
// both slots and climbs on (the same hand-off as the builder's k_fit).
__global__ void __launch_bounds__(kThreads) k_fast_fit(const float *__restrict__ tris,
                                                       const float *__restrict__ prim,
                                                       const int32_t *__restrict__ first,
                                                       const uint32_t *__restrict__ cnt,
                                                       const int32_t *__restrict__ leaf_parent,
                                                       const int32_t *__restrict__ parent,
                                                       const uint4 *__restrict__ nodes, uint32_t U,
                                                       float ox, float oy, float oz,
                                                       bool cons, float dmx, float dmy, float dmz,
                                                       uint32_t *__restrict__ arrive,
                                                       float *fast) {
    const uint32_t k = blockIdx.x * kThreads + threadIdx.x;
    if (U < 2 || k >= U) return;
    float lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
    const uint32_t b = (uint32_t)first[k], c = cnt[k];
    const float o[3] = {ox, oy, oz};
    for (uint32_t i = b; i < b + c; ++i) {
        if (!tri_alive(prim, i)) continue;
        float tlo[3], thi[3];
        if (cons) {
            const float dmax[3] = {dmx, dmy, dmz};
            miss_box(prim + 16ull * i, dmax, tlo, thi);
        } else {
            const float *t = tris + 9ull * i;
#pragma unroll
            for (int a = 0; a < 3; ++a) {
                const float v0 = t[a] - o[a], v1 = v0 + t[3 + a], v2 = v0 + t[6 + a];
                tlo[a] = fminf(v0, fminf(v1, v2));
                thi[a] = fmaxf(v0, fmaxf(v1, v2));
            }
        }
#pragma unroll
        for (int a = 0; a < 3; ++a) {
            lo[a] = fminf(lo[a], tlo[a]);
            hi[a] = fmaxf(hi[a], thi[a]);
        }
    }
    int32_t prev = (int32_t)k;
    bool prev_leaf = true;
    int32_t p = leaf_parent[k];
    while (p >= 0) {
        const uint32_t z = nodes[p].z;
        const uint32_t split = z & kIdxMask;
        const bool leafL = (z >> 29) & 1u;
        // child 0 is `split` (a leaf iff leafL), child 1 is split + 1
        const int side = ((uint32_t)prev == split && prev_leaf == leafL) ? 0 : 1;
        const int32_t pp = parent[p];
        fbox_put(fast + 16ull * p + 6 * side, lo, hi);
        if (atomicAdd(arrive + p, 1u) == 0u) return;
        float slo[3], shi[3];
        fbox_get(fast + 16ull * p + 6 * (1 - side), slo, shi);
#pragma unroll
        for (int a = 0; a < 3; ++a) { lo[a] = fminf(lo[a], slo[a]); hi[a] = fmaxf(hi[a], shi[a]); }
        prev = p;
        prev_leaf = false;
        p = pp;
    }
}

// Child refs of every record, once both boxes are in.
__global__ void __launch_bounds__(kThreads) k_fast_refs(const uint4 *__restrict__ nodes, uint32_t m,
                                                        const int32_t *__restrict__ first,
                                                        const uint32_t *__restrict__ cnt,
                                                        float *__restrict__ fast) {
    const uint32_t p = blockIdx.x * kThreads + threadIdx.x;
    if (p >= m) return;
    const uint32_t z = nodes[p].z;
    const uint32_t split = z & kIdxMask;
    float *r = fast + 16ull * p;
    uint32_t ref[2], fst[2] = {0u, 0u};
#pragma unroll
    for (int s = 0; s < 2; ++s) {
        const bool leaf = (z >> (29 + s)) & 1u;
        const bool dead = !(r[6 * s] <= r[6 * s + 3]);   // empty box (or never reached)
        ref[s] = dead ? kFastDead : leaf ? (kFastLeaf | (split + s)) : (split + s);
        if (dead)   // NaN box: every slab test of it fails
            for (int c = 0; c < 6; ++c) r[6 * s + c] = __uint_as_float(0x7fc00000u);
        if (leaf) {
            // first | count << 26 (count 63: read dup_cnt; first < 2^26 for
            // the scenes the packet kernel takes, packet_records_fit)
            const uint32_t c = cnt[split + s];
            fst[s] = (uint32_t)first[split + s] | ((c < 63u ? c : 63u) << 26);
        }
    }
    r[12] = __uint_as_float(ref[0]);
    r[13] = __uint_as_float(ref[1]);
    r[14] = __uint_as_float(fst[0]);
    r[15] = __uint_as_float(fst[1]);
}

std::mutex g_tab_mu;
uint32_t *g_tab_dev[64] = {nullptr};

enum class Variant { Packet1, Packet2, PacketAsm };

Variant variant_from_env() {
    const char *e = getenv("BIH_RENDER_KERNEL");
    if (e && strcmp(e, "packet1") == 0) return Variant::Packet1;
    if (e && strcmp(e, "packet2") == 0) return Variant::Packet2;
    return Variant::PacketAsm;
}

// The camera-relative records (k_node_prim) hold split << 8 and mid < 2^26,
// and the asm walk forms 32-bit triangle byte offsets (64 B records).
bool packet_records_fit(const RenderArgs &a) {
    return a.hdr_n_tris < (1u << 26) && a.n_nodes < (1u << 24);
}

template <int L>
hipError_t launch_persistent(Variant var, const RenderArgs &a, uint32_t traverse, hipStream_t st,
                             uint32_t blocks) {
    const bool stats = a.ray_stats != nullptr;
    const dim3 g(blocks), b(kThreads);
    if (var == Variant::Packet1 || !packet_records_fit(a)) {
        // packed canonical nodes: any scene size
        if (traverse == 0) {
            if (stats) hipLaunchKernelGGL((k_render_packet<true, true, L>), g, b, 0, st, a);
            else hipLaunchKernelGGL((k_render_packet<true, false, L>), g, b, 0, st, a);
        } else {
            if (stats) hipLaunchKernelGGL((k_render_packet<false, true, L>), g, b, 0, st, a);
            else hipLaunchKernelGGL((k_render_packet<false, false, L>), g, b, 0, st, a);
        }
    } else if (var == Variant::PacketAsm) {
        if (traverse == 0) {
            if (stats) hipLaunchKernelGGL((k_render_packet_asm<true, true, L>), g, b, 0, st, a);
            else hipLaunchKernelGGL((k_render_packet_asm<true, false, L>), g, b, 0, st, a);
        } else {
            if (stats) hipLaunchKernelGGL((k_render_packet_asm<false, true, L>), g, b, 0, st, a);
            else hipLaunchKernelGGL((k_render_packet_asm<false, false, L>), g, b, 0, st, a);
        }
    } else {
        if (traverse == 0) {
            if (stats) hipLaunchKernelGGL((k_render_packet2<true, true, L>), g, b, 0, st, a);
            else hipLaunchKernelGGL((k_render_packet2<true, false, L>), g, b, 0, st, a);
        } else {
            if (stats) hipLaunchKernelGGL((k_render_packet2<false, true, L>), g, b, 0, st, a);
            else hipLaunchKernelGGL((k_render_packet2<false, false, L>), g, b, 0, st, a);
        }
    }
    return hipGetLastError();
}

}  // namespace

int upload_rng_tables(int device) {
    if (device < 0 || device >= 64) return (int)hipErrorInvalidDevice;
    std::lock_guard<std::mutex> lk(g_tab_mu);
    if (g_tab_dev[device]) return 0;
    const size_t bytes = kRngInitWords * sizeof(uint32_t);
    uint32_t *p = nullptr;
    hipError_t e = hipMalloc((void **)&p, bytes);
    if (e != hipSuccess) return (int)e;
    e = hipMemcpy(p, xorwow_init_tables_host(), bytes, hipMemcpyHostToDevice);
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
    xorwow_skip(v, skip);   // M^skip commutes with the subsequence jumps
    const uint64_t threads = (uint64_t)nrows * ((w + 64 * kRngRun - 1) / (64 * kRngRun)) * 64;
    if (threads == 0) return 0;
    const uint32_t blocks = (uint32_t)((threads + kThreads - 1) / kThreads);
    hipLaunchKernelGGL(k_rng_init, dim3(blocks), dim3(kThreads), 0, (hipStream_t)stream, rng, w, row0,
                       nrows, band_h, band_step, v[0], v[1], v[2], v[3], v[4], tab);
    return (int)hipGetLastError();
}

int launch_stamp_init(unsigned long long *stamps, uint32_t ntiles, uint32_t frame, void *stream) {
    if (ntiles == 0) return 0;
    hipLaunchKernelGGL(k_stamp_init, dim3((ntiles + kThreads - 1) / kThreads), dim3(kThreads), 0,
                       (hipStream_t)stream, stamps, ntiles, frame);
    return (int)hipGetLastError();
}

int launch_rng_sync(unsigned long long *stamps, uint32_t *buf0, uint32_t *buf1, uint32_t *full, uint32_t w,
                    uint32_t nrows, uint32_t spp, uint32_t target, uint32_t seq, int device, void *stream) {
    const uint64_t P = (uint64_t)nrows * w;
    if (P == 0) return 0;
    const uint32_t *tab = rng_tables_device(device);
    if (!tab || spp == 0 || spp > 64 || (spp & (spp - 1))) return (int)hipErrorInvalidValue;
    const uint32_t L = (uint32_t)__builtin_ctz(spp);
    // 8 pixels per thread: 1/8 of the blocks load the 12.8 KB table
    const uint64_t blocks = (P + 8 * kThreads - 1) / (8 * kThreads);
    hipLaunchKernelGGL(k_rng_sync, dim3((uint32_t)blocks), dim3(kThreads), 0, (hipStream_t)stream, stamps, buf0, buf1,
                       full, w, nrows, L, target, seq, tab + kRngJumpOffset + L * kRngNibWords);
    return (int)hipGetLastError();
}

int launch_rng_advance(const uint32_t *src, uint32_t *dst, uint64_t pixels, uint32_t steps, int device,
                       void *stream) {
    if (pixels == 0 || (steps == 0 && src == dst)) return 0;
    const uint32_t *tab = rng_tables_device(device);
    if (!tab) return (int)hipErrorNotInitialized;
    // the two highest powers 2^7 .. 2^13 of `steps` through tables (index
    // k - 7; 7 = none), unless BIH_ADVANCE_JUMP=0 (A/B)
    static const bool jump = [] {
        const char *e = getenv("BIH_ADVANCE_JUMP");
        return !(e && e[0] == '0');
    }();
    uint32_t k0 = 7, k1 = 7, rest = steps;
    for (int k = 13; k >= 7 && jump && k1 == 7u; --k)
        if (rest >> k & 1u) {
            rest &= ~(1u << k);
            if (k0 == 7u) k0 = (uint32_t)k - 7;
            else k1 = (uint32_t)k - 7;
        }
    // with tables: up to 8 pixels per thread (fewer blocks load them), at
    // least ~2048 blocks (a rank's share of the rows is 1/8 of the frame)
    uint32_t ppt = 1;
    if (k0 < 7u)
        while (ppt < 8u && pixels > 2ull * ppt * 2048ull * kThreads) ppt *= 2;
    const uint64_t per = (uint64_t)ppt * kThreads;
    const uint32_t blocks = (uint32_t)((pixels + per - 1) / per);
    const uint32_t *jt = tab + kRngJumpOffset;
    const hipStream_t st = (hipStream_t)stream;
    if (ppt == 8)
        hipLaunchKernelGGL(k_rng_advance<8>, dim3(blocks), dim3(kThreads), 0, st, src, dst, (uint64_t)pixels, rest, jt, k0, k1);
    else if (ppt == 4)
        hipLaunchKernelGGL(k_rng_advance<4>, dim3(blocks), dim3(kThreads), 0, st, src, dst, (uint64_t)pixels, rest, jt, k0, k1);
    else if (ppt == 2)
        hipLaunchKernelGGL(k_rng_advance<2>, dim3(blocks), dim3(kThreads), 0, st, src, dst, (uint64_t)pixels, rest, jt, k0, k1);
    else
        hipLaunchKernelGGL(k_rng_advance<1>, dim3(blocks), dim3(kThreads), 0, st, src, dst, (uint64_t)pixels, rest, jt, k0, k1);
    return (int)hipGetLastError();
}

// triangle records, then the exact and the culled node records, each with
// one record of padding (the packet walk prefetches the record pair {split,
// split+1}, and split+1 may be one past the last internal node), then the
// leaf and node alive bytes
size_t alive_bytes(uint32_t m) { return ((size_t)(m + 1) + m + 15) & ~(size_t)15; }
size_t prim_bytes(uint32_t n, uint32_t m) {
    return (size_t)n * 64 + 2 * (size_t)(m + 1) * 16 + alive_bytes(m) +
           2 * (size_t)(m + 1) * 64 + (size_t)m * 4;
}
size_t fast_offset(uint32_t n, uint32_t m) {
    return (size_t)n * 64 + 2 * (size_t)(m + 1) * 16 + alive_bytes(m);
}

int launch_prim(const float *tris, uint32_t n, const uint4 *nodes, const int32_t *first_idx,
                const uint32_t *dup_cnt, const int32_t *leaf_parent, const int32_t *parent,
                uint32_t m, const float origin[3], const float dmax[3], float *prim,
                void *stream) {
    const hipStream_t st = (hipStream_t)stream;
    if (n > 0)
        hipLaunchKernelGGL(k_tri_prim, dim3((n + kThreads - 1) / kThreads), dim3(kThreads), 0, st,
                           tris, n, origin[0], origin[1], origin[2], prim);
    if (m > 0) {
        uint4 *rec = reinterpret_cast<uint4 *>(prim + 16ull * n);
        const dim3 gn((m + kThreads - 1) / kThreads);
        hipLaunchKernelGGL(k_node_prim, gn, dim3(kThreads), 0, st, nodes, m, origin[0], origin[1],
                           origin[2], nullptr, nullptr, rec, nullptr);
    }
    return (int)hipGetLastError();
}

// The culled node records (node_cull) for the records launch_prim wrote:
// only the BIH walk kernels read them, so renders through the frustum bins
// never pay for them (bih_capi.cpp builds them on first use per camera).
int launch_prim_cull(uint32_t n, const uint4 *nodes, const int32_t *first_idx, const uint32_t *dup_cnt,
                     uint32_t m, const float origin[3], float *prim, void *stream) {
    const hipStream_t st = (hipStream_t)stream;
    if (m > 0) {
        uint4 *rec = reinterpret_cast<uint4 *>(prim + 16ull * n);
        uint8_t *leaf_alive = reinterpret_cast<uint8_t *>(rec + 2 * (size_t)(m + 1));
        uint8_t *node_alive = leaf_alive + (m + 1);
        const dim3 gl((m + 1 + kThreads - 1) / kThreads), gn((m + kThreads - 1) / kThreads);
        hipLaunchKernelGGL(k_leaf_alive, gl, dim3(kThreads), 0, st, prim, first_idx, dup_cnt, m + 1,
                           leaf_alive);
        hipError_t e = hipMemsetAsync(node_alive, 1, m, st);
        if (e != hipSuccess) return (int)e;
        // dead subtrees of a random soup are a few levels high (1M triangles:
        // 12 % of the nodes, every one found within 7 passes)
        for (int pass = 0; pass < 8; ++pass)
            hipLaunchKernelGGL(k_node_alive, gn, dim3(kThreads), 0, st, nodes, m, leaf_alive,
                               node_alive);
        hipLaunchKernelGGL(k_node_prim, gn, dim3(kThreads), 0, st, nodes, m, origin[0], origin[1],
                           origin[2], leaf_alive, node_alive, rec, rec + (m + 1));
    }
    return (int)hipGetLastError();
}

// The any-hit BIH walk's shortcut boxes for the records launch_prim wrote
// (only renders without frustum bins read them).
int launch_fast_boxes(const float *tris, uint32_t n, const uint4 *nodes, const int32_t *first_idx,
                      const uint32_t *dup_cnt, const int32_t *leaf_parent, const int32_t *parent,
                      uint32_t m, const float origin[3], const float dmax[3], float *prim, void *stream) {
    const hipStream_t st = (hipStream_t)stream;
    if (m > 0) {
        const dim3 gl((m + 1 + kThreads - 1) / kThreads), gn((m + kThreads - 1) / kThreads);
        hipError_t e = hipSuccess;
        // shortcut boxes of the any-hit walk: tight (pass 1), miss-proof (pass 2)
        float *fast = reinterpret_cast<float *>(reinterpret_cast<char *>(prim) + fast_offset(n, m));
        uint32_t *arrive = reinterpret_cast<uint32_t *>(fast + 2 * 16ull * (m + 1));
        for (int pass = 0; pass < 2; ++pass) {
            float *boxes = fast + pass * 16ull * (m + 1);
            e = hipMemsetAsync(arrive, 0, sizeof(uint32_t) * m, st);
            if (e != hipSuccess) return (int)e;
            hipLaunchKernelGGL(k_fast_fit, gl, dim3(kThreads), 0, st, tris, prim, first_idx,
                               dup_cnt, leaf_parent, parent, nodes, m + 1, origin[0], origin[1],
                               origin[2], pass == 1, dmax[0], dmax[1], dmax[2], arrive, boxes);
            hipLaunchKernelGGL(k_fast_refs, gn, dim3(kThreads), 0, st, nodes, m, first_idx, dup_cnt,
                               boxes);
        }
    }
    return (int)hipGetLastError();
}

bool render_uses_prim(uint32_t spp) {
    return spp <= 64 && (spp & (spp - 1)) == 0;
}

// Resident blocks of the persistent kernels on `device` (grid size).
uint32_t wave_grid_blocks(int device) {
    static std::mutex mu;
    static uint32_t cache[64] = {0};
    std::lock_guard<std::mutex> lk(mu);
    if (device < 0 || device >= 64) return 0;
    if (!cache[device]) {
        // resident blocks per CU: the largest over the persistent kernels
        // (the LDS-stack kernels fit fewer than the register-stack packet ones)
        const void *kernels[] = {
            reinterpret_cast<const void *>(k_render_packet<true, false, 2>),
            reinterpret_cast<const void *>(k_render_packet2<true, false, 2>),
            reinterpret_cast<const void *>(k_render_packet_asm<true, false, 2>),
        };
        int cus = 0, per = 0;
        (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device);
        for (const void *k : kernels) {
            int p = 0;
            (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&p, k, kThreads, 0);
            if (p > per) per = p;
        }
        if (cus <= 0) cus = 256;
        if (per <= 0) per = 1;
        // tuning knob: resident blocks per CU (the occupancy API's answer otherwise)
        if (const char *e = getenv("BIH_BLOCKS_PER_CU")) {
            const int v = atoi(e);
            if (v > 0 && v <= 32) per = v;
        }
        cache[device] = (uint32_t)(cus * per);
    }
    return cache[device];
}

size_t spill_words(uint32_t blocks) {
    // per block: per-lane kernels [(32-kLdsStack)*3][256 lanes]; packet kernel
    // 4 waves x [(32-kPacketRegs)*3][64 lanes] -- size for the larger
    const size_t lane_k = (size_t)kThreads * (kStackDepth - kLdsStack) * 3;
    const size_t packet_k = (size_t)(kThreads / 64) * (kStackDepth - kPacketRegs) * 3 * 64;
    return (size_t)blocks * (lane_k > packet_k ? lane_k : packet_k);
}

uint32_t chunk_count(uint32_t w, uint32_t nrows, uint32_t spp, uint32_t *chunks_x) {
    if (spp == 0 || spp > 64 || (spp & (spp - 1)) != 0) return 0;
    const int L = __builtin_ctz(spp);
    const uint32_t pix = 64u >> L;
    const uint32_t tw = 1u << ((6 - L + 1) / 2), th = pix / tw;
    const uint32_t tiles_x = (w + tw - 1) / tw, tiles_y = (nrows + th - 1) / th;
    const uint32_t cx = (tiles_x + kChunkW - 1) / kChunkW;
    if (chunks_x) *chunks_x = cx;
    return cx * ((tiles_y + kChunkH - 1) / kChunkH);
}

int launch_chunk_order(const uint32_t *cost, uint32_t chunks_x, uint32_t nchunks, uint32_t *order,
                       void *stream) {
    if (nchunks == 0) return 0;
    hipLaunchKernelGGL(k_chunk_order, dim3(kRegions), dim3(kThreads), 0, (hipStream_t)stream, cost,
                       chunks_x, nchunks, order);
    return (int)hipGetLastError();
}

// Resident blocks of k_render_bins on `device` (its own occupancy: the list
// walk needs fewer registers than the BIH walks).  A launch of several
// frames takes fewer than the occupancy allows (kBinsMultiPerCU per CU): the
// calls in flight then overlap -- the next call's advance and first waves
// run in the free slots while this one drains (1080p headline, blocks per CU
// of 16-frame launches: 6 (all) 0.0420 ms per frame, 5 0.0419, 4 0.0399, 3
// 0.0397, 2 0.0400; r04zk/zl).  Only while another render is in flight
// (RenderArgs::shared_grid, from the other slots' events): a lone 16-frame
// launch is slower with fewer waves (4: 0.0494 ms per frame against 0.0454
// with all 6), so it takes every slot.  One-frame launches keep every slot
// (4 per CU: 0.087 -> 0.093 ms alone).
#ifndef BIH_BINS_MULTI_PER_CU
#define BIH_BINS_MULTI_PER_CU 4
#endif
uint32_t bins_grid_blocks(int device, uint32_t nframes, bool stamped) {
    static std::mutex mu;
    static uint32_t cache[64][2][2] = {{{0}}};
    std::lock_guard<std::mutex> lk(mu);
    if (device < 0 || device >= 64) return 0;
    if (!cache[device][stamped][0]) {
        int cus = 0, per = 0;
        (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device);
        (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(
            &per, stamped ? reinterpret_cast<const void *>(k_render_bins<2, kBinsStamped>)
                          : reinterpret_cast<const void *>(k_render_bins<2, 0>), kThreads, 0);
        if (cus <= 0) cus = 256;
        if (per <= 0) per = 1;
        int multi = BIH_BINS_MULTI_PER_CU < per ? BIH_BINS_MULTI_PER_CU : per;
        if (const char *e = getenv("BIH_BINS_BLOCKS_PER_CU")) {
            const int v = atoi(e);
            if (v > 0 && v <= 32) per = v;
        }
        if (const char *e = getenv("BIH_BINS_MULTI_PER_CU")) {
            const int v = atoi(e);
            if (v > 0 && v <= 32) multi = v;
        }
        cache[device][stamped][0] = (uint32_t)(cus * per);
        cache[device][stamped][1] = (uint32_t)(cus * multi);
    }
    return cache[device][stamped][nframes > 1 ? 1 : 0];
}

template <int L>
static hipError_t launch_bins(const RenderArgs &a, hipStream_t st, uint32_t blocks, uint32_t fb_blocks,
                              hipEvent_t k0, hipEvent_t k1) {
    hipError_t e = k0 ? hipEventRecord(k0, st) : hipSuccess;
    if (e != hipSuccess) return e;
    if (a.hit_mask)
        hipLaunchKernelGGL((k_render_bins<L, 1>), dim3(blocks), dim3(kThreads), 0, st, a);
    else if (a.bin_cost && a.stamps)
        hipLaunchKernelGGL((k_render_bins<L, 2 | kBinsStamped>), dim3(blocks), dim3(kThreads), 0, st, a);
    else if (a.bin_cost)
        hipLaunchKernelGGL((k_render_bins<L, 2>), dim3(blocks), dim3(kThreads), 0, st, a);
    else if (a.stamps)
        hipLaunchKernelGGL((k_render_bins<L, kBinsStamped>), dim3(blocks), dim3(kThreads), 0, st, a);
    else
        hipLaunchKernelGGL((k_render_bins<L, 0>), dim3(blocks), dim3(kThreads), 0, st, a);
    e = k1 ? hipEventRecord(k1, st) : hipSuccess;
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_render_fallback<L>, dim3(fb_blocks), dim3(kThreads), 0, st, a);
    return hipGetLastError();
}

// Diagnostic builds (BIH_BINS_TIMELINE): appends the per-item records of the
// k_render_bins launches since the last dump to `path` (raw uint4s) and
// resets the count.  Returns the number of records, or -1.
long bins_timeline_dump(const char *path) {
#if BIH_BINS_TIMELINE
    if (hipDeviceSynchronize() != hipSuccess) return -1;
    std::vector<uint32_t> cnt(kTlWaves);
    std::vector<uint4> rec((size_t)kTlWaves * kTlPerWave);
    if (hipMemcpyFromSymbol(cnt.data(), HIP_SYMBOL(g_tl_n), kTlWaves * 4) != hipSuccess) return -1;
    if (hipMemcpyFromSymbol(rec.data(), HIP_SYMBOL(g_tl_rec), rec.size() * sizeof(uint4)) != hipSuccess) return -1;
    std::vector<uint32_t> zero(kTlWaves, 0u);
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_tl_n), zero.data(), kTlWaves * 4) != hipSuccess) return -1;
    std::vector<uint4> out;
    uint32_t lost = 0;
    for (uint32_t w = 0; w < kTlWaves; ++w) {
        const uint32_t n = cnt[w] < kTlPerWave ? cnt[w] : kTlPerWave;
        lost += cnt[w] - n;
        for (uint32_t k = 0; k < n; ++k) out.push_back(rec[(size_t)w * kTlPerWave + k]);
    }
    if (FILE *f = fopen(path, "ab")) {
        const uint32_t hdr[4] = {0x544C4942u, (uint32_t)out.size(), lost, 0u};   // "BILT", count, dropped
        fwrite(hdr, sizeof hdr, 1, f);
        if (!out.empty()) fwrite(out.data(), sizeof(uint4), out.size(), f);
        fclose(f);
    }
    return (long)out.size();
#else
    (void)path;
    return -1;
#endif
}

int launch_render(const RenderArgs &a, uint32_t traverse, void *stream, void *ev_k0, void *ev_k1) {
    hipStream_t st = (hipStream_t)stream;
    const hipEvent_t k0 = (hipEvent_t)ev_k0, k1 = (hipEvent_t)ev_k1;
    const uint32_t spp = a.spp;
    int dev = 0;
    (void)hipGetDevice(&dev);
    const uint32_t grid = wave_grid_blocks(dev);
    if (a.bin_queue && spp <= 64 && (spp & (spp - 1)) == 0) {
        // frustum bins: the list-walk kernel, then the exact walk for what it
        // left undecided (the fallback grid stays within the spill area)
        const uint32_t fb = grid < 64u ? grid : 64u;
        const uint32_t gb = bins_grid_blocks(dev, a.shared_grid ? 2u : 1u, a.stamps != nullptr);
        if (BIH_FAST_COUNTERS || BIH_PHASES) {
            const hipError_t e = hipMemsetAsync(a.work, 0, kWorkWords * sizeof(uint32_t), st);
            if (e != hipSuccess) return (int)e;
        }
        switch (__builtin_ctz(spp)) {
        case 0: return (int)launch_bins<0>(a, st, gb, fb, k0, k1);
        case 1: return (int)launch_bins<1>(a, st, gb, fb, k0, k1);
        case 2: return (int)launch_bins<2>(a, st, gb, fb, k0, k1);
        case 3: return (int)launch_bins<3>(a, st, gb, fb, k0, k1);
        case 4: return (int)launch_bins<4>(a, st, gb, fb, k0, k1);
        case 5: return (int)launch_bins<5>(a, st, gb, fb, k0, k1);
        default: return (int)launch_bins<6>(a, st, gb, fb, k0, k1);
        }
    }
    if (spp <= 64 && (spp & (spp - 1)) == 0) {
        static const Variant var = variant_from_env();
        const int L = __builtin_ctz(spp);
        const uint32_t pix = 64u >> L;
        const uint32_t tw = 1u << ((6 - L + 1) / 2), th = pix / tw;
        const uint64_t tiles = (uint64_t)((a.w + tw - 1) / tw) * ((a.nrows + th - 1) / th);
        if (tiles == 0) return 0;
        uint32_t blocks = (uint32_t)((tiles + 3) / 4);
        if (blocks > grid) blocks = grid;
        // the tile queue of the per-CU slots starts from zero; the bins' item
        // queue resets itself (counter builds also count into a.work)
        hipError_t e = hipMemsetAsync(a.work, 0, kWorkWords * sizeof(uint32_t), st);
        if (e == hipSuccess && k0) e = hipEventRecord(k0, st);
        if (e != hipSuccess) return (int)e;
        switch (L) {
        case 0: e = launch_persistent<0>(var, a, traverse, st, blocks); break;
        case 1: e = launch_persistent<1>(var, a, traverse, st, blocks); break;
        case 2: e = launch_persistent<2>(var, a, traverse, st, blocks); break;
        case 3: e = launch_persistent<3>(var, a, traverse, st, blocks); break;
        case 4: e = launch_persistent<4>(var, a, traverse, st, blocks); break;
        case 5: e = launch_persistent<5>(var, a, traverse, st, blocks); break;
        default: e = launch_persistent<6>(var, a, traverse, st, blocks); break;
        }
        if (e == hipSuccess && k1) e = hipEventRecord(k1, st);
        return (int)e;
    }
    // any other spp: one lane per pixel, grid-stride, grid capped at the spill area
    const uint32_t tiles = ((a.w + 7) >> 3) * ((a.nrows + 7) >> 3);
    if (tiles == 0) return 0;
    uint32_t blocks = (tiles + 3) / 4;
    if (blocks > grid) blocks = grid;
    const bool stats = a.ray_stats != nullptr;
    if (k0) (void)hipEventRecord(k0, st);
    if (traverse == 0) {
        if (stats) hipLaunchKernelGGL((k_render_pixel<true, true>), dim3(blocks), dim3(kThreads), 0, st, a);
        else hipLaunchKernelGGL((k_render_pixel<true, false>), dim3(blocks), dim3(kThreads), 0, st, a);
    } else {
        if (stats) hipLaunchKernelGGL((k_render_pixel<false, true>), dim3(blocks), dim3(kThreads), 0, st, a);
        else hipLaunchKernelGGL((k_render_pixel<false, false>), dim3(blocks), dim3(kThreads), 0, st, a);
    }
    if (k1) (void)hipEventRecord(k1, st);
    return (int)hipGetLastError();
}

}  // namespace bih
