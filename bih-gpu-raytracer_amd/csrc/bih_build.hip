// bih_build.hip -- per-frame BIH builder for gfx950 (MI355X).
//
// Replaces Renderer::Render steps 1-7 (reference src/Renderer.cpp:422-503):
//   k_prep        per-triangle AABB + scene AABB        (App.cpp:103-142)
//   k_morton      normalised centroid -> 30-bit Morton  (App.cpp:144-156,
//                                                       Renderer.cpp:114-145)
//   radix sort    stable LSD sort of (code, tri idx)    (Renderer.cpp:441-445)
//   k_runs*       reduce_by_key + unique_by_key_copy    (Renderer.cpp:450-472)
//   k_karras      Karras-2012 internal nodes            (CUDAKernels.cu:591-710)
//   k_seg_build   leaf boxes + sorted {v0,e1,e2} triangles + segment tree
//   k_fit         clip planes as range queries over the segment tree of the
//                 leaf boxes instead of the leaf->root atomics of
//                 FindClipPlanes (CUDAKernels.cu:497-549): same max/min, no
//                 atomics; and the 16-B render nodes
// Everything is integer/byte work or exact f32 compares; all arithmetic is
// compiled with -ffp-contract=off so it matches the strict-IEEE oracle.
#include <hip/hip_runtime.h>

#include <atomic>
#include <stdlib.h>
#include <utility>
#include <float.h>

#include "bih_internal.h"
#include "bih_device.h"

namespace bih {
namespace {

constexpr int kThreads = 256;
constexpr int kScanItems = 8;
constexpr int kScanTile = kThreads * kScanItems;     // 2048
constexpr int kRsItems = 16;
constexpr int kRsTile = kThreads * kRsItems;          // 4096
constexpr uint32_t kPrepBlocks = 1024;                // k_prep grid (partials per block)

__device__ __forceinline__ int clz32(uint32_t x) { return x ? __clz((int)x) : 32; }

// IEEE totalOrder key (-0 < +0): the order atomicMaxFloat/atomicMinFloat
// implement (CUDAKernels.cu:52-66).
__device__ __forceinline__ int32_t tkey(float f) {
    uint32_t u = __float_as_uint(f);
    return (u & 0x80000000u) ? ((int32_t)(~u) ^ (int32_t)0x80000000) : (int32_t)u;
}
__device__ __forceinline__ float tmax(float a, float b) { return tkey(b) > tkey(a) ? b : a; }
__device__ __forceinline__ float tmin(float a, float b) { return tkey(b) < tkey(a) ? b : a; }

// Monotone u32 key with +-0 merged: the `<` that std::minmax uses.
__device__ __forceinline__ uint32_t lt_key(float f) {
    uint32_t u = __float_as_uint(f);
    if ((u & 0x7fffffffu) == 0u) u = 0u;
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

// ---------------------------------------------------------------------------
// Hash of the input soup: two XOR-sums of murmur3 finalisers of (word, index)
// (32-bit arithmetic), accumulated by k_prep as it reads the soup and folded
// by k_morton's blocks (prep_fold).  The build is a deterministic function of the soup, so an
// unchanged hash after a rebuild means an unchanged tree, and the per-camera
// structures derived from it (bih_capi.cpp finish_build) stay valid.
__device__ __forceinline__ uint32_t fmix32(uint32_t h) {
    h ^= h >> 16;
    h *= 0x85ebca6bu;
    h ^= h >> 13;
    h *= 0xc2b2ae35u;
    h ^= h >> 16;
    return h;
}
__device__ __forceinline__ void content_word(uint32_t w, uint32_t i, uint32_t &x, uint32_t &y) {
    x ^= fmix32(w ^ (i * 0x9E3779B1u));
    y ^= fmix32((w + 0x165667B1u) ^ fmix32(i + 0x27D4EB2Fu));
}

// Triangle AABB on one axis with std::minmax's rules (App.cpp:103-142):
// leftmost min, rightmost max (k_prep; k_seg_leaf recomputes it bit-equal).
__device__ __forceinline__ void axis_minmax(float x0, float x1, float x2, float &m, float &M) {
    m = x0; if (x1 < m) m = x1; if (x2 < m) m = x2;
    M = x0; if (!(x1 < M)) M = x1; if (!(x2 < M)) M = x2;
}

// k_prep: lo/hi per triangle (std::minmax: leftmost min, rightmost max) and
// the scene AABB.  The reference folds triangles sequentially with
// std::minmax({lo, hi, sceneLo, sceneHi}) (App.cpp:133-137), so sceneLo ends
// as the lo of the LAST triangle attaining the minimum and sceneHi as the hi
// of the FIRST triangle attaining the maximum (or the seed vertex if it ties).
// Ties only differ in the sign of zero; we reduce (value, index) keys.
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(kThreads) k_prep(const float *__restrict__ v, uint32_t n,
                                                   float *__restrict__ lo, float *__restrict__ hi,
                                                   TreeHeader *hdr,
                                                   unsigned long long *__restrict__ part,
                                                   uint32_t *__restrict__ epoch) {
    // the build's sequence number (scan_tag: the look-back tags of this
    // build's scans); the kernels that read it run after this one
    if (blockIdx.x == 0 && threadIdx.x == 0) *epoch += 1u;
    unsigned long long kmin[3] = {~0ull, ~0ull, ~0ull}, kmax[3] = {0ull, 0ull, 0ull};
    uint32_t bad = 0;
    uint32_t hx = 0u, hy = 0u;   // content hash (content_word): XOR of every word's term
    for (uint32_t i = blockIdx.x * kThreads + threadIdx.x; i < n; i += gridDim.x * kThreads) {
        const float *p = v + 9ull * i;
        float q[9];
#pragma unroll
        for (int k = 0; k < 9; ++k) q[k] = p[k];
#pragma unroll
        for (int k = 0; k < 9; ++k) content_word(__float_as_uint(q[k]), 9u * i + (uint32_t)k, hx, hy);
#pragma unroll
        for (int a = 0; a < 3; ++a) {
            float x0 = q[a], x1 = q[3 + a], x2 = q[6 + a];
            bad |= (uint32_t)!isfinite(x0) | (uint32_t)!isfinite(x1) | (uint32_t)!isfinite(x2);
            float m, M;
            axis_minmax(x0, x1, x2, m, M);
            lo[3ull * i + a] = m;
            hi[3ull * i + a] = M;
            unsigned long long tie = 0xFFFFFFFFull - i;
            unsigned long long km = ((unsigned long long)lt_key(m) << 32) | tie;
            unsigned long long kM = ((unsigned long long)lt_key(M) << 32) | tie;
            kmin[a] = km < kmin[a] ? km : kmin[a];   // smallest value, ties -> largest i
            kmax[a] = kM > kmax[a] ? kM : kmax[a];   // largest value, ties -> smallest i
        }
    }
    // wave reduce, block reduce through LDS, one partial per block (the
    // blocks of k_morton fold them: no contended atomics)
    __shared__ unsigned long long s_key[7][kThreads / 64];
    __shared__ uint32_t s_bad[kThreads / 64];
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        for (int off = 32; off > 0; off >>= 1) {
            unsigned long long om = __shfl_xor(kmin[a], off);
            unsigned long long oM = __shfl_xor(kmax[a], off);
            kmin[a] = om < kmin[a] ? om : kmin[a];
            kmax[a] = oM > kmax[a] ? oM : kmax[a];
        }
    }
    for (int off = 32; off > 0; off >>= 1) {
        hx ^= __shfl_xor(hx, off);
        hy ^= __shfl_xor(hy, off);
    }
    const unsigned long long anybad = __ballot(bad);
    const uint32_t wv = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) {
#pragma unroll
        for (int a = 0; a < 3; ++a) {
            s_key[a][wv] = kmin[a];
            s_key[3 + a][wv] = kmax[a];
        }
        s_key[6][wv] = ((unsigned long long)hy << 32) | hx;
        s_bad[wv] = anybad ? 1u : 0u;
    }
    __syncthreads();
    if (threadIdx.x < 7) {
        const int a = threadIdx.x;
        unsigned long long r = s_key[a][0];
        for (uint32_t w = 1; w < kThreads / 64; ++w) {
            const unsigned long long o = s_key[a][w];
            r = (a == 6) ? (r ^ o) : (a < 3) ? (o < r ? o : r) : (o > r ? o : r);
        }
        part[(size_t)a * gridDim.x + blockIdx.x] = r;
    }
    if (threadIdx.x == 7) {   // non-finite coordinates in this block (folded by prep_fold)
        uint32_t b = 0;
        for (uint32_t w = 0; w < kThreads / 64; ++w) b |= s_bad[w];
        part[(size_t)7 * gridDim.x + blockIdx.x] = b;
    }
}

__global__ void k_hdr_init(TreeHeader *hdr, uint32_t n) {
    int a = threadIdx.x;
    if (a < 3) {
        hdr->scene_lo[a] = 0.f;
        hdr->scene_hi[a] = 0.f;
        hdr->lo_key[a] = ~0ull;
        hdr->hi_key[a] = 0ull;
    }
    if (a == 0) {
        hdr->n_tris = n;
        hdr->n_unique = 0;
        hdr->nonfinite = 0;
        hdr->pad0 = 0;
        hdr->content = 0ull;
    }
}


// The fold of k_prep's per-block partials: the scene AABB with the
// reference's tie rules, the content hash, the non-finite flag.  Every block
// of k_morton folds them for itself (1024 threads: one partial per thread
// and array) into slo / shi, and block 0 writes the header -- no launch of
// its own (round 3's k_prep_final: one block, 0.012 ms).
template <uint32_t NT>
__device__ void prep_fold(const float *__restrict__ v, const float *__restrict__ lo, const float *__restrict__ hi,
                          TreeHeader *hdr, uint32_t n, const unsigned long long *__restrict__ part,
                          uint32_t nparts, float slo[3], float shi[3]) {
    constexpr uint32_t NW = NT / 64;
    __shared__ unsigned long long s_red[8][NW];
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
    for (int a = 0; a < 6; ++a) {
        unsigned long long r = a < 3 ? ~0ull : 0ull;
        for (uint32_t i = threadIdx.x; i < nparts; i += NT) {
            const unsigned long long o = part[(size_t)a * nparts + i];
            r = (a < 3) ? (o < r ? o : r) : (o > r ? o : r);
        }
        for (int off = 32; off > 0; off >>= 1) {
            const unsigned long long o = __shfl_xor(r, off);
            r = (a < 3) ? (o < r ? o : r) : (o > r ? o : r);
        }
        if (lane == 0) s_red[a][wv] = r;
    }
    {   // the content hash: XOR of the blocks' partials; non-finite flags
        unsigned long long hxy = 0ull, b = 0ull;
        for (uint32_t i = threadIdx.x; i < nparts; i += NT) {
            hxy ^= part[(size_t)6 * nparts + i];
            b |= part[(size_t)7 * nparts + i];
        }
        for (int off = 32; off > 0; off >>= 1) {
            hxy ^= __shfl_xor(hxy, off);
            b |= __shfl_xor(b, off);
        }
        if (lane == 0) {
            s_red[6][wv] = hxy;
            s_red[7][wv] = b;
        }
    }
    __syncthreads();
    if (threadIdx.x == 0 && blockIdx.x == 0) {
        unsigned long long hxy = 0ull, bad = 0ull;
        for (uint32_t w = 0; w < NW; ++w) {
            hxy ^= s_red[6][w];
            bad |= s_red[7][w];
        }
        hdr->content = hxy;
        hdr->nonfinite = bad ? 1u : 0u;
        hdr->n_unique = 0;
        hdr->pad0 = 0;
        hdr->n_tris = n;
    }
    const int a = threadIdx.x;
    if (a < 3) {
        unsigned long long kmin = s_red[a][0], kmax = s_red[3 + a][0];
        for (uint32_t w = 1; w < NW; ++w) {
            kmin = s_red[a][w] < kmin ? s_red[a][w] : kmin;
            kmax = s_red[3 + a][w] > kmax ? s_red[3 + a][w] : kmax;
        }
        const uint32_t ilo = 0xFFFFFFFFu - (uint32_t)(kmin & 0xFFFFFFFFull);
        const uint32_t ihi = 0xFFFFFFFFu - (uint32_t)(kmax & 0xFFFFFFFFull);
        const float mx = hi[3ull * ihi + a];
        const float seed = v[a];                   // first vertex (App.cpp:103-106)
        slo[a] = lo[3ull * ilo + a];
        shi[a] = (seed < mx) ? mx : seed;
        if (blockIdx.x == 0) {
            hdr->lo_key[a] = kmin;
            hdr->hi_key[a] = kmax;
            hdr->scene_lo[a] = slo[a];
            hdr->scene_hi[a] = shi[a];
        }
    }
    __syncthreads();
}

// ---------------------------------------------------------------------------
// k_morton: centre (App.cpp:128-131), normalise (:144-156), morton3D
// (Renderer.cpp:127-136).  Writes (code, index) pairs for the sort.
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint32_t expand_bits(uint32_t v) {
    v = (v * 0x00010001u) & 0xFF0000FFu;
    v = (v * 0x00000101u) & 0x0F00F00Fu;
    v = (v * 0x00000011u) & 0xC30C30C3u;
    v = (v * 0x00000005u) & 0x49249249u;
    return v;
}

__device__ __forceinline__ uint32_t morton_code(const float *__restrict__ lo, const float *__restrict__ hi,
                                                const float slo[3], const float shi[3], uint32_t i) {
    float q[3];
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        float c = (lo[3ull * i + a] + hi[3ull * i + a]) / 2.0f;
        float num = c - slo[a];
        float den = shi[a] - slo[a];
        float x = (num / den) * 1024.0f;
        q[a] = fminf(fmaxf(x, 0.0f), 1023.0f);
    }
    return expand_bits((uint32_t)q[0]) * 4 + expand_bits((uint32_t)q[1]) * 2 + expand_bits((uint32_t)q[2]);
}

// Radix sort digits: 3 passes of 10 bits cover the 30-bit codes.
constexpr int kRdBits = 10;
constexpr uint32_t kRdBins = 1u << kRdBits;
constexpr int kRdPasses = 3;

// Block b's tile [b kRsTile, (b+1) kRsTile): codes and indices, and the tile's
// counts of the first digit (hist[digit * nblocks + b], k_rs_scatter10's
// layout) -- the first pass's histogram without a pass of its own.
// A block of kRsBlock threads per tile: kRsTile / kRsBlock codes per thread.
constexpr int kRsBlock = 1024;
constexpr int kRsWaves = kRsBlock / 64;
constexpr int kRsPer = kRsTile / kRsBlock;            // 4
__global__ void __launch_bounds__(kRsBlock) k_morton(const float *__restrict__ v,
                                                     const float *__restrict__ lo,
                                                     const float *__restrict__ hi,
                                                     TreeHeader *__restrict__ hdr, uint32_t n,
                                                     const unsigned long long *__restrict__ part, uint32_t nparts,
                                                     uint32_t *__restrict__ keys,
                                                     uint32_t *__restrict__ vals,
                                                     uint32_t *__restrict__ hist, uint32_t nblocks) {
    __shared__ uint32_t h[kRdBins];
    __shared__ float s_lo[3], s_hi[3];
    for (uint32_t k = threadIdx.x; k < kRdBins; k += kRsBlock) h[k] = 0u;
    prep_fold<kRsBlock>(v, lo, hi, hdr, n, part, nparts, s_lo, s_hi);   // (ends with a barrier)
    const float slo[3] = {s_lo[0], s_lo[1], s_lo[2]}, shi[3] = {s_hi[0], s_hi[1], s_hi[2]};
    const uint64_t base = (uint64_t)blockIdx.x * kRsTile;
#pragma unroll
    for (int r = 0; r < kRsPer; ++r) {
        const uint64_t i = base + (uint64_t)r * kRsBlock + threadIdx.x;
        if (i < n) {
            const uint32_t key = morton_code(lo, hi, slo, shi, (uint32_t)i);
            keys[i] = key;
            vals[i] = (uint32_t)i;
            atomicAdd(&h[key & (kRdBins - 1u)], 1u);
        }
    }
    __syncthreads();
    for (uint32_t k = threadIdx.x; k < kRdBins; k += kRsBlock) hist[(uint64_t)k * nblocks + blockIdx.x] = h[k];
}

// ---------------------------------------------------------------------------
// Device-wide exclusive scan of u32 (one launch, decoupled look-back).
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint32_t block_exclusive_scan(uint32_t x, uint32_t *lds, uint32_t *total) {
    // 256 threads = 4 waves
    int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint32_t inc = x;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        uint32_t y = __shfl_up(inc, off);
        if (lane >= off) inc += y;
    }
    if (lane == 63) lds[wave] = inc;
    __syncthreads();
    uint32_t wbase = 0, tot = 0;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
        uint32_t s = lds[w];
        wbase += (w < wave) ? s : 0u;
        tot += s;
    }
    __syncthreads();
    *total = tot;
    return wbase + inc - x;
}

// Single-pass scan with decoupled look-back: tile t publishes its aggregate,
// adds its predecessors' published values walking back until one carries an
// inclusive prefix, then publishes its own inclusive prefix.  A status word is
// {tag:30 | flag:2 | value:32}, flag 1 = aggregate, 2 = inclusive prefix; the
// tag is unique per scan call (host counter), so no status memset is needed
// between calls.  Tiles are blockIdx.x: workgroups dispatch in id order, so
// every tile a block waits for is resident or done.  The flag and the value
// share one 64-bit word, so relaxed device-scope atomics suffice (no L2
// writeback/invalidate fences: each block's output is its own).
// Look-back tag of scan k (1..7) of the build whose sequence number k_prep
// wrote (DeviceTree::epoch): unique per build and scan, non-zero, and the same
// in every replay of a captured build graph's node -- the tag a node was
// captured with is not (next_scan_tag is a host counter).  The build's status
// words (DeviceTree::partials) only ever hold such tags.
__device__ __forceinline__ uint32_t scan_tag(const uint32_t *epoch, uint32_t k) {
    return epoch ? ((*epoch * 8u + k) & 0x3FFFFFFFu) : k;
}

__global__ void __launch_bounds__(kThreads) k_scan_onepass(const uint32_t *in, uint32_t *out, uint32_t n,
                                                           unsigned long long *status, uint32_t tag,
                                                           uint32_t *total_out, const uint32_t *epoch) {
    __shared__ uint32_t lds[4];
    tag = scan_tag(epoch, tag);
    __shared__ uint32_t s_prefix;
    const uint32_t tile = blockIdx.x;
    const uint64_t base = (uint64_t)tile * kScanTile + (uint64_t)threadIdx.x * kScanItems;
    uint32_t x[kScanItems];
    uint32_t sum = 0;
    // 16-byte loads and stores when the whole run of 8 is in range and the
    // arrays are 16-byte aligned (base is a multiple of 8 words)
    const bool vec = base + kScanItems <= n && ((((uintptr_t)in) | ((uintptr_t)out)) & 15u) == 0u;
    if (vec) {
        const uint4 q0 = *reinterpret_cast<const uint4 *>(in + base);
        const uint4 q1 = *reinterpret_cast<const uint4 *>(in + base + 4);
        x[0] = q0.x; x[1] = q0.y; x[2] = q0.z; x[3] = q0.w;
        x[4] = q1.x; x[5] = q1.y; x[6] = q1.z; x[7] = q1.w;
    } else {
#pragma unroll
        for (int k = 0; k < kScanItems; ++k) x[k] = (base + k < n) ? in[base + k] : 0u;
    }
#pragma unroll
    for (int k = 0; k < kScanItems; ++k) sum += x[k];
    uint32_t tot;
    const uint32_t ex = block_exclusive_scan(sum, lds, &tot);
    if (threadIdx.x < 64) {
        const uint32_t prefix = dev::lookback_prefix_wave(status, tile, tag, tot, threadIdx.x);
        if (threadIdx.x == 0) {
            s_prefix = prefix;
            if (tile == gridDim.x - 1 && total_out) *total_out = prefix + tot;
        }
    }
    __syncthreads();
    uint32_t run = s_prefix + ex;
    uint32_t o[kScanItems];
#pragma unroll
    for (int k = 0; k < kScanItems; ++k) {
        o[k] = run;
        run += x[k];
    }
    if (vec) {
        *reinterpret_cast<uint4 *>(out + base) = make_uint4(o[0], o[1], o[2], o[3]);
        *reinterpret_cast<uint4 *>(out + base + 4) = make_uint4(o[4], o[5], o[6], o[7]);
    } else {
#pragma unroll
        for (int k = 0; k < kScanItems; ++k)
            if (base + k < n) out[base + k] = o[k];
    }
}


// `partials`: scan_partials_words(n) u32 words, 8-byte aligned (status words).
// epoch (the builder's scans): tag = scan_tag(epoch, k); else a fresh host tag
hipError_t exclusive_scan(const uint32_t *in, uint32_t *out, uint32_t n, uint32_t *partials,
                          uint32_t *total_dev, hipStream_t st, const uint32_t *epoch = nullptr, uint32_t k = 0) {
    if (n == 0) return hipSuccess;
    const uint32_t nb = (n + kScanTile - 1) / kScanTile;
    const uint32_t tag = epoch ? k : next_scan_tag();
    hipLaunchKernelGGL(k_scan_onepass, dim3(nb), dim3(kThreads), 0, st, in, out, n,
                       reinterpret_cast<unsigned long long *>(partials), tag, total_dev, epoch);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Stable LSD radix sort of (key, value): 3 passes of 10-bit digits over the
// 30-bit codes (thrust::stable_sort_by_key semantics, Renderer.cpp:441-445).
// A pass is the digit counts of every block tile (k_morton for the first
// digit, k_rs_hist10 after), one exclusive scan over them (digit-major:
// every tile's start for every digit), and k_rs_scatter10.
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(kRsBlock) k_rs_hist10(const uint32_t *__restrict__ keys, uint32_t n,
                                                         int shift, uint32_t *__restrict__ hist,
                                                         uint32_t nblocks) {
    __shared__ uint32_t h[kRdBins];
    for (uint32_t k = threadIdx.x; k < kRdBins; k += kRsBlock) h[k] = 0u;
    __syncthreads();
    const uint64_t base = (uint64_t)blockIdx.x * kRsTile;
    uint32_t key[kRsPer];
#pragma unroll
    for (int r = 0; r < kRsPer; ++r) {
        const uint64_t i = base + (uint64_t)r * kRsBlock + threadIdx.x;
        key[r] = i < n ? keys[i] : 0u;
    }
#pragma unroll
    for (int r = 0; r < kRsPer; ++r) {
        const uint64_t i = base + (uint64_t)r * kRsBlock + threadIdx.x;
        if (i < n) atomicAdd(&h[(key[r] >> shift) & (kRdBins - 1u)], 1u);
    }
    __syncthreads();
    for (uint32_t k = threadIdx.x; k < kRdBins; k += kRsBlock) hist[(uint64_t)k * nblocks + blockIdx.x] = h[k];
}

// Each of the block's kRsWaves waves owns a contiguous part of the tile
// (kRsPer rounds of 64), so the pass is stable: the waves' per-digit counts
// are ranked once, then each wave walks its rounds with no block barrier --
// per round the lanes of one digit find each other by 10 ballots, the
// group's first lane advances the wave's digit cursor with one LDS atomic
// and the group reads its base from that lane.  The ranks are positions in
// the tile sorted by digit (LDS); the sorted tile then goes out in order,
// each digit's run to its place after the earlier tiles' (the scan), so
// consecutive threads write consecutive words.  (Writing each element
// straight to its global position -- up to 64 runs per store -- took
// 0.024 ms per pass at 1M, r04b.)
__global__ void __launch_bounds__(kRsBlock) k_rs_scatter10(const uint32_t *__restrict__ kin,
                                                           const uint32_t *__restrict__ vin, uint32_t n,
                                                           int shift, const uint32_t *__restrict__ hist_scan,
                                                           uint32_t nblocks, uint32_t *__restrict__ kout,
                                                           uint32_t *__restrict__ vout) {
    __shared__ uint32_t cnt[kRsWaves][kRdBins];   // per wave and digit: count, then cursor
    __shared__ uint32_t s_key[kRsTile], s_val[kRsTile];
    __shared__ uint32_t s_lstart[kRdBins];        // digit d's first position in the sorted tile
    __shared__ uint32_t s_gstart[kRdBins];        // its first position in the output
    __shared__ uint32_t s_wsum[kRsWaves];
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6;
    for (uint32_t k = tid; k < kRsWaves * kRdBins; k += kRsBlock) (&cnt[0][0])[k] = 0u;
    __syncthreads();
    const uint64_t tile0 = (uint64_t)blockIdx.x * kRsTile;
    const uint64_t base = tile0 + (uint64_t)wave * 64u * kRsPer;
    uint32_t key[kRsPer], val[kRsPer];
#pragma unroll
    for (int r = 0; r < kRsPer; ++r) {
        const uint64_t i = base + (uint64_t)r * 64u + lane;
        key[r] = i < n ? kin[i] : 0u;
        val[r] = i < n ? vin[i] : 0u;
    }
#pragma unroll
    for (int r = 0; r < kRsPer; ++r) {
        const uint64_t i = base + (uint64_t)r * 64u + lane;
        if (i < n) atomicAdd(&cnt[wave][(key[r] >> shift) & (kRdBins - 1u)], 1u);
    }
    __syncthreads();
    // digit d = tid: the waves' exclusive prefixes, the tile's total of d,
    // and the tile-exclusive scan of the totals over the digits
    static_assert(kRsBlock == kRdBins, "one thread per digit");
    const uint32_t d = tid;
    uint32_t tot = 0;
#pragma unroll
    for (uint32_t w = 0; w < kRsWaves; ++w) {
        const uint32_t c = cnt[w][d];
        cnt[w][d] = tot;
        tot += c;
    }
    uint32_t inc = tot;
#pragma unroll
    for (uint32_t o = 1; o < 64u; o <<= 1) {
        const uint32_t y = __shfl_up(inc, o, 64);
        if (lane >= o) inc += y;
    }
    if (lane == 63u) s_wsum[wave] = inc;
    __syncthreads();
    uint32_t lstart = inc - tot;
    for (uint32_t w = 0; w < wave; ++w) lstart += s_wsum[w];
    s_lstart[d] = lstart;
    s_gstart[d] = hist_scan[(uint64_t)d * nblocks + blockIdx.x];
#pragma unroll
    for (uint32_t w = 0; w < kRsWaves; ++w) cnt[w][d] += lstart;
    __syncthreads();
    const unsigned long long lt = (1ull << lane) - 1ull;
#pragma unroll
    for (int r = 0; r < kRsPer; ++r) {
        const uint64_t i = base + (uint64_t)r * 64u + lane;
        const bool valid = i < n;
        const uint32_t dg = (key[r] >> shift) & (kRdBins - 1u);
        unsigned long long peers = __ballot(valid);
#pragma unroll
        for (int b = 0; b < kRdBits; ++b) {
            const bool bit = (dg >> b) & 1u;
            const unsigned long long bb = __ballot(bit);
            peers &= bit ? bb : ~bb;
        }
        const uint32_t rank = (uint32_t)__popcll(peers & lt);
        uint32_t off = 0;
        if (valid && rank == 0u) off = atomicAdd(&cnt[wave][dg], (uint32_t)__popcll(peers));
        const uint32_t leader = valid ? (uint32_t)__builtin_ctzll(peers) : lane;
        off = (uint32_t)__shfl((int)off, (int)leader, 64);
        if (valid) {
            s_key[off + rank] = key[r];
            s_val[off + rank] = val[r];
        }
    }
    __syncthreads();
    const uint32_t m = (uint32_t)(n - tile0 < (uint64_t)kRsTile ? n - tile0 : (uint64_t)kRsTile);
    for (uint32_t j = tid; j < m; j += kRsBlock) {
        const uint32_t k = s_key[j];
        const uint32_t dg = (k >> shift) & (kRdBins - 1u);
        const uint32_t o = s_gstart[dg] + (j - s_lstart[dg]);
        kout[o] = k;
        vout[o] = s_val[j];
    }
}

// ---------------------------------------------------------------------------
// Runs of equal codes in one pass (reduce_by_key + unique_by_key_copy,
// Renderer.cpp:450-472): a run starts where the code changes; the start
// flags are scanned with the decoupled look-back (k_scan_onepass's), and
// each run's first element writes its code and first index, each element
// the leaf it falls in (DeviceTree::tri_leaf), and each run's last element
// its end (k_karras turns ends into counts).  The last tile writes U.
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(kThreads) k_runs(const uint32_t *__restrict__ keys, uint32_t n,
                                                   unsigned long long *status, uint32_t tag,
                                                   uint32_t *__restrict__ umc, int32_t *__restrict__ first,
                                                   uint32_t *__restrict__ run_end, uint32_t *__restrict__ leaf_of,
                                                   TreeHeader *hdr, const uint32_t *epoch) {
    __shared__ uint32_t lds[4];
    tag = scan_tag(epoch, tag);
    __shared__ uint32_t s_prefix;
    const uint32_t tile = blockIdx.x;
    const uint64_t base = (uint64_t)tile * kScanTile + (uint64_t)threadIdx.x * kScanItems;
    uint32_t key[kScanItems + 1];   // key[0] = the code before this thread's first element
    key[0] = (base > 0 && base - 1 < n) ? keys[base - 1] : 0u;
    static_assert(kScanItems == 8, "two 16-byte loads per thread");
    if (base + kScanItems <= n) {   // whole: 16-byte loads (base is a multiple of 8 words)
        const uint4 q0 = *reinterpret_cast<const uint4 *>(keys + base);
        const uint4 q1 = *reinterpret_cast<const uint4 *>(keys + base + 4);
        key[1] = q0.x; key[2] = q0.y; key[3] = q0.z; key[4] = q0.w;
        key[5] = q1.x; key[6] = q1.y; key[7] = q1.z; key[8] = q1.w;
    } else {
#pragma unroll
        for (int k = 0; k < kScanItems; ++k) key[k + 1] = base + k < n ? keys[base + k] : 0u;
    }
    uint32_t flags = 0, sum = 0;
#pragma unroll
    for (int k = 0; k < kScanItems; ++k) {
        const uint64_t i = base + k;
        const bool f = i < n && (i == 0 || key[k + 1] != key[k]);
        flags |= (f ? 1u : 0u) << k;
        sum += f ? 1u : 0u;
    }
    const uint32_t nxt = (base + kScanItems < n) ? keys[base + kScanItems] : 0u;
    uint32_t tot;
    const uint32_t ex = block_exclusive_scan(sum, lds, &tot);
    if (threadIdx.x < 64) {
        const uint32_t prefix = dev::lookback_prefix_wave(status, tile, tag, tot, threadIdx.x);
        if (threadIdx.x == 0) {
            s_prefix = prefix;
            if (tile == gridDim.x - 1) hdr->n_unique = prefix + tot;
        }
    }
    __syncthreads();
    uint32_t run = s_prefix + ex;   // runs started before element base
    uint32_t lf[kScanItems];
#pragma unroll
    for (int k = 0; k < kScanItems; ++k) {
        const uint64_t i = base + k;
        if (i >= n) break;
        const bool f = (flags >> k) & 1u;
        if (f) {
            umc[run] = key[k + 1];
            first[run] = (int32_t)i;
        }
        run += f ? 1u : 0u;
        const uint32_t leaf = run - 1u;
        lf[k] = leaf;
        const uint32_t after = k + 1 < kScanItems ? key[k + 2] : nxt;
        if (i + 1 == n || after != key[k + 1]) run_end[leaf] = (uint32_t)(i + 1);
    }
    if (base + kScanItems <= n) {
        *reinterpret_cast<uint4 *>(leaf_of + base) = make_uint4(lf[0], lf[1], lf[2], lf[3]);
        *reinterpret_cast<uint4 *>(leaf_of + base + 4) = make_uint4(lf[4], lf[5], lf[6], lf[7]);
    } else {
#pragma unroll
        for (int k = 0; k < kScanItems; ++k)
            if (base + k < n) leaf_of[base + k] = lf[k];
    }
}

// ---------------------------------------------------------------------------
// k_karras: BuildTree, CUDAKernels.cu:591-710, with its uint32/int mixing.
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(kThreads) k_karras(const uint32_t *__restrict__ umc,
                                                     const TreeHeader *__restrict__ hdr,
                                                     const int32_t *__restrict__ first,
                                                     uint32_t *__restrict__ dup_cnt,
                                                     int32_t *__restrict__ children,
                                                     uint8_t *__restrict__ is_leaf,
                                                     int32_t *__restrict__ axis_out,
                                                     int32_t *__restrict__ parent,
                                                     int32_t *__restrict__ leaf_parent,
                                                     int2 *__restrict__ node_rng) {
    const int U = (int)hdr->n_unique;
    uint32_t idx = blockIdx.x * kThreads + threadIdx.x;
    // leaf idx's triangle count (m_duplicatesCnts): k_runs left the run's end
    if (idx < (uint32_t)U) dup_cnt[idx] -= (uint32_t)first[idx];
    if (U == 1 && idx == 0) leaf_parent[0] = -1;   // no internal node (U >= 2: every leaf gets a parent below)
    // the codes around the block's nodes, staged in LDS: the searches of
    // most nodes (short leaf ranges) stay inside the window; farther probes
    // read global memory
    constexpr int kWin = 256, kWinN = kThreads + 2 * kWin;
    __shared__ uint32_t s_mc[kWinN];
    const int64_t w0 = (int64_t)blockIdx.x * kThreads - kWin;
    for (int k = threadIdx.x; k < kWinN; k += kThreads) {
        const int64_t g = w0 + k;
        s_mc[k] = (g >= 0 && g < U) ? umc[g] : 0u;
    }
    __syncthreads();
    auto mc = [&](int64_t i) -> uint32_t {
        const int64_t o = i - w0;
        return (o >= 0 && o < kWinN) ? s_mc[o] : umc[i];
    };
    if (U < 2 || idx > (uint32_t)(U - 2)) return;
    if (idx == 0) parent[0] = -1;   // the root; every other node is written as a child below
    uint32_t cur = mc(idx);
    uint32_t pre0 = 0xFFFFFFFFu, pre1 = 0xFFFFFFFFu;
    if (idx) pre0 = (uint32_t)clz32(cur ^ mc(idx - 1));
    if (idx < (uint32_t)(U - 1)) pre1 = (uint32_t)clz32(cur ^ mc(idx + 1));
    int32_t diff = (int32_t)(pre1 - pre0);
    int d = (0 < diff) - (diff < 0);
    int lcp_min = (int32_t)(((d + 1) / 2) ? pre0 : pre1);   // pre[1 - (d+1)/2]
    int lmax = 1, lcp, li;
    do {
        lmax *= 2;
        li = (int32_t)(idx + (uint32_t)(lmax * d));
        lcp = (li < 0 || li > U - 1) ? -1 : clz32(cur ^ mc(li));
    } while (lcp > lcp_min);
    int l = 0;
    for (int t = lmax / 2; t >= 1; t /= 2) {
        int ti = (int32_t)(idx + (uint32_t)((l + t) * d));
        lcp = (ti < 0 || ti > U - 1) ? -1 : clz32(cur ^ mc(ti));
        if (lcp > lcp_min) l += t;
    }
    int other = (int32_t)(idx + (uint32_t)(l * d));
    int lcp_ends = clz32(cur ^ mc(other));
    int s = 0, t = l;
    for (;;) {
        t = (int)ceilf((float)t / 2.0f);           // __float2int_ru(t / 2.0f)
        int ti = (int32_t)(idx + (uint32_t)((s + t) * d));
        lcp = (ti < 0 || ti > U - 1) ? -1 : clz32(cur ^ mc(ti));
        if (lcp > lcp_ends) s += t;
        if (t == 1) break;
    }
    int split = (int32_t)(idx + (uint32_t)(s * d)) + (d < 0 ? d : 0);
    children[2 * idx] = split;
    children[2 * idx + 1] = split + 1;
    uint32_t mn = idx < (uint32_t)other ? idx : (uint32_t)other;
    uint32_t mx = idx > (uint32_t)other ? idx : (uint32_t)other;
    node_rng[idx] = make_int2((int32_t)mn, (int32_t)mx);   // the node's leaves (k_fit)
    uint8_t l0 = (mn == (uint32_t)split), l1 = (mx == (uint32_t)(split + 1));
    is_leaf[2 * idx] = l0;
    is_leaf[2 * idx + 1] = l1;
    if (l0) leaf_parent[split] = (int32_t)idx; else parent[split] = (int32_t)idx;
    if (l1) leaf_parent[split + 1] = (int32_t)idx; else parent[split + 1] = (int32_t)idx;
    axis_out[idx] = (clz32(mc(split) ^ mc(split + 1)) + 1) % 3;
}

// ---------------------------------------------------------------------------
// k_fit: clip planes.  Reference: every leaf walks to the root doing
// atomicMaxFloat(clip[0], leafHi[axis]) / atomicMinFloat(clip[1],
// leafLo[axis]) (CUDAKernels.cu:511-547), i.e. clip[0] = max over the left
// subtree's leaves, clip[1] = min over the right subtree's leaves (IEEE
// totalOrder, tkey).  A Karras node's subtree is the contiguous leaf range
// [mn, mx] (k_karras, node_rng) with the left child [mn, split] and the right
// [split + 1, mx], so each clip is one range query over the leaf boxes:
//   k_seg_build leaf boxes (CUDAKernels.cu:511-529) = level 0 of a segment
//               tree of the six box components (SoA), entry i of level L =
//               leaves [i 2^L, (i+1) 2^L) (min for lo, max for hi), and
//               levels 1..10 through LDS; up to 2^20 leaves its last block
//               builds the rest (k_seg_up per 10 levels above that);
//   k_fit       per node two O(log U) queries (no atomics).
// totalOrder max/min is associative and commutative, so any grouping gives
// the reference's result bit for bit.  (Before: boxes handed bottom-up through
// device-scope atomics and arrival counters, three atomic round trips per
// level on the root's chain: 0.47 ms at 1M.)
// ---------------------------------------------------------------------------
constexpr uint32_t kSegBlock = 1024;   // level-L entries per k_seg_up block
constexpr int kSegSteps = 10;          // levels per k_seg_up launch (1024 = 2^10)
constexpr uint32_t kMaxKeyBits = 0xFFFFFFFFu;   // tkey minimum: identity of tmax
constexpr uint32_t kMinKeyBits = 0x7FFFFFFFu;   // tkey maximum: identity of tmin

// entries per component: sum over levels of ceil(nn / 2^L)
uint64_t seg_capacity(uint64_t nn) {
    uint64_t c = 0, s = nn;
    for (;;) {
        c += s;
        if (s <= 1) break;
        s = (s + 1) / 2;
    }
    return c;
}
__device__ __forceinline__ uint64_t seg_level_off(uint64_t nn, int L) {
    uint64_t off = 0, s = nn;
    for (int l = 0; l < L; ++l) {
        off += s;
        s = (s + 1) / 2;
    }
    return off;
}

// Sorted triangle i as the render reads it: {v0, e1 = v1 - v0, e2 = v2 - v0}
// (CUDAKernels.cu:18-19), from the input triangle p; returns its AABB (the
// values k_prep wrote, axis_minmax).
__device__ __forceinline__ void pack_tri(const float *__restrict__ p, float *__restrict__ o, float lo[3],
                                         float hi[3]) {
    float q[9];
#pragma unroll
    for (int k = 0; k < 9; ++k) q[k] = p[k];
    o[0] = q[0]; o[1] = q[1]; o[2] = q[2];
    o[3] = q[3] - q[0]; o[4] = q[4] - q[1]; o[5] = q[5] - q[2];   // v0v1, CUDAKernels.cu:18
    o[6] = q[6] - q[0]; o[7] = q[7] - q[1]; o[8] = q[8] - q[2];   // v0v2, :19
#pragma unroll
    for (int a = 0; a < 3; ++a) axis_minmax(q[a], q[3 + a], q[6 + a], lo[a], hi[a]);
}

// Leaf k's box (CUDAKernels.cu:511-529), and the sorted triangle records of
// its run (the runs partition the sorted triangles: read once with the
// vertices the boxes come from).
__device__ __forceinline__ void leaf_box(const uint32_t *__restrict__ tri_idx, const float *__restrict__ v,
                                         float *__restrict__ tris_s, const int32_t *__restrict__ first,
                                         const uint32_t *__restrict__ cnt, uint32_t k, float blo[3],
                                         float bhi[3]) {
    const int32_t f = first[k];
    const uint32_t c = cnt[k];
    pack_tri(v + 9ull * tri_idx[f], tris_s + 9ull * f, blo, bhi);
    for (uint32_t i = 1; i < c; ++i) {
        float tlo[3], thi[3];
        pack_tri(v + 9ull * tri_idx[f + i], tris_s + 9ull * (f + i), tlo, thi);
#pragma unroll
        for (int a = 0; a < 3; ++a) {
            blo[a] = tmin(blo[a], tlo[a]);
            bhi[a] = tmax(bhi[a], thi[a]);
        }
    }
}

// Levels L0+1 .. L0+kSegSteps of the segment tree from level-L0 entries
// [base, base + kSegBlock) held in LDS (vl).  Only entries of the U valid
// leaves are combined (a partial last entry is never read by a query).  The
// last level's entries are stored sc1 when `hand_off` (the last-block
// hand-off of k_seg_build).
template <uint32_t NT>
__device__ __forceinline__ void seg_levels(float (*vl)[kSegBlock], float *__restrict__ seg, uint64_t cap,
                                           uint64_t nn, uint32_t U, int L0, uint64_t base, bool hand_off) {
    static_assert(kSegBlock / 2 <= 4 * NT, "r[4]: at most 4 entries per thread per level");
    const uint32_t tid = threadIdx.x;
    uint64_t off = seg_level_off(nn, L0), size = nn;
    uint64_t vsize = U;                             // valid entries of the level
    for (int l = 0; l < L0; ++l) {
        size = (size + 1) / 2;
        vsize = (vsize + 1) / 2;
    }
    uint32_t cnt = kSegBlock;
    for (int s = 1; s <= kSegSteps; ++s) {
        if (size <= 1) break;                       // the top level is done (uniform)
        const uint64_t pvsize = vsize;
        off += size;
        size = (size + 1) / 2;
        vsize = (vsize + 1) / 2;
        cnt >>= 1;
        const uint64_t gb = base >> s;              // this block's first entry at level L0+s
        float r[4][6];
        uint32_t nj = 0;
        for (uint32_t j = tid; j < cnt; j += NT, ++nj) {
            const uint64_t g = gb + j;
            if (g < vsize) {
                const bool two = 2 * g + 1 < pvsize;
#pragma unroll
                for (int c = 0; c < 6; ++c) {
                    const float x = vl[c][2 * j];
                    r[nj][c] = two ? (c < 3 ? tmin(x, vl[c][2 * j + 1]) : tmax(x, vl[c][2 * j + 1])) : x;
                }
            }
        }
        __syncthreads();
        nj = 0;
        const bool sc1 = hand_off && s == kSegSteps;
        for (uint32_t j = tid; j < cnt; j += NT, ++nj) {
            const uint64_t g = gb + j;
            if (g < vsize)
#pragma unroll
                for (int c = 0; c < 6; ++c) {
                    vl[c][j] = r[nj][c];
                    if (sc1)
                        __hip_atomic_store(seg + c * cap + off + g, r[nj][c], __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT);
                    else
                        seg[c * cap + off + g] = r[nj][c];
                }
        }
        __syncthreads();
    }
}

// Leaf boxes (level 0, with the sorted triangle records of every run) and
// levels 1..10 of the segment tree in one launch: block b owns leaves
// [b kSegBlock, (b+1) kSegBlock).  With `top` (at most kSegBlock blocks,
// nn <= 2^20) the last block to finish also builds the levels above 10 from
// the blocks' level-10 entries -- stored sc1, waited for, a barrier, one
// agent-scope add per block, read sc1 by the block whose add came last
// (MI355X_MICROARCH.md, cross-workgroup table, row 1); larger trees take
// k_seg_up launches for those levels.  (Round 3: k_seg_leaf + 2 x k_seg_up,
// 0.035 + 0.018 + 0.012 ms at 1M, r04d.)
constexpr uint32_t kSegThreads = 1024;   // k_seg_build: one leaf per thread
__global__ void __launch_bounds__(kSegThreads) k_seg_build(const TreeHeader *__restrict__ hdr,
                                                        const uint32_t *__restrict__ tri_idx,
                                                        const float *__restrict__ v, float *__restrict__ tris_s,
                                                        const int32_t *__restrict__ first,
                                                        const uint32_t *__restrict__ cnt, float *__restrict__ seg,
                                                        uint64_t cap, uint64_t nn, int top,
                                                        unsigned long long *arrivals) {
    __shared__ float vl[6][kSegBlock];
    __shared__ uint32_t s_last;
    const uint32_t U = hdr->n_unique;
    if (U < 2) return;   // (uniform: no block takes part in the hand-off)
    const uint32_t tid = threadIdx.x;
    const uint64_t base = (uint64_t)blockIdx.x * kSegBlock;
    for (uint32_t j = tid; j < kSegBlock; j += kSegThreads) {
        const uint64_t k = base + j;
        if (k < U) {
            float blo[3], bhi[3];
            leaf_box(tri_idx, v, tris_s, first, cnt, (uint32_t)k, blo, bhi);
#pragma unroll
            for (int a = 0; a < 3; ++a) {
                vl[a][j] = blo[a];
                vl[3 + a][j] = bhi[a];
                seg[a * cap + k] = blo[a];
                seg[(3 + a) * cap + k] = bhi[a];
            }
        }
    }
    __syncthreads();
    seg_levels<kSegThreads>(vl, seg, cap, nn, U, 0, base, top != 0);
    if (!top) return;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0)
        s_last = __hip_atomic_fetch_add(arrivals, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
                 (unsigned long long)gridDim.x - 1ull;
    __syncthreads();
    if (!s_last) return;
    if (tid == 0) __hip_atomic_store(arrivals, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    // the level-10 entries of every block (sc1), then the levels above
    const uint64_t off10 = seg_level_off(nn, kSegSteps);
    uint64_t vs = U;
    for (int l = 0; l < kSegSteps; ++l) vs = (vs + 1) / 2;
    for (uint32_t j = tid; j < kSegBlock; j += kSegThreads)
        if (j < vs)
#pragma unroll
            for (int c = 0; c < 6; ++c)
                vl[c][j] = __hip_atomic_load(seg + c * cap + off10 + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    seg_levels<kSegThreads>(vl, seg, cap, nn, U, kSegSteps, 0, false);
}

// Levels L0+1 .. L0+kSegSteps from level L0 (trees over 2^20 leaves, levels
// above 10): block b owns level-L0 entries [b kSegBlock, (b+1) kSegBlock).
__global__ void __launch_bounds__(kThreads) k_seg_up(const TreeHeader *__restrict__ hdr,
                                                     float *__restrict__ seg, uint64_t cap, uint64_t nn,
                                                     int L0) {
    __shared__ float vl[6][kSegBlock];
    const uint32_t U = hdr->n_unique;
    if (U < 2) return;
    uint64_t off = seg_level_off(nn, L0), vsize = U;
    for (int l = 0; l < L0; ++l) vsize = (vsize + 1) / 2;
    const uint64_t base = (uint64_t)blockIdx.x * kSegBlock;
    for (uint32_t j = threadIdx.x; j < kSegBlock; j += kThreads)
        if (base + j < vsize)
#pragma unroll
            for (int c = 0; c < 6; ++c) vl[c][j] = seg[c * cap + off + base + j];
    __syncthreads();
    seg_levels<kThreads>(vl, seg, cap, nn, U, L0, base, false);
}

// totalOrder max (HI) / min over leaves [a, b] of component c
template <bool HI>
__device__ __forceinline__ float seg_query(const float *__restrict__ seg, uint64_t nn, uint32_t a,
                                           uint32_t b) {
    float res = __uint_as_float(HI ? kMaxKeyBits : kMinKeyBits);
    uint64_t l = a, r = (uint64_t)b + 1, off = 0, size = nn;
    while (l < r) {
        if (l & 1) {
            const float x = seg[off + l];
            res = HI ? tmax(res, x) : tmin(res, x);
            ++l;
        }
        if (r & 1) {
            --r;
            const float x = seg[off + r];
            res = HI ? tmax(res, x) : tmin(res, x);
        }
        l >>= 1;
        r >>= 1;
        off += size;
        size = (size + 1) / 2;
    }
    return res;
}

// seg_query with every load issued before any is combined (the segment
// nodes of a query follow from a, b and the level sizes alone, not from the
// values loaded): one memory round trip per query instead of one per level.
// Same nodes, and tmax / tmin are associative and commutative: the same
// result bit for bit.  Levels: ceil(log2(nn)) + 1 <= 28 for nn <= 2^27.
#ifndef BIH_FIT_PIPE
#define BIH_FIT_PIPE 0   // 1: slower (k_fit 0.048 vs 0.032 ms, r04a: 122 VGPRs, 4 waves)
#endif
constexpr int kSegMaxLevels = 28;
template <bool HI>
__device__ __forceinline__ float seg_query_pipe(const float *__restrict__ seg, uint64_t nn, uint32_t a,
                                                uint32_t b) {
    const float ident = __uint_as_float(HI ? kMaxKeyBits : kMinKeyBits);
    float x[2 * kSegMaxLevels];
    uint32_t l = a, r = b + 1u;
    uint64_t off = 0, size = nn;
#pragma unroll
    for (int lv = 0; lv < kSegMaxLevels; ++lv) {
        const bool act = l < r;
        const bool tl = act && (l & 1u), tr = act && (r & 1u);
        x[2 * lv] = tl ? seg[off + l] : ident;
        x[2 * lv + 1] = tr ? seg[off + r - 1u] : ident;
        l = (l + (tl ? 1u : 0u)) >> 1;
        r = (r - (tr ? 1u : 0u)) >> 1;
        off += size;
        size = (size + 1) / 2;
    }
    float res = ident;
#pragma unroll
    for (int k = 0; k < 2 * kSegMaxLevels; ++k) res = HI ? tmax(res, x[k]) : tmin(res, x[k]);
    return res;
}

// The clip planes of node p and its 16-byte render record (k_pack_nodes'
// layout, bih_internal.h) in one pass: the node's thread has every field.
// A one-leaf tree has no node: the threads pack the sorted triangle records
// instead (k_seg_build packs them for U >= 2).
__global__ void __launch_bounds__(kThreads) k_fit(const TreeHeader *__restrict__ hdr,
                                                  const int2 *__restrict__ node_rng,
                                                  const int32_t *__restrict__ children,
                                                  const int32_t *__restrict__ axis,
                                                  const float *__restrict__ seg, uint64_t cap, uint64_t nn,
                                                  float *__restrict__ clip,
                                                  const uint8_t *__restrict__ is_leaf,
                                                  const int32_t *__restrict__ first,
                                                  const uint32_t *__restrict__ cnt, uint4 *__restrict__ nodes,
                                                  const float *__restrict__ v, const uint32_t *__restrict__ tri_idx,
                                                  uint32_t n, float *__restrict__ tris_s,
                                                  TreeHeader *__restrict__ hdr_host) {
    const uint32_t U = hdr->n_unique;
    const uint32_t p = blockIdx.x * kThreads + threadIdx.x;
    if (p == 0) *hdr_host = *hdr;   // the host reads it after the stream synchronises (build_tree_device)
    if (U < 2) {
        for (uint32_t i = p; i < n; i += gridDim.x * kThreads) {
            float lo[3], hi[3];
            pack_tri(v + 9ull * tri_idx[i], tris_s + 9ull * i, lo, hi);
        }
        return;
    }
    if (p >= U - 1) return;
    const int2 rg = node_rng[p];
    const uint32_t split = (uint32_t)children[2 * p];
    const int ax = axis[p];
#if BIH_FIT_PIPE
    const float lhi = seg_query_pipe<true>(seg + (3 + ax) * cap, nn, (uint32_t)rg.x, split);
    const float rlo = seg_query_pipe<false>(seg + ax * cap, nn, split + 1u, (uint32_t)rg.y);
#else
    const float lhi = seg_query<true>(seg + (3 + ax) * cap, nn, (uint32_t)rg.x, split);
    const float rlo = seg_query<false>(seg + ax * cap, nn, split + 1u, (uint32_t)rg.y);
#endif
    const float c0 = tmax(-FLT_MAX, lhi);          // initial values GPUArrayManager.cpp:79-80
    const float c1 = tmin(FLT_MAX, rlo);
    clip[2 * p] = c0;
    clip[2 * p + 1] = c1;
    // the render record (k_pack_nodes until round 4)
    const uint32_t lL = is_leaf[2 * p], lR = is_leaf[2 * p + 1];
    const uint32_t mid = (uint32_t)first[split + 1];
    const uint32_t cL = lL ? cnt[split] : 0u, cR = lR ? cnt[split + 1] : 0u;
    const uint32_t codeL = (cL >= 1 && cL <= 3) ? cL : 0u;
    const uint32_t codeR = (cR >= 1 && cR <= 3) ? cR : 0u;
    uint4 nd;
    nd.x = __float_as_uint(c0);
    nd.y = __float_as_uint(c1);
    nd.z = split | ((uint32_t)ax << 27) | (lL << 29) | (lR << 30);
    nd.w = mid | (codeL << 27) | (codeR << 29);
    nodes[p] = nd;
}

inline uint32_t blocks_for(uint64_t n) { return (uint32_t)((n + kThreads - 1) / kThreads); }

}  // namespace

#define BIH_TRY(x)                                  \
    do {                                            \
        hipError_t e__ = (x);                       \
        if (e__ != hipSuccess) return (int)e__;     \
    } while (0)

template <class T>
static hipError_t dalloc(T **p, size_t count, DeviceTree &t) {
    size_t b = count * sizeof(T);
    if (b == 0) b = 16;
    if (t.fail_alloc && --t.fail_alloc == 0) return hipErrorOutOfMemory;   // tests
    const hipError_t e = hipMalloc((void **)p, b);
    if (e != hipSuccess) {
        *p = nullptr;
        return e;
    }
    t.bytes += b;
    ++t.allocs;
    return e;
}

// exclusive scan for the other translation units (frustum bins)
int scan_exclusive(const uint32_t *in, uint32_t *out, uint32_t n, uint32_t *partials,
                   uint32_t *total_dev, void *stream) {
    return (int)exclusive_scan(in, out, n, partials, total_dev, (hipStream_t)stream);
}
// tags of the look-back status words (dev::lookback_prefix): 1 .. 2^30-1,
// unique per call
uint32_t next_scan_tag() {
    static std::atomic<uint32_t> tag{0};
    return (tag.fetch_add(1) % 0x3FFFFFFFu) + 1u;
}

size_t scan_partials_words(uint32_t n) { return 2 * (size_t)((n + kScanTile - 1) / kScanTile) + 2; }

// The build's device buffers (not the soup, the events or the pinned
// header), freed and cleared: a tree whose allocation failed part-way holds
// none of them, so its next build allocates them all again.
static void free_build_buffers(DeviceTree &t) {
    void **ptrs[] = {(void **)&t.hdr, (void **)&t.tri_lo, (void **)&t.tri_hi, (void **)&t.keys,
                     (void **)&t.vals, (void **)&t.keys2, (void **)&t.vals2, (void **)&t.scan_tmp,
                     (void **)&t.flags, (void **)&t.unique_mc, (void **)&t.dup_cnt, (void **)&t.first_idx,
                     (void **)&t.leaf_parent, (void **)&t.clip, (void **)&t.axis, (void **)&t.children,
                     (void **)&t.parent, (void **)&t.is_leaf, (void **)&t.fit_rng, (void **)&t.fit_seg,
                     (void **)&t.nodes, (void **)&t.tris_s, (void **)&t.hist, (void **)&t.partials,
                     (void **)&t.prep_part};
    for (void **p : ptrs) {
        if (*p) (void)hipFree(*p);
        *p = nullptr;
    }
}

void free_tree_device(DeviceTree &t) {
    if (t.graph) (void)hipGraphExecDestroy(t.graph);
    free_build_buffers(t);
    if (t.hdr_host) (void)hipHostFree(t.hdr_host);
    if (t.ev0) (void)hipEventDestroy(t.ev0);
    if (t.ev1) (void)hipEventDestroy(t.ev1);
    if (t.owns_v && t.v) (void)hipFree(t.v);
    DeviceTree blank;
    blank.device = t.device;
    t = blank;
}

#define BIH_TRY_E(x)                                \
    do {                                            \
        hipError_t e__ = (x);                       \
        if (e__ != hipSuccess) return e__;          \
    } while (0)
static hipError_t alloc_build_buffers(DeviceTree &t, uint64_t nn, uint64_t hist_n, uint32_t max_parts,
                                      hipStream_t st) {
    BIH_TRY_E(dalloc(&t.hdr, 1, t));
    BIH_TRY_E(dalloc(&t.tri_lo, 3 * nn, t));
    BIH_TRY_E(dalloc(&t.tri_hi, 3 * nn, t));
    BIH_TRY_E(dalloc(&t.keys, nn, t));
    BIH_TRY_E(dalloc(&t.vals, nn, t));
    BIH_TRY_E(dalloc(&t.keys2, nn, t));
    BIH_TRY_E(dalloc(&t.vals2, nn, t));
    BIH_TRY_E(dalloc(&t.scan_tmp, nn + 1, t));
    BIH_TRY_E(dalloc(&t.unique_mc, nn, t));
    BIH_TRY_E(dalloc(&t.dup_cnt, nn, t));
    BIH_TRY_E(dalloc(&t.first_idx, nn, t));
    BIH_TRY_E(dalloc(&t.leaf_parent, nn, t));
    BIH_TRY_E(dalloc(&t.clip, 2 * nn, t));
    BIH_TRY_E(dalloc(&t.axis, nn, t));
    BIH_TRY_E(dalloc(&t.children, 2 * nn, t));
    BIH_TRY_E(dalloc(&t.parent, nn, t));
    BIH_TRY_E(dalloc(&t.is_leaf, 2 * nn, t));
    BIH_TRY_E(dalloc(&t.fit_rng, nn, t));
    BIH_TRY_E(dalloc(&t.fit_seg, 6 * seg_capacity(nn), t));
    BIH_TRY_E(dalloc(&t.nodes, nn, t));
    BIH_TRY_E(dalloc(&t.tris_s, 9 * nn, t));
    BIH_TRY_E(dalloc(&t.hist, hist_n, t));
    BIH_TRY_E(dalloc(&t.partials, 2 * (uint64_t)max_parts + 2, t));   // k_scan_onepass status words
    // + k_seg_build's arrival count (zero between launches) + the build's
    // sequence number (k_prep; scan_tag)
    BIH_TRY_E(dalloc(&t.prep_part, 8ull * kPrepBlocks + 3, t));
    BIH_TRY_E(hipMemsetAsync(t.prep_part + 8ull * kPrepBlocks, 0, 3 * sizeof(unsigned long long), st));
    // look-back words (k_scan_onepass) start at tag 0 (never a call's tag):
    // stale data in fresh memory must not pass for a predecessor's published
    // prefix; afterwards every word carries an older call's (unique) tag
    BIH_TRY_E(hipMemsetAsync(t.partials, 0, (2 * (uint64_t)max_parts + 2) * sizeof(uint32_t), st));
    return hipSuccess;
}
#undef BIH_TRY_E

#define BIH_TRY_H(x)                                \
    do {                                            \
        hipError_t e__ = (x);                       \
        if (e__ != hipSuccess) return e__;          \
    } while (0)
// The build's kernels for n > 0 triangles, in order, on `st` (issued
// directly or captured into the tree's graph: build_tree_device).
static hipError_t issue_build(DeviceTree &t, uint32_t n, hipStream_t st) {
    const uint64_t nn = n;
    const uint32_t rs_blocks = (uint32_t)((nn + kRsTile - 1) / kRsTile);
    const uint64_t hist_n = (uint64_t)kRdBins * rs_blocks;
    {
        const uint32_t prep_blocks = blocks_for(n) < kPrepBlocks ? blocks_for(n) : kPrepBlocks;
        uint32_t *epoch = reinterpret_cast<uint32_t *>(t.prep_part + 8ull * kPrepBlocks + 2);
        hipLaunchKernelGGL(k_prep, dim3(prep_blocks), dim3(kThreads), 0, st, t.v, n, t.tri_lo,
                           t.tri_hi, t.hdr, t.prep_part, epoch);
        // (the fold of the partials: every k_morton block for itself; in
        // k_prep's last block instead -- a device-scope fence per block: k_prep
        // 0.147 ms, r04a; an sc1 store / agent-add / sc1 load hand-off: 0.032
        // ms, r04e -- against 0.016 + 0.012 for k_prep + k_prep_final)
        hipLaunchKernelGGL(k_morton, dim3(rs_blocks), dim3(kRsBlock), 0, st, t.v, t.tri_lo, t.tri_hi, t.hdr, n,
                           t.prep_part, prep_blocks, t.keys2, t.vals2, t.hist, rs_blocks);
        // 3 stable passes of 10-bit digits over the 30-bit codes (k_morton
        // counted the first digit): keys2 -> keys -> keys2 -> keys, so the
        // sorted pairs end in keys / vals and no pointer changes between
        // builds (a captured graph replays the same buffers)
        uint32_t *ka = t.keys2, *va = t.vals2, *kb = t.keys, *vb = t.vals;
        for (int p = 0; p < kRdPasses; ++p) {
            const int shift = kRdBits * p;
            if (p > 0)
                hipLaunchKernelGGL(k_rs_hist10, dim3(rs_blocks), dim3(kRsBlock), 0, st, ka, n, shift, t.hist,
                                   rs_blocks);
            BIH_TRY_H(exclusive_scan(t.hist, t.hist, (uint32_t)hist_n, t.partials, nullptr, st, epoch, 1u + p));
            hipLaunchKernelGGL(k_rs_scatter10, dim3(rs_blocks), dim3(kRsBlock), 0, st, ka, va, n, shift, t.hist,
                               rs_blocks, kb, vb);
            uint32_t *tk = ka, *tv = va;
            ka = kb; va = vb; kb = tk; vb = tv;
        }
        static_assert(kRdPasses % 2 == 1, "an odd pass count leaves the result in keys / vals");
        // runs: codes, first indices, ends (k_karras: counts), leaf of each
        // sorted triangle, U
        {
            const uint32_t nb = (n + kScanTile - 1) / kScanTile;
            hipLaunchKernelGGL(k_runs, dim3(nb), dim3(kThreads), 0, st, t.keys, n,
                               reinterpret_cast<unsigned long long *>(t.partials), 4u, t.unique_mc,
                               t.first_idx, t.dup_cnt, t.scan_tmp, t.hdr, epoch);
        }
        hipLaunchKernelGGL(k_karras, dim3(blocks_for(n)), dim3(kThreads), 0, st, t.unique_mc, t.hdr, t.first_idx,
                           t.dup_cnt, t.children, t.is_leaf, t.axis, t.parent, t.leaf_parent, t.fit_rng);
        const uint64_t cap = seg_capacity(nn);
        // leaf boxes (and the sorted triangle records of every leaf run when U >= 2) + segment tree levels 0..10 (and, up to 2^20 leaves, the
        // levels above by the last block); larger trees: k_seg_up per 10 levels
        const uint64_t seg_blocks = (nn + kSegBlock - 1) / kSegBlock;
        // (one block builds a whole tree of <= kSegBlock leaves by itself)
        const int top = seg_blocks > 1 && seg_blocks <= kSegBlock ? 1 : 0;
        hipLaunchKernelGGL(k_seg_build, dim3((uint32_t)seg_blocks), dim3(kSegThreads), 0, st, t.hdr, t.vals, t.v,
                           t.tris_s, t.first_idx, t.dup_cnt, t.fit_seg, cap, nn, top, t.prep_part + 8ull * kPrepBlocks + 1);
        if (!top && seg_blocks > 1) {
            uint64_t lsize = seg_blocks;   // capacity of level 10 (>= its valid entries)
            for (int L0 = kSegSteps; lsize > 1; L0 += kSegSteps) {
                hipLaunchKernelGGL(k_seg_up, dim3((uint32_t)((lsize + kSegBlock - 1) / kSegBlock)), dim3(kThreads), 0,
                                   st, t.hdr, t.fit_seg, cap, nn, L0);
                for (int s2 = 0; s2 < kSegSteps; ++s2) lsize = (lsize + 1) / 2;
            }
        }
        hipLaunchKernelGGL(k_fit, dim3(blocks_for(n)), dim3(kThreads), 0, st, t.hdr, t.fit_rng, t.children,
                           t.axis, t.fit_seg, cap, nn, t.clip, t.is_leaf, t.first_idx, t.dup_cnt, t.nodes, t.v,
                           t.vals, n, t.tris_s, t.hdr_host);
    }
    return hipGetLastError();
}

#undef BIH_TRY_H

// Allocates (first call) and runs the whole build on `stream`; synchronises
// at the end to read U back (Renderer.cpp:459 also reads the reduce_by_key
// end pointer on the host).
int build_tree_device(DeviceTree &t, void *stream, float *ms_out, bool sync) {
    hipStream_t st = (hipStream_t)stream;
    const uint32_t n = t.n;
    const uint64_t nn = n ? n : 1;
    const uint32_t rs_blocks = (uint32_t)((nn + kRsTile - 1) / kRsTile);
    const uint64_t hist_n = (uint64_t)kRdBins * rs_blocks;
    const uint32_t max_parts =
        (uint32_t)(((hist_n > nn + 1 ? hist_n : nn + 1) + kScanTile - 1) / kScanTile);
    if (!t.hdr) {
        // all or nothing: a failure part-way frees what was allocated, so
        // that the tree never holds a header without its buffers (the next
        // build of it allocates them again)
        const size_t bytes0 = t.bytes;
        const hipError_t e = alloc_build_buffers(t, nn, hist_n, max_parts, st);
        t.fail_alloc = 0;
        if (e != hipSuccess) {
            (void)hipStreamSynchronize(st);   // the memsets, if any were issued
            (void)hipGetLastError();          // not sticky for the next build
            if (t.graph) (void)hipGraphExecDestroy(t.graph);
            t.graph = nullptr;
            free_build_buffers(t);
            t.bytes = bytes0;
            return (int)e;
        }
    }
    // timing events and the pinned copy of the header: once per tree
    if (!t.ev0) {
        BIH_TRY(hipEventCreate(&t.ev0));
        BIH_TRY(hipEventCreate(&t.ev1));
        BIH_TRY(hipHostMalloc((void **)&t.hdr_host, sizeof(TreeHeader), hipHostMallocDefault));
    }
    BIH_TRY(hipEventRecord(t.ev0, st));

    // header reset (no triangles; otherwise k_morton's block 0 writes the header)
    if (n == 0) hipLaunchKernelGGL(k_hdr_init, dim3(1), dim3(64), 0, st, t.hdr, n);

    if (n > 0) {
        // The chain of ~15 dependent launches depends only on n and the tree's
        // buffers: captured once per tree buffer into a hipGraph and replayed
        // with one launch per build (host issue ~0.2 ms -> one call; the
        // look-back tags come from the device epoch, scan_tag).
        // BIH_BUILD_GRAPH=0: issued launch by launch (A/B).
        static const bool use_graph = [] {
            const char *e = getenv("BIH_BUILD_GRAPH");
            return !(e && e[0] == '0');
        }();
        if (use_graph) {
            if (t.graph && (t.graph_n != n || t.graph_v != t.v)) {
                (void)hipGraphExecDestroy(t.graph);
                t.graph = nullptr;
            }
            if (!t.graph && hipStreamBeginCapture(st, hipStreamCaptureModeRelaxed) != hipSuccess) {
                // (a stream that cannot be captured, e.g. the legacy default
                // stream: launch by launch)
                (void)hipGetLastError();
                BIH_TRY(issue_build(t, n, st));
            } else if (!t.graph) {
                hipGraph_t g = nullptr;
                const hipError_t ce = issue_build(t, n, st);
                const hipError_t ee = hipStreamEndCapture(st, &g);
                if (ce != hipSuccess || ee != hipSuccess) {
                    if (g) (void)hipGraphDestroy(g);
                    return (int)(ce != hipSuccess ? ce : ee);
                }
                const hipError_t ie = hipGraphInstantiate(&t.graph, g, nullptr, nullptr, 0);
                (void)hipGraphDestroy(g);
                if (ie != hipSuccess) {
                    t.graph = nullptr;
                    return (int)ie;
                }
                t.graph_n = n;
                t.graph_v = t.v;
            }
            if (t.graph) BIH_TRY(hipGraphLaunch(t.graph, st));
        } else {
            BIH_TRY(issue_build(t, n, st));
        }
    }
    BIH_TRY(hipEventRecord(t.ev1, st));
    // the header comes back through pinned host memory that k_fit's first
    // thread writes (no copy-engine transfer after the last kernel); a tree
    // without triangles takes the copy
    if (n == 0) BIH_TRY(hipMemcpyAsync(t.hdr_host, t.hdr, sizeof(TreeHeader), hipMemcpyDeviceToHost, st));
    if (!sync) return 0;
    BIH_TRY(hipStreamSynchronize(st));
    const TreeHeader h = *t.hdr_host;
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, t.ev0, t.ev1);
    if (ms_out) *ms_out = ms;
    t.u = h.n_unique;
    t.content = h.content;
    if (h.nonfinite) return -1000;   // mapped to BIH_ERR_NONFINITE by the C ABI
    return 0;
}

}  // namespace bih
