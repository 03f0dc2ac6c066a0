// bih_device.h -- device helpers shared by the render kernels
// (bih_render.hip) and the Whitted path (bih_whitted.hip).  Every f32
// expression is the reference's, in its order (compiled -ffp-contract=off).
#pragma once
#include "bih_internal.h"

namespace bih {
namespace dev {

constexpr float kDetEps = 9.99999997475242708e-07f;   // 0x358637bd: largest f32 < 1e-6
constexpr uint32_t kWeyl = 362437u;

// bih_rows: local row -> global row (include/bih.h)
__device__ __forceinline__ uint32_t global_row(uint32_t lr, uint32_t row0, uint32_t band_h,
                                               uint32_t band_step) {
    return row0 + (lr / band_h) * band_h * band_step + (lr % band_h);
}

// curand_uniform on XORWOW (cuRAND semantics restated, xorwow_host.cpp)
__device__ __forceinline__ float xorwow_uniform(uint32_t v[5], uint32_t &d) {
    uint32_t t = v[0] ^ (v[0] >> 2);
    v[0] = v[1]; v[1] = v[2]; v[2] = v[3]; v[3] = v[4];
    v[4] = (v[4] ^ (v[4] << 4)) ^ (t ^ (t << 1));
    d += kWeyl;
    uint32_t x = v[4] + d;
    return (float)x * 2.3283064e-10f + (2.3283064e-10f / 2.0f);   // _curand_uniform
}

// One XORWOW step without the float conversion: the 32-bit output
// (curand(), the word xorwow_uniform converts); same state update.
__device__ __forceinline__ uint32_t xorwow_next(uint32_t v[5], uint32_t &d) {
    uint32_t t = v[0] ^ (v[0] >> 2);
    v[0] = v[1]; v[1] = v[2]; v[2] = v[3]; v[3] = v[4];
    v[4] = (v[4] ^ (v[4] << 4)) ^ (t ^ (t << 1));
    d += kWeyl;
    return v[4] + d;
}
__device__ __forceinline__ float xorwow_to_uniform(uint32_t x) {
    return (float)x * 2.3283064e-10f + (2.3283064e-10f / 2.0f);   // _curand_uniform
}

// clamp + rgbToInt, CUDAKernels.cu:74-88
__device__ __forceinline__ uint32_t rgb_to_int(float r, float g, float b) {
    r = fmaxf(0.0f, fminf(255.0f, r));
    g = fmaxf(0.0f, fminf(255.0f, g));
    b = fmaxf(0.0f, fminf(255.0f, b));
    return ((uint32_t)(int)b << 16) | ((uint32_t)(int)g << 8) | (uint32_t)(int)r;
}

// Camera::GetRay direction, Camera.cu:18-20: ((llc + u*h) + v*vert) - origin
__device__ __forceinline__ void camera_dir(const RenderArgs &a, float u, float v, float &dx, float &dy,
                                           float &dz) {
    dx = ((a.cam[3] + u * a.cam[6]) + v * a.cam[9]) - a.cam[0];
    dy = ((a.cam[4] + u * a.cam[7]) + v * a.cam[10]) - a.cam[1];
    dz = ((a.cam[5] + u * a.cam[8]) + v * a.cam[11]) - a.cam[2];
}

// Primary-ray triangle record of one Morton-ordered triangle t = {v0, e1, e2}
// for camera origin O: {e1, e2, s = O - v0, q = cross(s, e1), tnum =
// dot(e2, q), 0, 0, 0} -- the ray-independent half of
// RayTriangleIntersection (CUDAKernels.cu:18-19, :33, :40, :47), computed
// once per origin instead of once per ray.  Returns tnum.
__device__ __forceinline__ float tri_prim_record(const float *__restrict__ t, float ox, float oy, float oz,
                                                 float *__restrict__ prim) {
    const float v0x = t[0], v0y = t[1], v0z = t[2];
    const float e1x = t[3], e1y = t[4], e1z = t[5];
    const float e2x = t[6], e2y = t[7], e2z = t[8];
    const float sx = ox - v0x, sy = oy - v0y, sz = oz - v0z;    // tvec
    const float qx = sy * e1z - e1y * sz;                       // qvec = cross(tvec, e1)
    const float qy = sz * e1x - e1z * sx;
    const float qz = sx * e1y - e1x * sy;
    const float tn = (e2x * qx + e2y * qy) + e2z * qz;          // dot(e2, qvec)
    float4 *o = reinterpret_cast<float4 *>(prim);
    o[0] = make_float4(e1x, e1y, e1z, e2x);
    o[1] = make_float4(e2y, e2z, sx, sy);
    o[2] = make_float4(sz, qx, qy, qz);
    o[3] = make_float4(tn, 0.f, 0.f, 0.f);
    return tn;
}

// A primary ray from O can hit a triangle only if its tnum is a positive
// finite f32: t = tnum * (1/det) with 1/det > 0 finite for every lane that
// passes the det test (CUDAKernels.cu:33-47), so tnum <= 0, +inf or NaN gives
// t <= 0, inf or NaN, and the t > 0 && t < FLT_MAX test fails for every ray.
__device__ __forceinline__ bool tnum_alive(float tn) {
    return __float_as_uint(tn) - 1u < 0x7f7fffffu;   // 0 < bits < 0x7f800000
}

// Decoupled look-back (single-pass scan): tile `tile` of a grid publishes its
// aggregate `tot`, adds its predecessors' published values walking back
// until one carries an inclusive prefix, publishes its own inclusive prefix
// and returns its exclusive prefix.  A status word is {tag:30 | flag:2 |
// value:32} (flag 1 = aggregate, 2 = inclusive prefix); the tag is unique
// per call (next_scan_tag), so the words need no memset between calls.
// Tiles are blockIdx.x: workgroups dispatch in id order, so every tile a
// block waits for is resident or done.  Flag and value share one 64-bit word:
// relaxed device-scope atomics suffice.  One thread of the block calls it.
constexpr uint32_t kScanAgg = 1u, kScanPre = 2u;
__device__ __forceinline__ unsigned long long scan_word(uint32_t tag, uint32_t flag, uint32_t v) {
    return ((unsigned long long)((tag << 2) | flag) << 32) | v;
}
__device__ __forceinline__ uint32_t lookback_prefix(unsigned long long *status, uint32_t tile, uint32_t tag,
                                                    uint32_t tot) {
    if (tile == 0) {
        __hip_atomic_store(status, scan_word(tag, kScanPre, tot), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return 0u;
    }
    __hip_atomic_store(status + tile, scan_word(tag, kScanAgg, tot), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    uint32_t prefix = 0;
    for (uint32_t j = tile - 1;;) {
        const unsigned long long w = __hip_atomic_load(status + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const uint32_t hi = (uint32_t)(w >> 32);
        if ((hi >> 2) != tag || (hi & 3u) == 0u) {
            __builtin_amdgcn_s_sleep(1);
            continue;
        }
        prefix += (uint32_t)w;
        if ((hi & 3u) == kScanPre) break;
        --j;
    }
    __hip_atomic_store(status + tile, scan_word(tag, kScanPre, prefix + tot), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
    return prefix;
}

// The same look-back by one whole wave (all 64 lanes call it, `lane` =
// 0..63; every lane returns the prefix): lane j reads predecessor j + 1 of
// the current window, so one round trip covers 64 predecessors.  The window
// sums the values of its leading run of published words up to the nearest
// inclusive prefix; an unpublished word (stale tag or flag 0) ends the run
// and the window restarts there.  Same words, same values as lookback_prefix.
__device__ __forceinline__ uint32_t lookback_prefix_wave(unsigned long long *status, uint32_t tile,
                                                         uint32_t tag, uint32_t tot, uint32_t lane) {
    if (tile == 0) {
        if (lane == 0)
            __hip_atomic_store(status, scan_word(tag, kScanPre, tot), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return 0u;
    }
    if (lane == 0)
        __hip_atomic_store(status + tile, scan_word(tag, kScanAgg, tot), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    uint32_t prefix = 0;
    uint32_t j = tile;   // predecessors j-1, j-2, .. remain (wave-uniform)
    for (;;) {
        const bool in = lane < j;
        unsigned long long w = 0ull;
        if (in) w = __hip_atomic_load(status + (j - 1u - lane), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const uint32_t hi = (uint32_t)(w >> 32);
        const bool ok = in && (hi >> 2) == tag && (hi & 3u) != 0u;
        const unsigned long long pre = __ballot(ok && (hi & 3u) == kScanPre);
        const unsigned long long bad = __ballot(!ok);   // lanes past tile 0 are never reached (tile 0 is a prefix)
        // lanes [0, end) are summed: up to the nearest prefix when none before it is unpublished
        const uint32_t fp = pre ? (uint32_t)__builtin_ctzll(pre) : 64u;
        const uint32_t fb = bad ? (uint32_t)__builtin_ctzll(bad) : 64u;
        const bool done = fp < fb;
        const uint32_t end = done ? fp + 1u : fb;
        uint32_t v = lane < end ? (uint32_t)w : 0u;
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
        prefix += v;
        if (done) break;
        j -= end;
        if (end == 0u) __builtin_amdgcn_s_sleep(1);
    }
    if (lane == 0)
        __hip_atomic_store(status + tile, scan_word(tag, kScanPre, prefix + tot), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    return prefix;
}

}  // namespace dev
}  // namespace bih
