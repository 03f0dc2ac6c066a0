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

}  // namespace dev
}  // namespace bih
