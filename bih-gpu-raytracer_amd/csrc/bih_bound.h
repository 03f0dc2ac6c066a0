// bih_bound.h -- the rounding bound of the primary-ray intersector shared by
// the any-hit walk's miss-proof boxes (bih_render.hip, miss_box) and the
// frustum bins (bih_bins.hip).
//
// For one alive triangle's primary-ray record r = {e1, e2, s = O - v0,
// q = cross(s, e1), tnum} (k_tri_prim) and dmax[] >= |D| per component for
// every primary ray of the camera: if the exact intersector
// (RayTriangleIntersection, CUDAKernels.cu:17-50, as the kernels evaluate it:
// f32, no contraction) returns a hit for direction D, the exact line O + t D
// meets the triangle's plane {O - s + u e1 + v e2} at barycentrics
//   u* >= -a,  v* >= -b,  u* + v* <= 1 + c,
// i.e. inside the triangle with barycentric corners (-a, -b), (1+b+c, -b),
// (-a, 1+a+c).  Proof sketch (unit roundoff e = 2^-24, first order): the
// f32 evaluation errs by at most
//   |p_c - p| <= 2e P,  P = (|dy||e2z| + |e2y||dz|, ...)   (abs cross product)
//   |un_c - s.p|   <= 5e |s|.P     =: Eu
//   |det_c - e1.p| <= 5e |e1|.P    =: Ed
//   |vn_c - D.q|   <= 5e |D|.Q     =: Ev,  Q = abs cross(|s|, |e1|)
// and a hit has det_c > 1e-6 (kDetEps), u_c in [0, 1], v_c >= 0,
// u_c + v_c <= 1, so with den = 0.99e-6 - Ed > 0: a = 4e + Eu/den,
// b = 4e + Ev/den, c = 8e + 1.01 (Eu + Ev + 2 Ed)/den.  The constants are
// taken 6e (BIH_MISS_E), not 5e: margin for the second-order terms and the
// f32 evaluation of the bound.  Returns false (no bound) for a non-finite
// bound or den <= 0.5e-6.  tests/test_miss_box.py checks the claim.
#pragma once

#ifndef BIH_MISS_E
#define BIH_MISS_E 6   // error constant in units of 2^-24 (the analysis gives 5)
#endif

namespace bih {

// den_lb > 0: a lower bound of the exact det over every ray the intersector
// accepts, known from elsewhere (the frustum bins' geometric bound, below);
// the larger of it and 0.99e-6 - Ed is used.
__device__ __forceinline__ bool miss_bary(const float *r, const float *dmax, float &a, float &bb,
                                          float &c, float den_lb = 0.0f) {
    const float E = (float)BIH_MISS_E * 0x1p-24f;
    const float ae1[3] = {fabsf(r[0]), fabsf(r[1]), fabsf(r[2])};
    const float ae2[3] = {fabsf(r[3]), fabsf(r[4]), fabsf(r[5])};
    const float as[3] = {fabsf(r[6]), fabsf(r[7]), fabsf(r[8])};
    const float P[3] = {dmax[1] * ae2[2] + ae2[1] * dmax[2], dmax[2] * ae2[0] + ae2[2] * dmax[0],
                        dmax[0] * ae2[1] + ae2[0] * dmax[1]};
    const float Q[3] = {as[1] * ae1[2] + ae1[1] * as[2], as[2] * ae1[0] + ae1[2] * as[0],
                        as[0] * ae1[1] + ae1[0] * as[1]};
    const float Eu = E * (as[0] * P[0] + as[1] * P[1] + as[2] * P[2]);
    const float Ed = E * (ae1[0] * P[0] + ae1[1] * P[1] + ae1[2] * P[2]);
    const float Ev = E * (dmax[0] * Q[0] + dmax[1] * Q[1] + dmax[2] * Q[2]);
    const float den0 = 0.99e-6f - Ed;
    const float den = den_lb > den0 ? den_lb : den0;
    a = 4.0f * E + Eu / den;
    bb = 4.0f * E + Ev / den;
    c = 8.0f * E + 1.01f * (Eu + Ev + 2.0f * Ed) / den;
    return den0 > 0.5e-6f && a < 1e30f && bb < 1e30f && c < 1e30f;
}

// A geometric lower bound of the exact det for the frustum bins.  Every
// primary ray shares the origin O and has D.n = A.n (n the camera's forward
// normal, A = lower_left - O; the f32 D deviates by delta, so D.n >= dn_lb).
// The exact line O + t D meets the triangle's plane at P with
// t det = tnum (the exact triple product s.(e1 x e2)) and depth(P) =
// (P - O).n = t D.n, so det = tnum D.n / depth(P).  When the intersector
// accepts D, P lies in the inflated triangle of miss_bary's 0.99e-6 - Ed
// bound; if its three corners have depth > 0, the largest of them bounds
// depth(P), and tnum >= tnum_c - 8e |e2|.Q (q_c = cross(s, e1) errs by
// 2e Q, the dot by 3e) gives
//   det >= (tnum_c - 8e |e2|.Q) dn_lb / max depth.
// A soup triangle seen face-on has det ~ 1e-3, three orders above the
// 1e-6 threshold, so the inflation (~ E / det) shrinks by as much.  Returns
// 0 when the bound does not apply.  tests/test_bin_pretest.py checks the
// refined inflation on near-edge-on triangles and a soup.
__device__ __forceinline__ double det_lower_bound(const float *r, double dn_lb, double max_depth) {
    const double as[3] = {fabs((double)r[6]), fabs((double)r[7]), fabs((double)r[8])};
    const double ae1[3] = {fabs((double)r[0]), fabs((double)r[1]), fabs((double)r[2])};
    const double Q[3] = {as[1] * ae1[2] + ae1[1] * as[2], as[2] * ae1[0] + ae1[2] * as[0],
                         as[0] * ae1[1] + ae1[0] * as[1]};
    const double et = 8.0 * 0x1p-24 * (fabs((double)r[3]) * Q[0] + fabs((double)r[4]) * Q[1] +
                                       fabs((double)r[5]) * Q[2]);
    const double tlb = (double)r[12] - et;
    if (!(tlb > 0.0) || !(dn_lb > 0.0) || !(max_depth > 0.0)) return 0.0;
    const double L = 0.99 * tlb * dn_lb / max_depth;   // 1 % for the f64 evaluation
    return (L < 1e30) ? L : 0.0;
}

}  // namespace bih
