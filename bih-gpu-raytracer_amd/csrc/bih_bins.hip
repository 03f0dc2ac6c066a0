// bih_bins.hip -- frustum bins: the any-hit walk's acceleration structure for
// rays that share one origin.
//
// Every primary ray of a frame starts at the camera origin O (Camera.cu:18-20)
// and its direction is fixed by the pixel and the jitter, so the triangles a
// sample can hit are the ones whose projection onto the image covers it.
// Per camera and image size, every alive triangle (tri_alive: tnum > 0, the
// only ones that can produce t > 0) gets a conservative pixel footprint, and
// every TW x TH pixel tile (one 64-ray packet of the render kernel) a list of
// the triangles whose footprint touches it:
//
//   footprint: the miss-proof bound (miss_bary, bih_bound.h) puts the point
//     where the exact line of an accepted ray meets the triangle's plane in an
//     inflated triangle with corners C_j (camera-relative, evaluated in f64
//     from the f32 record).  When all three corners lie in front of the image
//     plane (depth C_j . n > 0, n the camera's forward normal), that point has
//     t > 0 and its projection (u*, v*) lies in the projection of the inflated
//     triangle, the triangle of the projected corners.  The sample's own
//     (u, v) -- the kernel's f32 (x + r) / W -- and the f32 D differ from
//     (u*, v*) by ~1e-6 of the image: the footprint's pixel range is padded
//     by half a pixel on each side;
//   behind the camera: all corners at negative depth and tnum_c larger than
//     its rounding bound (exact t* has the sign of tnum* and det* > 0) --
//     no primary ray can hit the triangle: no footprint;
//   anything else (corners on both sides, no bound): the global list, tested
//     by every packet.
//
// A lane of a packet that tests every triangle of its tile's list and of the
// global list with the exact intersector and finds no hit has no triangle the
// intersector accepts: a proven miss of the reference walk.  A lane that finds
// one keeps it as a candidate; it stands only after fast_verify replays the
// reference's BIH decisions along the leaf's root path (bih_render.hip).
//
// List entries are 64-byte records {edge pre-test (9 f32), triangle, leaf}:
//   edge pre-test: MT accepting direction D implies (miss_bary) the exact
//     line's barycentrics u* >= -a, v* >= -b, u* + v* <= 1 + c, i.e. with
//     det* > 0: D.Gu >= 0, D.Gv >= 0, D.Gw >= 0 for Gu = Nu + a Nd,
//     Gv = Q + b Nd, Gw = (1 + c) Nd - Nu - Q, Nu = e2 x s, Nd = e2 x e1,
//     Q = s x e1 (exact, from the f32 record).  The kernel's f32 D is
//     A + u h + v vert + delta (A = lower_left - O, u and v the f32 values it
//     forms, |delta_i| <= 4e (|llc_i| + |h_i| + |vert_i| + |O_i|)), so
//     K0 + Ku u + Kv v >= -M with K0 = A.G, Ku = h.G, Kv = vert.G and
//     M >= |delta|.|G|; the record holds (K0 + M rounded up, Ku, Kv) per
//     edge with M also covering the f32 rounding of the K's and of the
//     kernel's fmaf evaluation (x4 margin).  A lane failing one edge cannot
//     be accepted by MT: the packet skips the triangle for it;
//   leaf: the leaf holding the triangle (the one fast_verify checks).
// Per leaf whose triangle's plan is the full check, the root path goes into a
// per-camera table of 32 8-byte steps {clip - O[axis] of the side taken,
// axis | side << 2}, end = 8 (16: path too deep, never verified), so that the
// check loads it without a dependent chain.
#include <hip/hip_runtime.h>
#include <float.h>
#include <math.h>
#include <stdlib.h>

#include "bih_internal.h"
#include "bih_bound.h"

namespace bih {
namespace {

constexpr int kThreads = 256;

__device__ __forceinline__ bool alive(const float *prim, uint32_t k) {
    const uint32_t b = __float_as_uint(prim[16ull * k + 12]);
    return b - 1u < 0x7f7fffffu;                 // 0 < tnum < +inf (tri_alive)
}

// r[13] = leaf of each Morton-ordered triangle (the leaf fast_verify checks)
__global__ void __launch_bounds__(kThreads) k_bin_leaf(const int32_t *__restrict__ first,
                                                       const uint32_t *__restrict__ cnt, uint32_t U,
                                                       float *__restrict__ prim) {
    const uint32_t k = blockIdx.x * kThreads + threadIdx.x;
    if (k >= U) return;
    const uint32_t b = (uint32_t)first[k], c = cnt[k];
    for (uint32_t i = b; i < b + c; ++i) prim[16ull * i + 13] = __uint_as_float(k);
}

__device__ __forceinline__ double dot3(const double *a, const double *b) {
    return a[0] * b[0] + a[1] * b[1] + a[2] * b[2];
}

__device__ __forceinline__ void cross3(const double *a, const double *b, double *o) {
    o[0] = a[1] * b[2] - a[2] * b[1];
    o[1] = a[2] * b[0] - a[0] * b[2];
    o[2] = a[0] * b[1] - a[1] * b[0];
}

// f32 >= x (x finite): rounded up
__device__ __forceinline__ float f32_up(double x) {
    float f = (float)x;
    if ((double)f < x) f = nextafterf(f, INFINITY);
    return f;
}

// The edge pre-test of one triangle (header comment): 3 x {K0 + M, Ku, Kv}.
__device__ __forceinline__ void edge_pretest(const float *rr, float a, float b, float cc,
                                             const BinCamera &c, float *out) {
    double e1[3], e2[3], sv[3];
    for (int k = 0; k < 3; ++k) {
        e1[k] = rr[k];
        e2[k] = rr[3 + k];
        sv[k] = rr[6 + k];
    }
    double Nu[3], Nd[3], Q[3], G[3][3];
    cross3(e2, sv, Nu);
    cross3(e2, e1, Nd);
    cross3(sv, e1, Q);
    for (int k = 0; k < 3; ++k) {
        G[0][k] = Nu[k] + (double)a * Nd[k];
        G[1][k] = Q[k] + (double)b * Nd[k];
        G[2][k] = (1.0 + (double)cc) * Nd[k] - Nu[k] - Q[k];
    }
    const double e = 0x1p-24;
    for (int j = 0; j < 3; ++j) {
        const double K0 = dot3(c.A, G[j]), Ku = dot3(c.hh, G[j]), Kv = dot3(c.vert, G[j]);
        const double dg = fabs(G[j][0]) * c.delta[0] + fabs(G[j][1]) * c.delta[1] +
                          fabs(G[j][2]) * c.delta[2];
        // |delta|.|G| (the f64 G errs by ~1e-16 relative), the K roundings
        // (e each) and the fmaf evaluation (2e of |K0'| + |Ku| + |Kv|, u, v
        // in [0, 1]); x4
        const double M = 4.0 * (dg + 8.0 * e * (fabs(K0) + fabs(Ku) + fabs(Kv)) + 1e-30);
        out[3 * j] = f32_up(K0 + M + 8.0 * e * M);
        out[3 * j + 1] = (float)Ku;
        out[3 * j + 2] = (float)Kv;
    }
}


// Which of the reference walk's decisions on the way to this triangle's
// leaf can go differently from the exact hit point's, for some ray the
// intersector accepts?  The answer replaces the root-path check
// (path_verify) with at most two comparisons carried in the list entry.
//
// The walk's decisions (path_step, root first) each compare two computed
// plane parameters t_p = fl(val_p * fl(1 / D[a_p])), val_p the
// camera-relative plane as the kernels hold it (f32): t_p = tau_p (1 + d),
// |d| <= 2.0001e, tau_p = val_p / D[a_p] exact.  A plane is an entry (the ray
// enters the child's region there) or an exit by the sign of D[a] -- that of
// X[a] over the whole inflated triangle when min|X[a]| > 0 (X = P - O,
// camera-relative hit point).  A node's entry plane is compared with the
// current hi, which is the t of the last exit plane above it (nhi = t,
// never a min) or the slab test's tMax; an exit plane with lo, the last
// entry plane's t or tMin.
//
// The exact line meets the triangle's plane at X inside the inflated
// triangle (corners X_j), at t* = X[a] / D[a] for every axis a.  Plane p
// has signed gap g_p(X) = val - X[a] ("X[a] <= val" side) or X[a] - val, so
// in t-units the separation minus rounding is (g_p - 2.0001e |val_p|) / |D[a]|
// and, divided by t*, >= h_p(X) / |X[a]| with h_p = g_p - 4e |val_p| (linear
// in X) >= L_p(X) = min(h_p / min|X[a]|, h_p / max|X[a]|) over the hull
// (-inf when the hull reaches X[a] = 0 and h_p < 0).  A comparison of p and
// k comes out as for the exact hit point (the child is visited) when
// L_p(X) + L_k(X) > 0; L_p + L_k is concave (sums of minima of linear
// functions), so it suffices at the three corners.  Against the slab test's
// tMin / tMax the smallest L over the faces that can be entries / exits is
// taken.  The leaf's parent plane is the triangle's own extreme coordinate
// and pokes through by the inflation near one vertex; its partner is
// usually far from that vertex.
//
// Plan (rec[11] = meta, rec[12..15] = vals, rec[10] bit 31 = no check):
//   n = meta & 3: 0 = every decision proven, 1-2 = that many critical
//   comparisons c, 3 = full root-path check (more than two, a plane of
//   either kind, val = 0 where 0 * inf = NaN, or a path deeper than 64);
//   comparison c: bits 2+6c: axis of k (2), k is an exit (1), axis of the
//   partner p (2), p is the slab's tMin / tMax (1); vals: val_k, val_p.
//   The kernel evaluates g = t_k > t_p (k exit) or !(t_k > t_p) (k entry),
//   as path_step does.
struct PlanL {
    double L[3];
};
// ramin / ramax: 1 / min|X[a]|, 1 / max|X[a]| over the hull (0: that bound
// is 0; the f64 reciprocal's rounding is far below the 4e margins)
__device__ __forceinline__ PlanL plane_l(const double (*X)[3], int ax, double val, bool le, double ramin,
                                         double ramax) {
    PlanL o;
    const double r = 4.0 * 0x1p-24 * fabs(val);
    for (int j = 0; j < 3; ++j) {
        const double h = (le ? val - X[j][ax] : X[j][ax] - val) - r;
        double m;
        if (h >= 0.0) m = ramax > 0.0 ? h * ramax : INFINITY;
        else m = ramin > 0.0 ? h * ramin : -INFINITY;
        o.L[j] = (m == m) ? m : -INFINITY;
    }
    return o;
}
__device__ uint32_t triangle_plan(const double (*X)[3], uint32_t leaf, const TreeHeader *hdr,
                                  const float *o, const uint4 *node_prim, const int32_t *leaf_parent,
                                  const int32_t *parent, float *vals) {
    constexpr uint32_t kFull = 3u;
    double amin[3], amax[3];
    int sgn[3];
    for (int ax = 0; ax < 3; ++ax) {
        const double lo = fmin(fmin(X[0][ax], X[1][ax]), X[2][ax]);
        const double hi = fmax(fmax(X[0][ax], X[1][ax]), X[2][ax]);
        const double mn = lo > 0.0 ? lo : (hi < 0.0 ? -hi : 0.0);
        const double mx = fmax(fabs(lo), fabs(hi));
        amin[ax] = mn > 0.0 ? 1.0 / mn : 0.0;   // reciprocals (plane_l)
        amax[ax] = mx > 0.0 ? 1.0 / mx : 0.0;
        sgn[ax] = lo > 0.0 ? 1 : (hi < 0.0 ? -1 : 0);
    }
    // slab faces: the smallest L over the faces that can be entries / exits
    PlanL slabE, slabX;
    for (int j = 0; j < 3; ++j) slabE.L[j] = slabX.L[j] = INFINITY;
    for (int ax = 0; ax < 3; ++ax)
        for (int f = 0; f < 2; ++f) {
            const bool le = f == 1;   // hi face: region X[a] <= hi - O
            const float v = le ? hdr->scene_hi[ax] - o[ax] : hdr->scene_lo[ax] - o[ax];
            if (v == 0.0f || !(v == v)) return kFull;
            const PlanL l = plane_l(X, ax, (double)v, le, amin[ax], amax[ax]);
            const bool can_exit = sgn[ax] == 0 || (le == (sgn[ax] > 0));
            const bool can_entry = sgn[ax] == 0 || !(le == (sgn[ax] > 0));
            for (int j = 0; j < 3; ++j) {
                if (can_entry) slabE.L[j] = fmin(slabE.L[j], l.L[j]);
                if (can_exit) slabX.L[j] = fmin(slabX.L[j], l.L[j]);
            }
        }
    // the root path, root first (Karras: leaf k lies left of node n iff
    // k <= split(n); every thread reads the top levels from cache), each
    // plane against the last plane of the other kind
    PlanL lastE = slabE, lastX = slabX;
    float lastEv = 0.0f, lastXv = 0.0f;
    uint32_t lastEa = 0, lastXa = 0;
    bool lastEslab = true, lastXslab = true;
    uint32_t meta = 0, nc = 0, node = 0;
    for (int depth = 0;; ++depth) {
        if (depth == 64) return kFull;
        const uint4 r = node_prim[node];
        const uint32_t split = r.z >> 8, ax = r.z & 0xffu;
        if (ax > 2u) return kFull;
        const bool le = leaf <= split;             // left child: region X[a] <= clip0 - O
        const bool child_leaf = le ? ((r.w >> 26) & 1u) != 0u : (r.w >> 31) != 0u;
        const float val = __uint_as_float(le ? r.x : r.y);
        if (sgn[ax] == 0 || val == 0.0f || !(val == val)) return kFull;
        const bool is_exit = le == (sgn[ax] > 0);
        const PlanL l = plane_l(X, ax, (double)val, le, amin[ax], amax[ax]);
        const PlanL &q = is_exit ? lastE : lastX;
        bool ok = true;
        for (int j = 0; j < 3; ++j) ok = ok && (l.L[j] + q.L[j] > 0.0);
        if (!ok) {
            if (nc == 2) return kFull;
            const bool qslab = is_exit ? lastEslab : lastXslab;
            const uint32_t qa = is_exit ? lastEa : lastXa;
            meta |= (ax | (is_exit ? 4u : 0u) | ((qslab ? 0u : qa) << 3) | (qslab ? 32u : 0u)) << (2 + 6 * nc);
            vals[2 * nc] = val;
            vals[2 * nc + 1] = qslab ? 0.0f : (is_exit ? lastEv : lastXv);
            ++nc;
        }
        if (is_exit) {
            lastX = l;
            lastXv = val;
            lastXa = ax;
            lastXslab = false;
        } else {
            lastE = l;
            lastEv = val;
            lastEa = ax;
            lastEslab = false;
        }
        const uint32_t child = le ? split : split + 1u;
        if (child_leaf) {
            if (child != leaf) return kFull;       // (a malformed tree: never)
            break;
        }
        node = child;
    }
    return meta | nc;
}

// Root path of leaf k as 32 steps root-first (header comment).  Written by
// k_bin_fp for the leaves of the entries whose plan is the full check (the
// only readers); several triangles of one leaf write the same values.
__device__ void write_path(const uint4 *__restrict__ node_prim, uint32_t k, uint2 *__restrict__ path) {
    uint2 *out = path + 32ull * k;
    uint32_t node = 0;
    for (int j = 0;; ++j) {
        if (j == 31) {
            out[0] = make_uint2(0u, 8u | 16u);   // too deep: never verified, the exact walk decides
            return;
        }
        const uint4 r = node_prim[node];
        const uint32_t split = r.z >> 8, axis = r.z & 0xffu;
        const bool le = k <= split;
        const uint32_t side = le ? 0u : 1u;
        out[j] = make_uint2(le ? r.x : r.y, axis | (side << 2));
        const bool child_leaf = le ? ((r.w >> 26) & 1u) != 0u : (r.w >> 31) != 0u;
        if (child_leaf) {
            out[j + 1] = make_uint2(0u, 8u);
            return;
        }
        node = le ? split : split + 1u;
    }
}

// The triangles a primary ray from the camera can hit (alive: 0 < tnum <
// inf; about half of a soup, the other half faces away), compacted in
// Morton order: k_bin_fp, k_bin_count and k_bin_fill run over this list, so
// their waves are not half idle.  Per-block counts (k_bin_alive_count), an
// exclusive scan, then the writes (k_bin_compact): one atomic per wave on a
// single counter cost 0.18 ms (the head-word limit of k_render_bins' queue).
// A dead triangle gets the empty footprint here.
__device__ __forceinline__ uint32_t block_alive(const float *prim, uint32_t n, uint32_t *s_w,
                                                unsigned long long &m, uint32_t &wave_off) {
    const uint32_t i = blockIdx.x * kThreads + threadIdx.x, lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
    const bool al = i < n && alive(prim, i);
    m = __ballot(al);
    if (lane == 0) s_w[w] = (uint32_t)__popcll(m);
    __syncthreads();
    uint32_t tot = 0;
    wave_off = 0;
    for (uint32_t k = 0; k < kThreads / 64; ++k) {
        if (k == w) wave_off = tot;
        tot += s_w[k];
    }
    return tot;
}
__global__ void __launch_bounds__(kThreads) k_bin_alive_count(float *__restrict__ prim, uint32_t n,
                                                              uint2 *__restrict__ brect,
                                                              uint32_t *__restrict__ bcnt) {
    __shared__ uint32_t s_w[kThreads / 64];
    const uint32_t i = blockIdx.x * kThreads + threadIdx.x;
    if (i < n && !alive(prim, i)) {
        brect[i] = make_uint2(1u, 0u);
        prim[16ull * i + 14] = __uint_as_float(1u);   // empty pixel range
        prim[16ull * i + 15] = __uint_as_float(1u);
    }
    unsigned long long m;
    uint32_t wo;
    const uint32_t tot = block_alive(prim, n, s_w, m, wo);
    if (threadIdx.x == 0) bcnt[blockIdx.x] = tot;
}
__global__ void __launch_bounds__(kThreads) k_bin_compact(const float *__restrict__ prim, uint32_t n,
                                                          const uint32_t *__restrict__ boff,
                                                          uint32_t *__restrict__ live) {
    __shared__ uint32_t s_w[kThreads / 64];
    const uint32_t i = blockIdx.x * kThreads + threadIdx.x, lane = threadIdx.x & 63u;
    unsigned long long m;
    uint32_t wo;
    (void)block_alive(prim, n, s_w, m, wo);
    if ((m >> lane) & 1ull) live[boff[blockIdx.x] + wo + (uint32_t)__popcll(m & ((1ull << lane) - 1ull))] = i;
}

// Footprint of triangle i: bin rectangle brect[i] (bx0 | bx1 << 16,
// by0 | by1 << 16; empty = bx0 > bx1), the pixel rectangle in r[14..15] and
// its list entry binrec[i]; the global list takes the rest.
__global__ void __launch_bounds__(kThreads) k_bin_fp(float *__restrict__ prim, uint32_t n,
                                                     BinCamera c, const TreeHeader *__restrict__ hdr,
                                                     const uint4 *__restrict__ node_prim,
                                                     const int32_t *__restrict__ leaf_parent,
                                                     const int32_t *__restrict__ parent,
                                                     uint2 *__restrict__ path, uint2 *__restrict__ brect,
                                                     float *__restrict__ binrec,
                                                     uint32_t *__restrict__ gcount,
                                                     uint32_t *__restrict__ glist,
                                                     const uint32_t *__restrict__ live,
                                                     const uint32_t *__restrict__ live_count) {
    const uint32_t j = blockIdx.x * kThreads + threadIdx.x;
    if (j >= *live_count) return;
    const uint32_t i = live[j];   // k_bin_compact
    float *r = prim + 16ull * i;
    const uint2 none = make_uint2(1u, 0u);
    if (!alive(prim, i)) {
        brect[i] = none;
        r[14] = __uint_as_float(1u);   // empty pixel range
        r[15] = __uint_as_float(1u);
        return;
    }
    float rr[13];
#pragma unroll
    for (int k = 0; k < 13; ++k) rr[k] = r[k];
    float a, b, cc;
    const bool ok = miss_bary(rr, c.dmax, a, b, cc);
    int side = 0;                      // 1: all in front, -1: all behind, 0: neither / no bound
    uint32_t plan = 3u;                // triangle_plan: 3 = full root-path check
    float plan_vals[4] = {0.0f, 0.0f, 0.0f, 0.0f};
    double umin = INFINITY, umax = -INFINITY, vmin = INFINITY, vmax = -INFINITY;
    if (ok) {
        // corners of the inflated triangle: depth and image (u, v)
        int front = 0, back = 0;
        double max_depth = 0.0;
        double cx[3][3];               // corners X_j (camera-relative)
        auto corners = [&](float a_, float b_, float c_) {
            const double cu[3] = {-(double)a_, 1.0 + (double)b_ + (double)c_, -(double)a_};
            const double cv[3] = {-(double)b_, -(double)b_, 1.0 + (double)a_ + (double)c_};
            front = back = 0;
            max_depth = 0.0;
            umin = vmin = INFINITY;
            umax = vmax = -INFINITY;
            for (int j = 0; j < 3; ++j) {
                double *X = cx[j];
                for (int ax = 0; ax < 3; ++ax)
                    X[ax] = (cu[j] * (double)rr[ax] + cv[j] * (double)rr[3 + ax]) - (double)rr[6 + ax];
                const double depth = dot3(X, c.n);
                const double mag = sqrt(dot3(X, X)) * c.nlen;
                if (depth > 1e-9 * mag) {
                    ++front;
                    max_depth = fmax(max_depth, depth);
                    // X = lambda (A + u h + v vert), lambda = depth / (A.n)
                    const double inv = c.an / depth;
                    const double u = dot3(X, c.hu) * inv - c.ahu;
                    const double v = dot3(X, c.vv) * inv - c.avv;
                    umin = fmin(umin, u);
                    umax = fmax(umax, u);
                    vmin = fmin(vmin, v);
                    vmax = fmax(vmax, v);
                } else if (depth < -1e-9 * mag) {
                    ++back;
                }
            }
        };
        corners(a, b, cc);
        if (front == 3) {
            // the inflated triangle lies in front of the camera: the exact det
            // of an accepted ray has a geometric lower bound (det_lower_bound),
            // usually far above 1e-6 -- a much tighter inflation, a smaller
            // footprint and a sharper pre-test (the refined triangle lies
            // inside the first, so it is still in front)
            const double L = det_lower_bound(rr, c.dn_lb, max_depth);
            if (L > 0.0) {
                float a2, b2, c2;
                if (miss_bary(rr, c.dmax, a2, b2, c2, (float)L) && a2 <= a && b2 <= b && c2 <= cc) {
                    a = a2;
                    b = b2;
                    cc = c2;
                    corners(a, b, cc);
                }
            }
        }
        if (front == 3) {
            side = 1;
            plan = triangle_plan(cx, __float_as_uint(r[13]), hdr, c.o, node_prim, leaf_parent, parent,
                                 plan_vals);
        } else if (back == 3) {
            // exact t* = tnum* / det* with det* > 0 (miss_bary's den); tnum_c
            // errs by at most 5e |e2|.Q (q_c = cross(s, e1): 2e Q, the dot
            // 3e): above 8e |e2|.Q its sign is exact, t* > 0, and the hit
            // point would have positive depth -- none lies behind
            const double as[3] = {fabs((double)rr[6]), fabs((double)rr[7]), fabs((double)rr[8])};
            const double ae1[3] = {fabs((double)rr[0]), fabs((double)rr[1]), fabs((double)rr[2])};
            const double Q[3] = {as[1] * ae1[2] + ae1[1] * as[2], as[2] * ae1[0] + ae1[2] * as[0],
                                 as[0] * ae1[1] + ae1[0] * as[1]};
            const double et = 8.0 * 0x1p-24 * (fabs((double)rr[3]) * Q[0] +
                                               fabs((double)rr[4]) * Q[1] +
                                               fabs((double)rr[5]) * Q[2]);
            if ((double)rr[12] > et) side = -1;
        }
    }
    if (side == -1) {
        brect[i] = none;
        r[14] = __uint_as_float(1u);
        r[15] = __uint_as_float(1u);
        return;
    }
    // the list entry: edge pre-test (or the always-passing one), triangle, leaf
    {
        float rec[16];
        if (ok) {
            edge_pretest(rr, a, b, cc, c, rec);
        } else {
            for (int j = 0; j < 3; ++j) {
                rec[3 * j] = INFINITY;
                rec[3 * j + 1] = 0.0f;
                rec[3 * j + 2] = 0.0f;
            }
        }
        rec[9] = __uint_as_float(i);
        rec[10] = __uint_as_float(__float_as_uint(r[13]) | (plan == 0u ? 0x80000000u : 0u));
        rec[11] = __uint_as_float(plan);
#ifndef BIH_FAST_COUNTERS
#define BIH_FAST_COUNTERS 0
#endif
        // counter builds check every plan against the root-path check: all paths
        if (plan == 3u || BIH_FAST_COUNTERS) write_path(node_prim, __float_as_uint(r[13]), path);
        for (int k = 0; k < 4; ++k) rec[12 + k] = plan_vals[k];
        float4 *o = reinterpret_cast<float4 *>(binrec + 16ull * i);
        for (int k = 0; k < 4; ++k) o[k] = make_float4(rec[4 * k], rec[4 * k + 1], rec[4 * k + 2], rec[4 * k + 3]);
    }
    if (side == 0) {                   // every packet tests it
        brect[i] = none;
        r[14] = __uint_as_float(0xffff0000u);
        r[15] = __uint_as_float(0xffff0000u);
        glist[atomicAdd(gcount, 1u)] = i;
        return;
    }
    // pixel x holds the samples u in (x / W, (x + 1) / W]: pixels
    // [floor(W umin - 1/2) - 1, floor(W umax + 1/2)], clipped to the image
    const double W = (double)c.w, H = (double)c.h;
    const double fx0 = floor(fmax(fmin(umin * W - 0.5, 1e9), -1e9)) - 1.0;
    const double fx1 = floor(fmax(fmin(umax * W + 0.5, 1e9), -1e9));
    const double fy0 = floor(fmax(fmin(vmin * H - 0.5, 1e9), -1e9)) - 1.0;
    const double fy1 = floor(fmax(fmin(vmax * H + 0.5, 1e9), -1e9));
    if (!(fx1 >= 0.0 && fy1 >= 0.0 && fx0 <= W - 1.0 && fy0 <= H - 1.0)) {
        brect[i] = none;               // off the image
        r[14] = __uint_as_float(1u);
        r[15] = __uint_as_float(1u);
        return;
    }
    const uint32_t x0 = (uint32_t)fmax(fx0, 0.0), x1 = (uint32_t)fmin(fx1, W - 1.0);
    const uint32_t y0 = (uint32_t)fmax(fy0, 0.0), y1 = (uint32_t)fmin(fy1, H - 1.0);
    r[14] = __uint_as_float(x0 | ((x1 - x0) << 16));
    r[15] = __uint_as_float(y0 | ((y1 - y0) << 16));
    brect[i] = make_uint2((x0 / c.tw) | ((x1 / c.tw) << 16), (y0 / c.th) | ((y1 / c.th) << 16));
}

// Tile (bx, by) against a triangle's edge pre-test (k0..k8 = 3 x {K0', Ku,
// Kv}, the kernel evaluates fmaf(Kv, v, fmaf(Ku, u, K0'))): 0 = no sample of
// the tile passes all three edges (the triangle stays off the tile's list),
// 2 = every sample passes (listed first: it most likely hits every lane),
// 1 = otherwise.  A sample of pixel x has u = fl(fl(x + r) / W), r in (0, 1]:
// u in [x / W, (x + 1) / W] up to 2 roundings (|u| <= 1; padded 2^-20).  Over
// the tile's (u, v) rectangle the affine function ranges over [lo, hi]
// (f64, exact enough); the kernel's two fmaf roundings err by at most
// 2e (|K0'| + |Ku| + |Kv|), taken 4e (sl).  NaN / inf coefficients never
// exclude a tile.
__device__ __forceinline__ int tile_class(const float4 r0, const float4 r1, const float4 r2,
                                          uint32_t bx, uint32_t by, uint32_t w, uint32_t h,
                                          uint32_t tw, uint32_t th) {
    const double pad = 0x1p-20;
    // x / W as x * (1 / W): off by ~1e-16, far inside the pad
    const double iw = 1.0 / (double)w, ih = 1.0 / (double)h;
    const uint32_t xe = (bx + 1) * tw < w ? (bx + 1) * tw : w;
    const uint32_t ye = (by + 1) * th < h ? (by + 1) * th : h;
    const double u0 = (double)(bx * tw) * iw - pad, u1 = (double)xe * iw + pad;
    const double v0 = (double)(by * th) * ih - pad, v1 = (double)ye * ih + pad;
    const float k[9] = {r0.x, r0.y, r0.z, r0.w, r1.x, r1.y, r1.z, r1.w, r2.x};
    bool all = true;
#pragma unroll
    for (int j = 0; j < 3; ++j) {
        const double K0 = k[3 * j], Ku = k[3 * j + 1], Kv = k[3 * j + 2];
        const double sl = 0x1p-22 * (fabs(K0) + fabs(Ku) + fabs(Kv));
        const double hi = K0 + fmax(Ku * u0, Ku * u1) + fmax(Kv * v0, Kv * v1);
        const double lo = K0 + fmin(Ku * u0, Ku * u1) + fmin(Kv * v0, Kv * v1);
        if (hi < -sl) return 0;
        if (!(lo > sl)) all = false;
    }
    return all ? 2 : 1;
}

// Pixel mask of a 4 x 4-pixel tile against a triangle's edge pre-test: bit
// 4 * row + col is clear only when no sample of that pixel can pass all
// three edges (tile_class's test on the pixel's own rectangle).  The list
// walk skips an entry for a packet whose remaining lanes all sit in pixels
// outside its mask.  Other tile shapes: all ones.
__device__ __forceinline__ uint32_t pixel_mask(const float4 r0, const float4 r1, const float4 r2,
                                               uint32_t bx, uint32_t by, uint32_t w, uint32_t h,
                                               uint32_t tw, uint32_t th) {
    if (tw != 4u || th != 4u) return 0xFFFFu;
    const float k[9] = {r0.x, r0.y, r0.z, r0.w, r1.x, r1.y, r1.z, r1.w, r2.x};
    // NaN coefficients never exclude a pixel
    if (!(k[0] == k[0] && k[3] == k[3] && k[6] == k[6])) return 0xFFFFu;
    const double pad = 0x1p-20;
    const double iw = 1.0 / (double)w, ih = 1.0 / (double)h;
    // the affine edge function's largest value over pixel (px, py)'s (u, v)
    // rectangle is K0 + cu[px] + cv[py] (the same f64 expressions, in the
    // same order, as tile_class on the pixel's rectangle): 8 products per edge
    // instead of 16 rectangles
    uint32_t m = 0xFFFFu;
#pragma unroll
    for (int e = 0; e < 3; ++e) {
        const double K0 = k[3 * e], Ku = k[3 * e + 1], Kv = k[3 * e + 2];
        const double sl = 0x1p-22 * (fabs(K0) + fabs(Ku) + fabs(Kv));
        double cu[4], cv[4];
#pragma unroll
        for (uint32_t j = 0; j < 4u; ++j) {
            const uint32_t x = bx * 4u + j, y = by * 4u + j;
            const double u0 = (double)x * iw - pad, u1 = (double)(x + 1u) * iw + pad;
            const double v0 = (double)y * ih - pad, v1 = (double)(y + 1u) * ih + pad;
            cu[j] = fmax(Ku * u0, Ku * u1);
            cv[j] = fmax(Kv * v0, Kv * v1);
        }
#pragma unroll
        for (uint32_t py = 0; py < 4u; ++py)
#pragma unroll
            for (uint32_t px = 0; px < 4u; ++px)
                if (K0 + cu[px] + cv[py] < -sl) m &= ~(1u << (4u * py + px));
    }
    return m;
}

// A lane walks its own triangle's tile rectangle when it has at most
// kBigRect tiles; larger rectangles (triangles close to the camera or seen
// edge-on) are walked by the whole wave afterwards, 64 tiles at a time, so
// one big footprint does not hold up its wave.
constexpr uint32_t kBigRect = 32;
// Lane j takes the j-th alive triangle (k_bin_compact's list).
template <typename F>
__device__ __forceinline__ void for_rect_tiles(const uint2 *__restrict__ brect, const uint32_t *__restrict__ live,
                                               const uint32_t *__restrict__ live_count, F &&visit) {
    const uint32_t j0 = blockIdx.x * kThreads + threadIdx.x, lane = threadIdx.x & 63u;
    const uint32_t nl = *live_count;
    uint2 q = make_uint2(1u, 0u);
    uint32_t i = 0;
    if (j0 < nl) {
        i = live[j0];
        q = brect[i];
    }
    uint32_t bx0 = q.x & 0xffffu, bx1 = q.x >> 16, by0 = q.y & 0xffffu, by1 = q.y >> 16;
    const bool any = j0 < nl && bx0 <= bx1;
    const uint32_t area = any ? (bx1 - bx0 + 1) * (by1 - by0 + 1) : 0u;
    if (any && area <= kBigRect)
        for (uint32_t by = by0; by <= by1; ++by)
            for (uint32_t bx = bx0; bx <= bx1; ++bx) visit(i, bx, by);
    unsigned long long big = __ballot(area > kBigRect);
    while (big) {
        const uint32_t j = (uint32_t)__builtin_ctzll(big);
        big &= big - 1ull;
        const uint32_t t = __builtin_amdgcn_readlane(i, j);
        const uint2 r = brect[t];
        const uint32_t x0 = r.x & 0xffffu, x1 = r.x >> 16, y0 = r.y & 0xffffu, y1 = r.y >> 16;
        const uint32_t wx = x1 - x0 + 1, na = wx * (y1 - y0 + 1);
        for (uint32_t k = lane; k < na; k += 64u) visit(t, x0 + k % wx, y0 + k / wx);
    }
}

// Counts per tile.  A block's alive triangles are Morton neighbours, so
// their footprints share tiles (bench: ~10 visits per tile per block): the
// block counts in LDS over the bounding rectangle of its footprints and
// adds each non-zero count to the tile's global counter once.  Blocks whose
// rectangle exceeds kCountLds tiles count with global atomics directly.
constexpr uint32_t kCountLds = 4096;
__global__ void __launch_bounds__(kThreads) k_bin_count(const uint2 *__restrict__ brect,
                                                        const uint32_t *__restrict__ live,
                                                        const uint32_t *__restrict__ live_count,
                                                        uint32_t bins_x, const float4 *__restrict__ binrec,
                                                        uint32_t w, uint32_t h, uint32_t tw, uint32_t th,
                                                        uint32_t *__restrict__ cnt,
                                                        unsigned long long *__restrict__ total64) {
    __shared__ uint32_t s_cnt[kCountLds];
    __shared__ uint32_t s_rect[4];   // x0, x1, y0, y1 of the block's footprints
    __shared__ unsigned long long s_tot;   // the block's entries (64-bit: the list total may pass 2^32)
    const uint32_t tid = threadIdx.x, j0 = blockIdx.x * kThreads + tid;
    if (tid == 0) {
        s_rect[0] = s_rect[2] = 0xffffu;
        s_rect[1] = s_rect[3] = 0u;
        s_tot = 0ull;
    }
    __syncthreads();
    {
        const uint32_t nl = *live_count;
        if (j0 < nl) {
            const uint2 q = brect[live[j0]];
            const uint32_t bx0 = q.x & 0xffffu, bx1 = q.x >> 16, by0 = q.y & 0xffffu, by1 = q.y >> 16;
            if (bx0 <= bx1) {
                atomicMin(&s_rect[0], bx0);
                atomicMax(&s_rect[1], bx1);
                atomicMin(&s_rect[2], by0);
                atomicMax(&s_rect[3], by1);
            }
        }
    }
    __syncthreads();
    const uint32_t rx0 = s_rect[0], rx1 = s_rect[1], ry0 = s_rect[2], ry1 = s_rect[3];
    const uint32_t rw = rx1 - rx0 + 1;
    const bool use_lds = rx0 <= rx1 && (uint64_t)rw * (ry1 - ry0 + 1) <= kCountLds;   // block-uniform
    const uint32_t rarea = use_lds ? rw * (ry1 - ry0 + 1) : 0u;
    for (uint32_t k = tid; k < rarea; k += kThreads) s_cnt[k] = 0u;
    __syncthreads();
    unsigned long long mine = 0ull;
    for_rect_tiles(brect, live, live_count, [&](uint32_t i, uint32_t bx, uint32_t by) {
        const float4 r0 = binrec[4ull * i], r1 = binrec[4ull * i + 1], r2 = binrec[4ull * i + 2];
        if (!tile_class(r0, r1, r2, bx, by, w, h, tw, th)) return;
        ++mine;
        if (use_lds) atomicAdd(&s_cnt[(by - ry0) * rw + (bx - rx0)], 1u);
        else atomicAdd(cnt + by * bins_x + bx, 1u);
    });
    if (mine) atomicAdd(&s_tot, mine);
    __syncthreads();
    for (uint32_t k = tid; k < rarea; k += kThreads) {
        const uint32_t c = s_cnt[k];
        if (c) atomicAdd(cnt + (ry0 + k / rw) * bins_x + rx0 + k % rw, c);
    }
    if (tid == 0 && s_tot) atomicAdd(total64, s_tot);
}

// A thread per triangle copies its 64-byte entry into each of its tiles'
// lists: every-sample entries from the front (fill), the others from the
// back (fill2, the per-tile counts, counted down: no second memset), so a
// packet meets the triangles that cover its whole tile first.  The order
// within each part follows the atomics (it can change which candidate a
// lane verifies, never a pixel).  Positions stay per-entry global atomics:
// taking them from per-block LDS cursors (as k_bin_count counts) made the
// fill 0.20 -> 0.13 ms but the render 1 % slower (A/B on one box,
// 0.0938 vs 0.0929 ms/frame): the block-grouped list order costs more per
// frame than it saves per camera.
__global__ void __launch_bounds__(kThreads) k_bin_fill(const uint2 *__restrict__ brect,
                                                       const uint32_t *__restrict__ live,
                                                       const uint32_t *__restrict__ live_count,
                                                       uint32_t bins_x, uint32_t w, uint32_t h,
                                                       uint32_t tw, uint32_t th,
                                                       const uint32_t *__restrict__ off,
                                                       uint32_t *__restrict__ fill,
                                                       uint32_t *__restrict__ fill2,
                                                       const float4 *__restrict__ binrec,
                                                       const uint32_t *__restrict__ gstat,
                                                       float4 *__restrict__ list) {
    if (*gstat == kBinsUnusable) return;   // the lists would not fit: the render falls back
    for_rect_tiles(brect, live, live_count, [&](uint32_t i, uint32_t bx, uint32_t by) {
        const float4 r0 = binrec[4ull * i], r1 = binrec[4ull * i + 1], r2 = binrec[4ull * i + 2];
        const int cls = tile_class(r0, r1, r2, bx, by, w, h, tw, th);
        if (!cls) return;
        const uint32_t b = by * bins_x + bx;
        // fill: front cursors (zeroed); fill2: the counts k_bin_count left,
        // counted down (off[b] + count - 1 = off[b + 1] - 1 first)
        const uint32_t pos = cls == 2 ? off[b] + atomicAdd(fill + b, 1u)
                                      : off[b] + atomicSub(fill2 + b, 1u) - 1u;
        // the entry's word 11: plan meta (bits 0-13) | pixel mask << 16
        const uint32_t pm = cls == 2 ? 0xFFFFu : pixel_mask(r0, r1, r2, bx, by, w, h, tw, th);
        float4 *o = list + 4ull * pos;
        o[0] = r0;
        o[1] = r1;
        o[2] = make_float4(r2.x, r2.y, r2.z, __uint_as_float((__float_as_uint(r2.w) & 0xFFFFu) | (pm << 16)));
        o[3] = binrec[4ull * i + 3];
    });
}

// The global list's entries (the same 64-byte records); gstat as k_bin_status
// left it (a grid over kBinGlobalMax entries: no host copy of the count).
__global__ void __launch_bounds__(kThreads) k_bin_gfill(const uint32_t *__restrict__ gstat,
                                                        const uint32_t *__restrict__ glist,
                                                        const float4 *__restrict__ binrec,
                                                        float4 *__restrict__ gent) {
    const uint32_t j = blockIdx.x * kThreads + threadIdx.x;
    const uint32_t gn = *gstat;
    if (gn == kBinsUnusable || j >= gn) return;
    const uint32_t i = glist[j];
    for (int k = 0; k < 4; ++k) gent[4ull * j + k] = binrec[4ull * i + k];
    const float4 r2 = binrec[4ull * i + 2];   // every pixel of every tile
    gent[4ull * j + 2] = make_float4(r2.x, r2.y, r2.z, __uint_as_float(__float_as_uint(r2.w) | 0xFFFF0000u));
}

// The bins' device status word (gstat = gcount + 1, RenderArgs::bin_gstat):
// the global list length when the lists fit `cap` entries and the global list
// kBinGlobalMax, else kBinsUnusable -- k_bin_fill then writes nothing and the
// render hands every live packet to the exact walk (k_render_fallback).  With
// it the lists are built without a host round trip; the host reads {gcount,
// gstat, total} back later (bih_capi.cpp: resolve_bins) and regrows.
// The total is k_bin_count's 64-bit sum (g[4..5]), not the u32 scan's, so a
// list total past 2^32 (whose u32 offsets wrapped) is unusable too.
__global__ void k_bin_status(uint32_t *__restrict__ g, uint32_t cap) {
    if (threadIdx.x != 0) return;
    const unsigned long long tot = *reinterpret_cast<const unsigned long long *>(g + 4);
    const uint32_t gc = g[0];
    g[1] = (tot <= cap && gc <= kBinGlobalMax) ? gc : kBinsUnusable;
    g[2] = tot > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)tot;
}

// Work queue of one launch's tiles (local tile ids t = ty * tiles_x + tx of
// its rows, bih_rows), in kRegions bands of tile rows, one per XCD (the
// render kernel's waves on XCD x draw from band x first, then from the
// others): per band the tiles with a non-empty list, by descending list
// length in power-of-two classes (longest processing time first), then the
// tiles no triangle touches (background).  Built once per camera, image and
// row set (bih_render.hip draws from it).
constexpr uint32_t kQBands = 8, kQClasses = 34;   // classes 0..32: clz(length); 33: background
__device__ __forceinline__ uint32_t queue_bin(uint32_t t, uint32_t tiles_x, uint32_t row0,
                                              uint32_t band_h, uint32_t band_step, uint32_t th,
                                              uint32_t bins_x) {
    const uint32_t ty = t / tiles_x, tx = t - ty * tiles_x;
    const uint32_t lr = ty * th;
    const uint32_t gy = row0 + (lr / band_h) * band_h * band_step + (lr % band_h);
    return (gy / th) * bins_x + tx;
}
// qw: [0, 272) class counts, [288, 560) class starts, [576, 848) fill
// cursors, [896, 928) per band {start, live, background, items}
__global__ void __launch_bounds__(kThreads) k_queue_class(const uint32_t *__restrict__ off,
                                                          const uint32_t *__restrict__ gstat,
                                                          uint32_t ntiles, uint32_t tiles_x,
                                                          uint32_t tiles_y, uint32_t row0,
                                                          uint32_t band_h, uint32_t band_step,
                                                          uint32_t th, uint32_t bins_x, uint32_t lpt,
                                                          uint16_t *__restrict__ cls,
                                                          uint32_t *__restrict__ qw) {
    // class counts aggregated per block in LDS: one global atomic per class
    // present (a tile row band has a handful), not one per tile
    __shared__ uint32_t hist[kQBands * kQClasses];
    for (uint32_t k = threadIdx.x; k < kQBands * kQClasses; k += kThreads) hist[k] = 0;
    __syncthreads();
    const uint32_t t = blockIdx.x * kThreads + threadIdx.x;
    if (t < ntiles) {
        const uint32_t b = queue_bin(t, tiles_x, row0, band_h, band_step, th, bins_x);
        // unusable bins: every tile live (the render hands them to the exact walk)
        const uint32_t g = *gstat, gn = g == kBinsUnusable ? 1u : g;
        const uint32_t len = off[b + 1] - off[b] + gn;
        const uint32_t band = (uint32_t)(((uint64_t)(t / tiles_x) * kQBands) / tiles_y);
        const uint32_t k = band * kQClasses + (len ? (lpt ? (uint32_t)__clz(len) : 0u) : kQClasses - 1);
        cls[t] = (uint16_t)k;
        atomicAdd(&hist[k], 1u);
    }
    __syncthreads();
    for (uint32_t k = threadIdx.x; k < kQBands * kQClasses; k += kThreads)
        if (hist[k]) atomicAdd(qw + k, hist[k]);
}
__global__ void __launch_bounds__(kThreads) k_queue_scan(uint32_t *__restrict__ qw) {
    // one block: the counts to LDS in one parallel load, band totals and
    // starts from LDS, then each band's class starts (a serial chain of
    // global loads took 19 us)
    __shared__ uint32_t c[kQBands * kQClasses], bstart[kQBands + 1];
    const uint32_t t = threadIdx.x;
    for (uint32_t k = t; k < kQBands * kQClasses; k += kThreads) c[k] = qw[k];
    __syncthreads();
    if (t == 0) {
        uint32_t acc = 0;
        for (uint32_t b = 0; b < kQBands; ++b) {
            bstart[b] = acc;
            for (uint32_t k = 0; k < kQClasses; ++k) acc += c[b * kQClasses + k];
        }
        bstart[kQBands] = acc;
    }
    __syncthreads();
    if (t < kQBands) {
        const uint32_t b = t, start = bstart[b];
        uint32_t acc = start;
        for (uint32_t k = 0; k < kQClasses; ++k) {
            qw[288 + b * kQClasses + k] = acc;
            qw[576 + b * kQClasses + k] = 0;
            acc += c[b * kQClasses + k];
        }
        const uint32_t bg = c[b * kQClasses + kQClasses - 1];
        const uint32_t live = acc - start - bg;
        qw[896 + 4 * b] = start;
        qw[896 + 4 * b + 1] = live;
        qw[896 + 4 * b + 2] = bg;
        qw[896 + 4 * b + 3] = live + (bg + 63u) / 64u;
    }
}
__global__ void __launch_bounds__(kThreads) k_queue_fill(const uint16_t *__restrict__ cls, uint32_t ntiles,
                                                         uint32_t *__restrict__ qw,
                                                         uint32_t *__restrict__ queue) {
    // ranks within the block by LDS atomics, then one global reservation per
    // class present
    __shared__ uint32_t hist[kQBands * kQClasses], base[kQBands * kQClasses];
    for (uint32_t k = threadIdx.x; k < kQBands * kQClasses; k += kThreads) hist[k] = 0;
    __syncthreads();
    const uint32_t t = blockIdx.x * kThreads + threadIdx.x;
    uint32_t k = 0, r = 0;
    if (t < ntiles) {
        k = cls[t];
        r = atomicAdd(&hist[k], 1u);
    }
    __syncthreads();
    for (uint32_t j = threadIdx.x; j < kQBands * kQClasses; j += kThreads)
        if (hist[j]) base[j] = qw[288 + j] + atomicAdd(qw + 576 + j, hist[j]);
    __syncthreads();
    if (t < ntiles) queue[base[k] + r] = t;
}

}  // namespace

bool bin_camera(const float cam[12], const float dmax[3], uint32_t w, uint32_t h, uint32_t tw,
                uint32_t th, BinCamera *out) {
    const double O[3] = {cam[0], cam[1], cam[2]};
    double A[3], hh[3], vv[3];
    for (int k = 0; k < 3; ++k) {
        A[k] = (double)cam[3 + k] - O[k];
        hh[k] = cam[6 + k];
        vv[k] = cam[9 + k];
    }
    auto cross = [](const double *a, const double *b, double *o) {
        o[0] = a[1] * b[2] - a[2] * b[1];
        o[1] = a[2] * b[0] - a[0] * b[2];
        o[2] = a[0] * b[1] - a[1] * b[0];
    };
    auto dot = [](const double *a, const double *b) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; };
    double n[3];
    cross(hh, vv, n);
    const double nl = sqrt(dot(n, n)), al = sqrt(dot(A, A));
    if (!(nl > 0.0) || !(al > 0.0) || !std::isfinite(nl) || !std::isfinite(al)) return false;
    double an = dot(A, n);
    if (an < 0.0) {
        for (double &x : n) x = -x;
        an = -an;
    }
    // every ray direction must point clearly into the front half-space (D.n
    // = A.n for every (u, v); the f32 D errs by ~1e-6 |D|)
    if (!(an > 1e-3 * nl * al)) return false;
    double vn[3], nh[3];
    cross(vv, n, vn);
    cross(n, hh, nh);
    const double hvn = dot(hh, vn), vnh = dot(vv, nh);
    if (!(fabs(hvn) > 0.0) || !(fabs(vnh) > 0.0)) return false;
    BinCamera c;
    for (int k = 0; k < 3; ++k) {
        c.n[k] = n[k];
        c.hu[k] = vn[k] / hvn;
        c.vv[k] = nh[k] / vnh;
        c.dmax[k] = dmax[k];
    }
    for (int k = 0; k < 3; ++k) {
        c.A[k] = A[k];
        c.hh[k] = hh[k];
        c.vert[k] = vv[k];
        // |f32 D - exact D(u, v)| per component (header comment): 4e, taken 8e
        c.delta[k] = 8.0 * 0x1p-24 * (fabs((double)cam[3 + k]) + fabs(hh[k]) + fabs(vv[k]) +
                                      fabs(O[k]));
    }
    c.nlen = nl;
    c.an = an;
    for (int k = 0; k < 3; ++k) c.o[k] = cam[k];
    // D.n = A.n exactly for D(u, v); the f32 D errs by delta per component
    c.dn_lb = an - 2.0 * (c.delta[0] * fabs(n[0]) + c.delta[1] * fabs(n[1]) + c.delta[2] * fabs(n[2]));
    c.ahu = dot(A, c.hu);
    c.avv = dot(A, c.vv);
    c.w = w;
    c.h = h;
    c.tw = tw;
    c.th = th;
    *out = c;
    return true;
}

int launch_bin_footprints(float *prim, uint32_t n, const TreeHeader *hdr, const int32_t *first_idx,
                          const uint32_t *dup_cnt,
                          const int32_t *leaf_parent, const int32_t *parent, const uint4 *node_prim,
                          uint32_t U, const BinCamera &c, const BinBuffers &b, void *stream) {
    const hipStream_t st = (hipStream_t)stream;
    const uint32_t nb = b.bins_x * b.bins_y;
    // gcount[0] = global list length, gcount[3] = alive triangles (k_bin_compact),
    // gcount[4..5] = the list total as a 64-bit sum (k_bin_count)
    hipError_t e = hipMemsetAsync(b.gcount, 0, 6 * sizeof(uint32_t), st);
    if (e == hipSuccess) e = hipMemsetAsync(b.cnt, 0, (size_t)nb * sizeof(uint32_t), st);
    if (e != hipSuccess) return (int)e;
    if (U > 0) {
        const dim3 g((U + kThreads - 1) / kThreads);
        hipLaunchKernelGGL(k_bin_leaf, g, dim3(kThreads), 0, st, first_idx, dup_cnt, U, prim);

    }
    if (n > 0) {
        const dim3 g((n + kThreads - 1) / kThreads);
        hipLaunchKernelGGL(k_bin_alive_count, g, dim3(kThreads), 0, st, prim, n, b.brect, b.bcnt);
        e = (hipError_t)scan_exclusive(b.bcnt, b.boff, g.x, b.bpart, b.gcount + 3, stream);
        if (e != hipSuccess) return (int)e;
        hipLaunchKernelGGL(k_bin_compact, g, dim3(kThreads), 0, st, prim, n, b.boff, b.live);
        hipLaunchKernelGGL(k_bin_fp, g, dim3(kThreads), 0, st, prim, n, c, hdr, node_prim, leaf_parent,
                           parent, b.path, b.brect, b.binrec, b.gcount,
                           b.glist, b.live, b.gcount + 3);
        hipLaunchKernelGGL(k_bin_count, g, dim3(kThreads), 0, st, b.brect, b.live, b.gcount + 3, b.bins_x,
                           reinterpret_cast<const float4 *>(b.binrec), c.w, c.h, c.tw, c.th, b.cnt,
                           reinterpret_cast<unsigned long long *>(b.gcount + 4));
    }
    e = hipGetLastError();
    if (e != hipSuccess) return (int)e;
    // off[nb] = the total (list length)
    return scan_exclusive(b.cnt, b.off, nb, b.partials, b.off + nb, stream);
}

int launch_bin_status(const BinBuffers &b, size_t cap, void *stream) {
    const uint32_t nb = b.bins_x * b.bins_y;
    (void)nb;
    hipLaunchKernelGGL(k_bin_status, dim3(1), dim3(64), 0, (hipStream_t)stream, b.gcount,
                       (uint32_t)(cap < 0xFFFFFFFFull ? cap : 0xFFFFFFFFull));
    return (int)hipGetLastError();
}

int launch_bin_fill(uint32_t n, const BinCamera &c, const BinBuffers &b, float *list, float *gent,
                    void *stream) {
    const hipStream_t st = (hipStream_t)stream;
    const uint32_t nb = b.bins_x * b.bins_y;
    const uint32_t *gstat = b.gcount + 1;
    hipError_t e = hipMemsetAsync(b.cnt2, 0, (size_t)nb * sizeof(uint32_t), st);
    if (e != hipSuccess) return (int)e;
    if (n > 0)
        hipLaunchKernelGGL(k_bin_fill, dim3((n + kThreads - 1) / kThreads), dim3(kThreads), 0, st,
                           b.brect, b.live, b.gcount + 3, b.bins_x, c.w, c.h, c.tw, c.th, b.off, b.cnt2, b.cnt,
                           reinterpret_cast<const float4 *>(b.binrec), gstat, reinterpret_cast<float4 *>(list));
    if (n > 0)
        hipLaunchKernelGGL(k_bin_gfill, dim3((kBinGlobalMax + kThreads - 1) / kThreads), dim3(kThreads), 0, st,
                           gstat, b.glist, reinterpret_cast<const float4 *>(b.binrec),
                           reinterpret_cast<float4 *>(gent));
    return (int)hipGetLastError();
}

size_t bin_queue_bytes(uint32_t ntiles) { return ((size_t)ntiles * 6 + 1024 * 4 + 255) & ~(size_t)255; }

int launch_bin_queue(const uint32_t *off, const uint32_t *gstat, uint32_t bins_x, uint32_t tiles_x, uint32_t ntiles,
                     uint32_t row0, uint32_t band_h, uint32_t band_step, uint32_t th, void *mem,
                     uint32_t **queue, uint32_t **qhdr, void *stream) {
    const hipStream_t st = (hipStream_t)stream;
    uint32_t *qw = reinterpret_cast<uint32_t *>(mem);
    uint32_t *q = qw + 1024;
    uint16_t *cls = reinterpret_cast<uint16_t *>(q + ntiles);
    *queue = q;
    *qhdr = qw + 896;
    hipError_t e = hipMemsetAsync(qw, 0, 1024 * sizeof(uint32_t), st);
    if (e != hipSuccess) return (int)e;
    const uint32_t tiles_y = tiles_x ? (ntiles + tiles_x - 1) / tiles_x : 0;
    // BIH_QUEUE_LPT=0: live tiles in tile order (A/B)
    static const uint32_t lpt = [] {
        const char *v = getenv("BIH_QUEUE_LPT");
        return (v && v[0] == '0') ? 0u : 1u;
    }();
    if (ntiles > 0) {
        const dim3 g((ntiles + kThreads - 1) / kThreads);
        hipLaunchKernelGGL(k_queue_class, g, dim3(kThreads), 0, st, off, gstat, ntiles, tiles_x, tiles_y, row0,
                           band_h, band_step, th, bins_x, lpt, cls, qw);
    }
    hipLaunchKernelGGL(k_queue_scan, dim3(1), dim3(kThreads), 0, st, qw);
    if (ntiles > 0)
        hipLaunchKernelGGL(k_queue_fill, dim3((ntiles + kThreads - 1) / kThreads), dim3(kThreads), 0, st, cls,
                           ntiles, qw, q);
    return (int)hipGetLastError();
}

}  // namespace bih
