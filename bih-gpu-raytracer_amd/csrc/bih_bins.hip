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
// List entries are 48-byte records {edge pre-test (9 f32), triangle, leaf, plan meta |
// pixel mask}; the plan values stay in the triangle's 64-byte record (binrec):
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
#include "bih_device.h"

namespace bih {
namespace {

constexpr int kThreads = 256;


// The camera's primary-ray records and its alive triangles (a thread per
// Morton-ordered triangle i and per internal node i):
//   - the triangle record (dev::tri_prim_record; bih_render.hip's k_tri_prim)
//     and the camera-relative node record (k_node_prim's, no culled set);
//   - which triangles a primary ray from the camera can hit (tnum_alive:
//     about half of a soup, the other half faces away): per block a 256-bit
//     mask and its count, for k_live_compact;
//   - zeroes the per-tile counters (zero[0 .. zero_words)) and the bins'
//     status words (gcount[0..2], [4..5]).
// (A decoupled look-back here made the kernel 0.08 ms instead of 0.03: 3900
// blocks waiting on their predecessors' status words.)
__global__ void __launch_bounds__(kThreads) k_cam_tris(const float *__restrict__ tris, uint32_t n,
                                                       float ox, float oy, float oz,
                                                       float *__restrict__ prim,
                                                       const uint4 *__restrict__ nodes, uint32_t m,
                                                       uint4 *__restrict__ node_out,
                                                       unsigned long long *__restrict__ bmask,
                                                       uint32_t *__restrict__ bcnt,
                                                       uint32_t *__restrict__ zero, uint32_t zero_words,
                                                       uint32_t *__restrict__ gcount) {
    __shared__ uint32_t s_w[kThreads / 64];
    const uint32_t i = blockIdx.x * kThreads + threadIdx.x, lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
    bool al = false;
    if (i < n) al = dev::tnum_alive(dev::tri_prim_record(tris + 9ull * i, ox, oy, oz, prim + 16ull * i));
    if (i < m) {
        const uint4 nd = nodes[i];
        const uint32_t ax = (nd.z >> 27) & 3u;
        const float org = ax == 0u ? ox : (ax == 1u ? oy : oz);
        const uint32_t split = nd.z & 0x7ffffffu;
        const uint32_t wd = nd.w | (((nd.z >> 29) & 1u) << 26) | (((nd.z >> 30) & 1u) << 31);
        node_out[i] = make_uint4(__float_as_uint(__uint_as_float(nd.x) - org),
                                 __float_as_uint(__uint_as_float(nd.y) - org), (split << 8) | ax, wd);
    }
    for (uint32_t k = i; k < zero_words; k += gridDim.x * kThreads) zero[k] = 0u;
    if (i == 0) {
        gcount[0] = gcount[1] = gcount[2] = 0u;
        gcount[4] = gcount[5] = 0u;
        gcount[6] = gcount[7] = 0u;   // pair-result positions (k_bin_count), 64-bit
    }
    const unsigned long long mk = __ballot(al);
    if (lane == 0) {
        s_w[w] = (uint32_t)__popcll(mk);
        bmask[4ull * blockIdx.x + w] = mk;
    }
    __syncthreads();
    if (threadIdx.x == 0) bcnt[blockIdx.x] = s_w[0] + s_w[1] + s_w[2] + s_w[3];
}

// live[] = the alive triangles in Morton order (boff = exclusive scan of
// k_cam_tris' block counts), so that k_bin_fp, k_bin_count and k_bin_fill
// run over whole waves of them.
__global__ void __launch_bounds__(kThreads) k_live_compact(const unsigned long long *__restrict__ bmask,
                                                           const uint32_t *__restrict__ boff,
                                                           uint32_t *__restrict__ live) {
    const uint32_t lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
    const unsigned long long *bm = bmask + 4ull * blockIdx.x;
    const unsigned long long mk = bm[w];
    if (!((mk >> lane) & 1ull)) return;
    uint32_t off = boff[blockIdx.x];
    for (uint32_t k = 0; k < w; ++k) off += (uint32_t)__popcll(bm[k]);
    live[off + (uint32_t)__popcll(mk & ((1ull << lane) - 1ull))] = blockIdx.x * kThreads + threadIdx.x;
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
// m(h) of plane_l: h / max|X[a]| (h >= 0) or h / min|X[a]| (h < 0), NaN -> -inf;
// nondecreasing in h
__device__ __forceinline__ double plane_m(double h, double ramin, double ramax) {
    double m;
    if (h >= 0.0) m = ramax > 0.0 ? h * ramax : INFINITY;
    else m = ramin > 0.0 ? h * ramin : -INFINITY;
    return (m == m) ? m : -INFINITY;
}
// ramin / ramax: 1 / min|X[a]|, 1 / max|X[a]| over the hull (0: that bound
// is 0; the f64 reciprocal's rounding is far below the 4e margins)
__device__ __forceinline__ PlanL plane_l(const double (*X)[3], int ax, double val, bool le, double ramin,
                                         double ramax) {
    PlanL o;
    const double r = 4.0 * 0x1p-24 * fabs(val);
    for (int j = 0; j < 3; ++j) o.L[j] = plane_m((le ? val - X[j][ax] : X[j][ax] - val) - r, ramin, ramax);
    return o;
}
// The smallest of plane_l's three values: the same expression at the corner
// with the extreme coordinate (xmax for le, xmin otherwise; fmax / fmin return
// one of the corners' own values), and fl and plane_m are monotone, so it is
// <= every corner's value.  With no NaN among the corners, lmin_p + lmin_q > 0
// (rounded: fl(a + b) is monotone too) implies every corner's
// L_p + L_q > 0, so triangle_plan tests the three corners only when this
// one-value test fails -- with the same outcome as testing them always.
__device__ __forceinline__ double plane_lmin(double xmin, double xmax, double val, bool le, double ramin,
                                             double ramax) {
    const double r = 4.0 * 0x1p-24 * fabs(val);
    return plane_m((le ? val - xmax : xmin - val) - r, ramin, ramax);
}
// TAB: the per-axis values the walk picks by the node's axis (1 / min|X[a]|,
// 1 / max|X[a]|, the corners' extent) come from a per-thread table in LDS
// (tab[k * kThreads], k = 4 axis + field) -- one LDS read each instead of a
// chain of selects over the three axes in registers.
template <bool TAB>
__device__ uint32_t triangle_plan(const double (*X)[3], uint32_t leaf, const TreeHeader *hdr,
                                  const float *o, const uint4 *node_prim, const int32_t *leaf_parent,
                                  const int32_t *parent, float *vals, double *tab) {
    constexpr uint32_t kFull = 3u;
#ifndef BIH_PLAN_LEAN
#define BIH_PLAN_LEAN 0   // 1: the corners' extent per axis recomputed per level, not kept (12 VGPRs; slower)
#endif
    double amin[3], amax[3];
#if !BIH_PLAN_LEAN
    double xlo[3], xhi[3];
#endif
    int sgn[3];
    bool finite_ok = true;   // no NaN corner coordinate: the one-value test is exact
    for (int ax = 0; ax < 3; ++ax) {
        const double lo = fmin(fmin(X[0][ax], X[1][ax]), X[2][ax]);
        const double hi = fmax(fmax(X[0][ax], X[1][ax]), X[2][ax]);
        finite_ok = finite_ok && X[0][ax] == X[0][ax] && X[1][ax] == X[1][ax] && X[2][ax] == X[2][ax];
#if !BIH_PLAN_LEAN
        xlo[ax] = lo;
        xhi[ax] = hi;
#endif
        const double mn = lo > 0.0 ? lo : (hi < 0.0 ? -hi : 0.0);
        const double mx = fmax(fabs(lo), fabs(hi));
        amin[ax] = mn > 0.0 ? 1.0 / mn : 0.0;   // reciprocals (plane_l)
        amax[ax] = mx > 0.0 ? 1.0 / mx : 0.0;
        sgn[ax] = lo > 0.0 ? 1 : (hi < 0.0 ? -1 : 0);
        if (TAB) {
            tab[(4 * ax + 0) * kThreads] = amin[ax];
            tab[(4 * ax + 1) * kThreads] = amax[ax];
            tab[(4 * ax + 2) * kThreads] = lo;
            tab[(4 * ax + 3) * kThreads] = hi;
        }
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
    // plane against the last plane of the other kind.  The last planes are
    // kept as {value, axis} plus their smallest L (plane_lmin); their three
    // corner values are recomputed (plane_l, the same values) only for a
    // comparison the one-value test does not settle.
    double lastEmin = fmin(fmin(slabE.L[0], slabE.L[1]), slabE.L[2]);
    double lastXmin = fmin(fmin(slabX.L[0], slabX.L[1]), slabX.L[2]);
    float lastEv = 0.0f, lastXv = 0.0f;
    uint32_t lastEa = 0, lastXa = 0;
    bool lastEslab = true, lastXslab = true;
    uint32_t meta = 0, nc = 0;
    // the next level's record is requested before this level's f64 work
    // (the walk is a chain of dependent loads)
    uint4 rn = node_prim[0];
    for (int depth = 0;; ++depth) {
        if (depth == 64) return kFull;
        const uint4 r = rn;
        const uint32_t split = r.z >> 8, ax = r.z & 0xffu;
        if (ax > 2u) return kFull;
        const bool le = leaf <= split;             // left child: region X[a] <= clip0 - O
        const bool child_leaf = le ? ((r.w >> 26) & 1u) != 0u : (r.w >> 31) != 0u;
        const uint32_t child = le ? split : split + 1u;
        if (!child_leaf) rn = node_prim[child];
        const float val = __uint_as_float(le ? r.x : r.y);
        if (sgn[ax] == 0 || val == 0.0f || !(val == val)) return kFull;
        const bool is_exit = le == (sgn[ax] > 0);
        double am, aM, lmin;
        if (TAB) {
            am = tab[(4 * ax + 0) * kThreads];
            aM = tab[(4 * ax + 1) * kThreads];
            lmin = plane_lmin(tab[(4 * ax + 2) * kThreads], tab[(4 * ax + 3) * kThreads], (double)val, le, am, aM);
        } else {
            am = amin[ax];
            aM = amax[ax];
#if BIH_PLAN_LEAN
        const double c0 = ax == 0u ? X[0][0] : (ax == 1u ? X[0][1] : X[0][2]);
        const double c1 = ax == 0u ? X[1][0] : (ax == 1u ? X[1][1] : X[1][2]);
        const double c2 = ax == 0u ? X[2][0] : (ax == 1u ? X[2][1] : X[2][2]);
        lmin = plane_lmin(fmin(fmin(c0, c1), c2), fmax(fmax(c0, c1), c2), (double)val, le, am, aM);
#else
        lmin = plane_lmin(xlo[ax], xhi[ax], (double)val, le, am, aM);
#endif
        }
        bool ok = finite_ok && lmin + (is_exit ? lastEmin : lastXmin) > 0.0;
        if (!ok) {
            // the three corners: this plane and the partner (the last plane
            // of the other kind: an entry plane has le = sgn < 0, an exit
            // plane le = sgn > 0)
            const PlanL l = plane_l(X, ax, (double)val, le, am, aM);
            const bool qslab = is_exit ? lastEslab : lastXslab;
            const uint32_t qa = is_exit ? lastEa : lastXa;
            PlanL q;
            if (qslab) {
                q = is_exit ? slabE : slabX;
            } else {
                const float qv = is_exit ? lastEv : lastXv;
                const bool qle = is_exit ? sgn[qa] < 0 : sgn[qa] > 0;
                q = TAB ? plane_l(X, qa, (double)qv, qle, tab[(4 * qa + 0) * kThreads], tab[(4 * qa + 1) * kThreads])
                        : plane_l(X, qa, (double)qv, qle, amin[qa], amax[qa]);
            }
            ok = true;
            for (int j = 0; j < 3; ++j) ok = ok && (l.L[j] + q.L[j] > 0.0);
            if (!ok) {
                if (nc == 2) return kFull;
                meta |= (ax | (is_exit ? 4u : 0u) | ((qslab ? 0u : qa) << 3) | (qslab ? 32u : 0u)) << (2 + 6 * nc);
                vals[2 * nc] = val;
                vals[2 * nc + 1] = qslab ? 0.0f : (is_exit ? lastEv : lastXv);
                ++nc;
            }
        }
        if (is_exit) {
            lastXmin = lmin;
            lastXv = val;
            lastXa = ax;
            lastXslab = false;
        } else {
            lastEmin = lmin;
            lastEv = val;
            lastEa = ax;
            lastEslab = false;
        }
        if (child_leaf) {
            if (child != leaf) return kFull;       // (a malformed tree: never)
            break;
        }
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

// BIH_FP_SPLIT: the verification plans (triangle_plan's f64 root-path walk,
// a chain of dependent node loads) run in k_bin_plan, a kernel of their own
// with fewer registers and so more waves to hide the chain's latency; k_bin_fp
// leaves (a, b, cc, 1) of each triangle in front of the camera in its
// record's plan slots (rec[12..15]; 0 = no plan).
#ifndef BIH_FP_SPLIT
#define BIH_FP_SPLIT 0   // 1: slower (0.027 + 0.073 ms with the LDS table vs 0.0965 in one kernel, r04y)
#endif
#ifndef BIH_FP_TAB
#define BIH_FP_TAB 1      // k_bin_fp's plan walk with triangle_plan<true> (LDS per-axis table): 0.0865 vs 0.0963 ms (r04z)
#endif
// Footprint of alive triangle i = live[j]: bin rectangle brect[i] (bx0 |
// bx1 << 16, by0 | by1 << 16; empty = bx0 > bx1) and its list entry
// binrec[i]; the global list takes the rest.  leaf = the leaf of each sorted
// triangle (DeviceTree::tri_leaf).
#ifndef BIH_FP_WAVES_PER_EU
#define BIH_FP_WAVES_PER_EU 0   // 0: the compiler's choice (128 VGPRs, 4 waves/SIMD)
#endif
#if BIH_FP_WAVES_PER_EU
#define BIH_FP_OCC __attribute__((amdgpu_waves_per_eu(BIH_FP_WAVES_PER_EU, BIH_FP_WAVES_PER_EU)))
#else
#define BIH_FP_OCC
#endif
__global__ void __launch_bounds__(kThreads) BIH_FP_OCC k_bin_fp(const float *__restrict__ prim, uint32_t n,
                                                     BinCamera c, const TreeHeader *__restrict__ hdr,
                                                     const uint4 *__restrict__ node_prim,
                                                     const uint32_t *__restrict__ tri_leaf,
                                                     const int32_t *__restrict__ leaf_parent,
                                                     const int32_t *__restrict__ parent,
                                                     uint2 *__restrict__ path, uint2 *__restrict__ brect,
                                                     float *__restrict__ binrec,
                                                     uint32_t *__restrict__ gcount,
                                                     uint32_t *__restrict__ glist,
                                                     const uint32_t *__restrict__ live,
                                                     const uint32_t *__restrict__ live_count) {
#if BIH_FP_TAB
    __shared__ double s_tab[12 * kThreads];
#endif
    const uint32_t j = blockIdx.x * kThreads + threadIdx.x;
    if (j >= *live_count) return;
    const uint32_t i = live[j];   // k_cam_tris
    const float *r = prim + 16ull * i;
    const uint32_t leaf = tri_leaf[i];
    const uint2 none = make_uint2(1u, 0u);
    float rr[13];
#pragma unroll
    for (int k = 0; k < 13; ++k) rr[k] = r[k];
    float a, b, cc;
    const bool ok = miss_bary(rr, c.dmax, a, b, cc);
    int side = 0;                      // 1: all in front, -1: all behind, 0: neither / no bound
    uint32_t plan = 3u;                // triangle_plan: 3 = full root-path check
    float plan_vals[4] = {0.0f, 0.0f, 0.0f, 0.0f};
    double umin = INFINITY, umax = -INFINITY, vmin = INFINITY, vmax = -INFINITY;
    float rec[16];
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
#ifndef BIH_FP_EXP
#define BIH_FP_EXP 0   // timing experiments only (wrong plans): 1 no plan walk, 2 no det refinement,
                       // 4 no edge pre-test, 8 no root paths
#endif
        if (front == 3 && !(BIH_FP_EXP & 2)) {
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
        if (side == -1) {
            brect[i] = none;
            return;
        }
        uint2 rect = none;
        if (side == 1) {
            // pixel x holds the samples u in (x / W, (x + 1) / W]: pixels
            // [floor(W umin - 1/2) - 1, floor(W umax + 1/2)], clipped to the image
            const double W = (double)c.w, H = (double)c.h;
            const double fx0 = floor(fmax(fmin(umin * W - 0.5, 1e9), -1e9)) - 1.0;
            const double fx1 = floor(fmax(fmin(umax * W + 0.5, 1e9), -1e9));
            const double fy0 = floor(fmax(fmin(vmin * H - 0.5, 1e9), -1e9)) - 1.0;
            const double fy1 = floor(fmax(fmin(vmax * H + 0.5, 1e9), -1e9));
            if (!(fx1 >= 0.0 && fy1 >= 0.0 && fx0 <= W - 1.0 && fy0 <= H - 1.0)) {
                brect[i] = none;       // off the image: never listed (no entry, no plan)
                return;
            }
            const uint32_t x0 = (uint32_t)fmax(fx0, 0.0), x1 = (uint32_t)fmin(fx1, W - 1.0);
            const uint32_t y0 = (uint32_t)fmax(fy0, 0.0), y1 = (uint32_t)fmin(fy1, H - 1.0);
            rect = make_uint2((x0 / c.tw) | ((x1 / c.tw) << 16), (y0 / c.th) | ((y1 / c.th) << 16));
        }
        // the edge pre-test now (rr, a, b, cc end here), the plan after
        if (!(BIH_FP_EXP & 4)) edge_pretest(rr, a, b, cc, c, rec);
#if BIH_FP_SPLIT
        // the plan is k_bin_plan's: it recomputes the corners from (a, b, cc)
        if (side == 1) {
            plan_vals[0] = a;
            plan_vals[1] = b;
            plan_vals[2] = cc;
            plan_vals[3] = 1.0f;
        }
#elif BIH_FP_EXP & 1
        plan = 1u;
#else
#if BIH_FP_TAB
        if (side == 1) plan = triangle_plan<true>(cx, leaf, hdr, c.o, node_prim, leaf_parent, parent, plan_vals,
                                                  s_tab + threadIdx.x);
#else
        if (side == 1) plan = triangle_plan<false>(cx, leaf, hdr, c.o, node_prim, leaf_parent, parent, plan_vals, nullptr);
#endif
#endif
        brect[i] = rect;
    } else {
        // no bound: the always-passing pre-test, every packet tests it
        for (int j = 0; j < 3; ++j) {
            rec[3 * j] = INFINITY;
            rec[3 * j + 1] = 0.0f;
            rec[3 * j + 2] = 0.0f;
        }
        brect[i] = none;
    }
    // the list entry: edge pre-test, triangle, leaf, plan
    rec[9] = __uint_as_float(i);
    rec[10] = __uint_as_float(leaf | (plan == 0u ? 0x80000000u : 0u));
    rec[11] = __uint_as_float(plan);
#ifndef BIH_FAST_COUNTERS
#define BIH_FAST_COUNTERS 0
#endif
    // counter builds check every plan against the root-path check: all paths
    if (!BIH_FP_SPLIT && (plan == 3u || BIH_FAST_COUNTERS) && !(BIH_FP_EXP & 8)) write_path(node_prim, leaf, path);
    for (int k = 0; k < 4; ++k) rec[12 + k] = plan_vals[k];
    float4 *o = reinterpret_cast<float4 *>(binrec + 16ull * i);
    for (int k = 0; k < 4; ++k) o[k] = make_float4(rec[4 * k], rec[4 * k + 1], rec[4 * k + 2], rec[4 * k + 3]);
    if (side == 0) glist[atomicAdd(gcount, 1u)] = i;   // every packet tests it
}

// The verification plan of alive triangle i = live[j] (k_bin_fp's, split
// off: BIH_FP_SPLIT): the inflated triangle's corners again from the record
// and k_bin_fp's (a, b, cc) -- the same f64 expressions, the same corners --
// then triangle_plan, the entry's leaf word and plan, and the root path of a
// full-check leaf.
#ifndef BIH_PLAN_TAB
#define BIH_PLAN_TAB 1     // triangle_plan<true>: per-axis values from an LDS table
#endif
#ifndef BIH_PLAN_WAVES
#define BIH_PLAN_WAVES 0   // waves per SIMD forced on k_bin_plan (0: the compiler's choice)
#endif
#if BIH_PLAN_WAVES
#define BIH_PLAN_OCC __attribute__((amdgpu_waves_per_eu(BIH_PLAN_WAVES, BIH_PLAN_WAVES)))
#else
#define BIH_PLAN_OCC
#endif
__global__ void __launch_bounds__(kThreads) BIH_PLAN_OCC k_bin_plan(const float *__restrict__ prim, BinCamera c,
                                                       const TreeHeader *__restrict__ hdr,
                                                       const uint4 *__restrict__ node_prim,
                                                       const uint32_t *__restrict__ tri_leaf,
                                                       const int32_t *__restrict__ leaf_parent,
                                                       const int32_t *__restrict__ parent,
                                                       uint2 *__restrict__ path, float *__restrict__ binrec,
                                                       const uint32_t *__restrict__ live,
                                                       const uint32_t *__restrict__ live_count) {
#if BIH_PLAN_TAB
    __shared__ double s_tab[12 * kThreads];
#endif
    const uint32_t j = blockIdx.x * kThreads + threadIdx.x;
    if (j >= *live_count) return;
    const uint32_t i = live[j];
    float *rec = binrec + 16ull * i;
    const float4 abc = *reinterpret_cast<const float4 *>(rec + 12);
    const uint32_t leaf = tri_leaf[i];
    uint32_t plan = 3u;
    float vals[4] = {0.0f, 0.0f, 0.0f, 0.0f};
    if (abc.w != 0.0f) {
        const float *r = prim + 16ull * i;
        float rr[9];
#pragma unroll
        for (int k = 0; k < 9; ++k) rr[k] = r[k];
        const double cu[3] = {-(double)abc.x, 1.0 + (double)abc.y + (double)abc.z, -(double)abc.x};
        const double cv[3] = {-(double)abc.y, -(double)abc.y, 1.0 + (double)abc.x + (double)abc.z};
        double cx[3][3];
        for (int q = 0; q < 3; ++q)
            for (int ax = 0; ax < 3; ++ax)
                cx[q][ax] = (cu[q] * (double)rr[ax] + cv[q] * (double)rr[3 + ax]) - (double)rr[6 + ax];
#if BIH_PLAN_TAB
        plan = triangle_plan<true>(cx, leaf, hdr, c.o, node_prim, leaf_parent, parent, vals, s_tab + threadIdx.x);
#else
        plan = triangle_plan<false>(cx, leaf, hdr, c.o, node_prim, leaf_parent, parent, vals, nullptr);
#endif
    }
    rec[10] = __uint_as_float(leaf | (plan == 0u ? 0x80000000u : 0u));
    rec[11] = __uint_as_float(plan);
    *reinterpret_cast<float4 *>(rec + 12) = make_float4(vals[0], vals[1], vals[2], vals[3]);
    if (plan == 3u || BIH_FAST_COUNTERS) write_path(node_prim, leaf, path);
}

// Tile (bx, by) against a triangle's edge pre-test (k0..k8 = 3 x {K0', Ku,
// Kv}, the kernel evaluates fmaf(Kv, v, fmaf(Ku, u, K0'))): 0 = no sample of
// the tile passes all three edges (the triangle stays off the tile's list),
// 2 = every sample passes (listed first: it most likely hits every lane),
// 1 = otherwise.  In f32 with margins (tests/test_bin_pretest.py mirrors it
// op for op and checks it on kernel-rounded samples):
//   - a sample of pixel x has u = fl(fl(x + r) / W), r in (0, 1], so
//     u in [x / W - e, (x + 1) / W + e] (e = 2^-24); the rectangle's
//     u0 = fl(fl(X * fl(1 / W)) - 2^-20) and u1 = fl(fl(XE * fl(1 / W)) +
//     2^-20) lie outside that by more than 12e (X <= W: |fl(X fl(1/W)) -
//     X / W| <= 2e, the pad's rounding e);
//   - hi = fl(fl(K0 + max(fl(Ku u0), fl(Ku u1))) + max(fl(Kv v0), fl(Kv v1)))
//     errs from the affine function's largest value over the rectangle by
//     at most 3e S (S = |K0| + |Ku| + |Kv|: three roundings of terms bounded
//     by S; fl is monotone, so the max of rounded products is the rounded
//     max), lo likewise from its smallest, and the kernel's two fmaf roundings
//     by 2e S more;
//   - the threshold T = 2^-21 fl(S) + 2^-125 >= 8e S (1 - 3e) covers the 5e S
//     and, through the absolute term, subnormal roundings.
// hi < -T: every sample's f < 0 (the kernel rejects it); lo > T: f > 0.
// NaN / inf coefficients never exclude a tile (T = inf or NaN compares false).
__device__ __forceinline__ float edge_margin(float K0, float Ku, float Kv) {
    return 0x1p-21f * ((fabsf(K0) + fabsf(Ku)) + fabsf(Kv)) + 0x1p-125f;
}
__device__ __forceinline__ int tile_class(const float4 r0, const float4 r1, const float4 r2,
                                          uint32_t bx, uint32_t by, uint32_t w, uint32_t h,
                                          uint32_t tw, uint32_t th) {
    const float pad = 0x1p-20f;
    const float iw = 1.0f / (float)w, ih = 1.0f / (float)h;
    const uint32_t xe = (bx + 1) * tw < w ? (bx + 1) * tw : w;
    const uint32_t ye = (by + 1) * th < h ? (by + 1) * th : h;
    const float u0 = (float)(bx * tw) * iw - pad, u1 = (float)xe * iw + pad;
    const float v0 = (float)(by * th) * ih - pad, v1 = (float)ye * ih + pad;
    const float k[9] = {r0.x, r0.y, r0.z, r0.w, r1.x, r1.y, r1.z, r1.w, r2.x};
    bool all = true;
#pragma unroll
    for (int j = 0; j < 3; ++j) {
        const float K0 = k[3 * j], Ku = k[3 * j + 1], Kv = k[3 * j + 2];
        const float T = edge_margin(K0, Ku, Kv);
        const float au0 = Ku * u0, au1 = Ku * u1, bv0 = Kv * v0, bv1 = Kv * v1;
        const float hi = (K0 + fmaxf(au0, au1)) + fmaxf(bv0, bv1);
        const float lo = (K0 + fminf(au0, au1)) + fminf(bv0, bv1);
        if (hi < -T) return 0;
        if (!(lo > T)) all = false;
    }
    return all ? 2 : 1;
}

// Pixel mask of a 4 x 4-pixel tile against a triangle's edge pre-test: bit
// 4 * row + col is clear only when no sample of that pixel can pass all
// three edges (tile_class's hi test on the pixel's own rectangle: the
// largest value is K0 + cu[px] + cv[py], 8 products per edge instead of 16
// rectangles).  The list walk skips an entry for a packet whose remaining
// lanes all sit in pixels outside its mask.  Other tile shapes: all ones.
__device__ __forceinline__ uint32_t pixel_mask(const float4 r0, const float4 r1, const float4 r2,
                                               uint32_t bx, uint32_t by, uint32_t w, uint32_t h,
                                               uint32_t tw, uint32_t th) {
    if (tw != 4u || th != 4u) return 0xFFFFu;
    const float k[9] = {r0.x, r0.y, r0.z, r0.w, r1.x, r1.y, r1.z, r1.w, r2.x};
    const float pad = 0x1p-20f;
    const float iw = 1.0f / (float)w, ih = 1.0f / (float)h;
    float ua[4], ub[4], va[4], vb[4];   // each pixel's u0, u1 / row's v0, v1
#pragma unroll
    for (uint32_t j = 0; j < 4u; ++j) {
        const uint32_t x = bx * 4u + j, y = by * 4u + j;
        ua[j] = (float)x * iw - pad;
        ub[j] = (float)(x + 1u) * iw + pad;
        va[j] = (float)y * ih - pad;
        vb[j] = (float)(y + 1u) * ih + pad;
    }
    uint32_t m = 0xFFFFu;
#pragma unroll
    for (int e = 0; e < 3; ++e) {
        const float K0 = k[3 * e], Ku = k[3 * e + 1], Kv = k[3 * e + 2];
        const float T = edge_margin(K0, Ku, Kv);
        float cu[4], cv[4];
#pragma unroll
        for (uint32_t j = 0; j < 4u; ++j) {
            cu[j] = K0 + fmaxf(Ku * ua[j], Ku * ub[j]);
            cv[j] = fmaxf(Kv * va[j], Kv * vb[j]);
        }
#pragma unroll
        for (uint32_t py = 0; py < 4u; ++py)
#pragma unroll
            for (uint32_t px = 0; px < 4u; ++px)
                if (cu[px] + cv[py] < -T) m &= ~(1u << (4u * py + px));
    }
    return m;
}

// The (triangle, tile) pairs of a block's alive triangles (k_cam_tris' list,
// entries blockIdx.x * kThreads ..): the tile rectangles' areas are scanned in
// LDS and the block's threads take the pairs in turn (pair p: the triangle
// whose area range holds p, tile p - its start in row-major order), so a
// large rectangle (a triangle close to the camera or seen edge-on) is spread
// over the whole block and every lane runs the same `visit` code.
// `reserve(tot)` (thread 0, after the scan) returns the block's base in the
// pair-result buffer (k_bin_count reserves it, k_bin_fill reads it back; ~0:
// none); `visit` gets (triangle, tile x, tile y, base, pair index).
struct PairLds {
    uint32_t off[kThreads + 1];   // exclusive scan of the areas; off[kThreads] = the block's pairs
    uint32_t tri[kThreads];
    uint2 rect[kThreads];
    uint32_t wsum[kThreads / 64];
    uint32_t base;
};
template <typename R, typename F>
__device__ __forceinline__ void for_block_pairs(const uint2 *__restrict__ brect, const uint32_t *__restrict__ live,
                                                const uint32_t *__restrict__ live_count, PairLds &L, R &&reserve,
                                                F &&visit) {
    const uint32_t tid = threadIdx.x, j0 = blockIdx.x * kThreads + tid, lane = tid & 63u, w = tid >> 6;
    const uint32_t nl = *live_count;
    uint2 q = make_uint2(1u, 0u);
    uint32_t i = 0;
    if (j0 < nl) {
        i = live[j0];
        q = brect[i];
    }
    const uint32_t bx0 = q.x & 0xffffu, bx1 = q.x >> 16, by0 = q.y & 0xffffu, by1 = q.y >> 16;
    const uint32_t area = (j0 < nl && bx0 <= bx1) ? (bx1 - bx0 + 1) * (by1 - by0 + 1) : 0u;
    // inclusive wave scan of the areas, then the waves' totals
    uint32_t x = area;
#pragma unroll
    for (uint32_t d = 1; d < 64u; d <<= 1) {
        const uint32_t y = __shfl_up(x, d, 64);
        if (lane >= d) x += y;
    }
    if (lane == 63u) L.wsum[w] = x;
    L.tri[tid] = i;
    L.rect[tid] = make_uint2(bx0 | (by0 << 16), bx1 - bx0 + 1);
    __syncthreads();
    uint32_t base = 0, tot = 0;
    for (uint32_t k = 0; k < kThreads / 64; ++k) {
        base += k < w ? L.wsum[k] : 0u;
        tot += L.wsum[k];
    }
    L.off[tid] = base + x - area;
    if (tid == 0) {
        L.off[kThreads] = tot;
        L.base = reserve(tot);
    }
    __syncthreads();
    const uint32_t pbase = L.base;
    for (uint32_t p = tid; p < tot; p += kThreads) {
        // the last triangle t with off[t] <= p (zero areas repeat an offset)
        uint32_t lo = 0, hi = kThreads;   // off[lo] <= p < off[hi]
        while (hi - lo > 1u) {
            const uint32_t mid = (lo + hi) >> 1;
            if (L.off[mid] <= p) lo = mid;
            else hi = mid;
        }
        const uint2 r = L.rect[lo];
        const uint32_t k = p - L.off[lo], wx = r.y;
        const uint32_t ty = k / wx;
        visit(L.tri[lo], (r.x & 0xffffu) + (k - ty * wx), (r.x >> 16) + ty, pbase, p);
    }
}

// List order.  A tile's list is walked front to back until every lane of
// the packet has a verified hit (or the list ends), so triangles that cover
// more of the tile go first: bucket 0 = every sample passes the pre-test
// (tile_class 2), then the others by the pixel mask's population, most
// pixels first (other tile shapes: all in bucket 1).  The order never
// changes a pixel (any verified hit of a lane is the same bit); on the bench
// frame it halves the entries walked against arrival order.  Per (tile,
// bucket) counts are packed kBucketBits each in a u64 (a block adds at most
// 256 per field).
constexpr uint32_t kBuckets = kBinBuckets;    // 4: {2}, 12..16, 6..11, <6 px; 6: {2}, 16, 13..15, 10..12, 7..9, <7
constexpr uint32_t kBucketBits = 64 / kBuckets >= 16 ? 16 : 64 / kBuckets;
constexpr unsigned long long kBucketMask = (1ull << kBucketBits) - 1ull;
static_assert(kBuckets * kBucketBits <= 64 && (1u << kBucketBits) > kThreads, "bucket fields");
__device__ __forceinline__ uint32_t entry_bucket(int cls, uint32_t pm) {
    if (cls == 2) return 0u;
    const uint32_t pc = (uint32_t)__popc(pm);
    if (kBuckets == 4) return pc >= 12u ? 1u : (pc >= 6u ? 2u : 3u);
    const uint32_t q = kBuckets >= 7u ? 1u + (16u - pc + 1u) / 2u : 1u + (16u - pc + 2u) / 3u;
    return q < kBuckets - 1u ? q : kBuckets - 1u;
}

// Counts per tile (cnt: all entries, for the offsets) and per tile and
// bucket 0 .. kBuckets-2 (cntq[(kBuckets - 1) * b + q]; the last bucket is
// the rest).  A block's alive
// triangles are Morton neighbours, so their footprints share tiles: the block
// counts in LDS over the bounding rectangle of its footprints and adds each
// non-zero count to the global counters once.  Blocks whose rectangle exceeds
// kBlockTiles tiles count with global atomics directly.  The block's LDS
// counts also go to blkcnt[block][..] for k_bin_fill, which takes the same
// blocks and rectangles (a pass of its own would recount them).
constexpr uint32_t kBlockTiles = kBinBlockTiles;
__global__ void __launch_bounds__(kThreads) k_bin_count(const uint2 *__restrict__ brect,
                                                        const uint32_t *__restrict__ live,
                                                        const uint32_t *__restrict__ live_count,
                                                        uint32_t bins_x, const float4 *__restrict__ binrec,
                                                        uint32_t w, uint32_t h, uint32_t tw, uint32_t th,
                                                        uint32_t *__restrict__ cnt, uint32_t *__restrict__ cntq,
                                                        unsigned long long *__restrict__ blkcnt,
                                                        unsigned long long *__restrict__ total64,
                                                        uint32_t *__restrict__ pres, uint32_t pres_cap,
                                                        unsigned long long *__restrict__ pcount,
                                                        uint32_t *__restrict__ pbase_out) {
    __shared__ unsigned long long s_cnt[kBlockTiles];
    __shared__ uint32_t s_rect[4];   // x0, x1, y0, y1 of the block's footprints
    __shared__ unsigned long long s_tot;   // the block's entries (64-bit: the list total may pass 2^32)
    __shared__ PairLds L;
    const uint32_t tid = threadIdx.x, j0 = blockIdx.x * kThreads + tid;
    if (tid == 0) {
        s_rect[0] = s_rect[2] = 0xffffu;
        s_rect[1] = s_rect[3] = 0u;
        s_tot = 0ull;
    }
    __syncthreads();
    if (j0 < *live_count) {
        const uint2 q = brect[live[j0]];
        const uint32_t bx0 = q.x & 0xffffu, bx1 = q.x >> 16, by0 = q.y & 0xffffu, by1 = q.y >> 16;
        if (bx0 <= bx1) {
            atomicMin(&s_rect[0], bx0);
            atomicMax(&s_rect[1], bx1);
            atomicMin(&s_rect[2], by0);
            atomicMax(&s_rect[3], by1);
        }
    }
    __syncthreads();
    const uint32_t rx0 = s_rect[0], rx1 = s_rect[1], ry0 = s_rect[2], ry1 = s_rect[3];
    const uint32_t rw = rx1 - rx0 + 1;
    const bool use_lds = rx0 <= rx1 && (uint64_t)rw * (ry1 - ry0 + 1) <= kBlockTiles;   // block-uniform
    const uint32_t rarea = use_lds ? rw * (ry1 - ry0 + 1) : 0u;
    for (uint32_t k = tid; k < rarea; k += kThreads) s_cnt[k] = 0ull;
    __syncthreads();
    unsigned long long mine = 0ull;
    auto reserve = [&](uint32_t tot) {
        uint32_t b = ~0u;
        if (pres && tot) {
            // a 64-bit cursor: the pairs of all blocks may pass 2^32 (a u32
            // cursor would wrap and hand a later block an earlier block's range)
            const unsigned long long b64 = atomicAdd(pcount, (unsigned long long)tot);
            if (b64 <= pres_cap && pres_cap - b64 >= tot) b = (uint32_t)b64;   // else the fill recomputes
        }
        pbase_out[blockIdx.x] = b;
        return b;
    };
    for_block_pairs(brect, live, live_count, L, reserve, [&](uint32_t i, uint32_t bx, uint32_t by, uint32_t pb,
                                                             uint32_t p) {
        const float4 r0 = binrec[4ull * i], r1 = binrec[4ull * i + 1], r2 = binrec[4ull * i + 2];
        const int cls = tile_class(r0, r1, r2, bx, by, w, h, tw, th);
        const uint32_t pm = cls == 2 ? 0xFFFFu : (cls ? pixel_mask(r0, r1, r2, bx, by, w, h, tw, th) : 0u);
        const uint32_t q = entry_bucket(cls, pm);
        // the pair's result for k_bin_fill: listed | pixel mask << 8 | bucket
        if (pb != ~0u) pres[pb + p] = cls ? (0x80000000u | (pm << 8) | q) : 0u;
        if (!cls) return;
        ++mine;
        if (use_lds) {
            atomicAdd(&s_cnt[(by - ry0) * rw + (bx - rx0)], 1ull << (kBucketBits * q));
        } else {
            const uint32_t b = by * bins_x + bx;
            atomicAdd(cnt + b, 1u);
            if (q < kBuckets - 1u) atomicAdd(cntq + (kBuckets - 1ull) * b + q, 1u);
        }
    });
    if (mine) atomicAdd(&s_tot, mine);
    __syncthreads();
    for (uint32_t k = tid; k < rarea; k += kThreads) {
        const unsigned long long c = s_cnt[k];
        blkcnt[(uint64_t)blockIdx.x * kBlockTiles + k] = c;
        if (!c) continue;
        const uint32_t b = (ry0 + k / rw) * bins_x + rx0 + k % rw;
        uint32_t all = 0;
#pragma unroll
        for (uint32_t q = 0; q < kBuckets; ++q) {
            const uint32_t cq = (uint32_t)((c >> (kBucketBits * q)) & kBucketMask);
            all += cq;
            if (q < kBuckets - 1u && cq) atomicAdd(cntq + (kBuckets - 1ull) * b + q, cq);
        }
        atomicAdd(cnt + b, all);
    }
    if (tid == 0 && s_tot) atomicAdd(total64, s_tot);
}

// The lists: each (triangle, tile) pair k_bin_count counted copies the
// first 48 bytes of the triangle's record into the tile's list, in its bucket's range
// (off[b] + the counts of the buckets before it) at a position from the
// bucket's cursor cur[kBuckets * b + q] (zeroed).  When the block's tile
// rectangle fits kBlockTiles tiles, k_bin_count's per-(tile, bucket) counts
// of the same block (blkcnt) are reserved with one global atomic per (tile,
// bucket), and the pass over the pairs ranks them through LDS atomics;
// larger rectangles take one global atomic per entry.  (Per-entry global
// atomics throughout cost 0.10 of this kernel's 0.15 ms.)  Within a bucket
// the order is the blocks' (Morton order, roughly) -- it can change which
// candidate a lane verifies, never a pixel.
__global__ void __launch_bounds__(kThreads) k_bin_fill(const uint2 *__restrict__ brect,
                                                       const uint32_t *__restrict__ live,
                                                       const uint32_t *__restrict__ live_count,
                                                       uint32_t bins_x, uint32_t w, uint32_t h,
                                                       uint32_t tw, uint32_t th,
                                                       const uint32_t *__restrict__ off,
                                                       const uint32_t *__restrict__ cntq,
                                                       const unsigned long long *__restrict__ blkcnt,
                                                       uint32_t *__restrict__ cur,
                                                       const float4 *__restrict__ binrec,
                                                       const uint32_t *__restrict__ gstat,
                                                       float4 *__restrict__ list,
                                                       const uint32_t *__restrict__ pres,
                                                       const uint32_t *__restrict__ pbase_in) {
    if (*gstat == kBinsUnusable) return;   // the lists would not fit: the render falls back
    constexpr uint32_t kS = kBlockTiles;
    __shared__ unsigned long long s_cnt[kS];
    __shared__ uint32_t s_base[kBuckets][kS];
    __shared__ uint32_t s_rect[4];   // x0, x1, y0, y1 of the block's footprints
    __shared__ PairLds L;
    const uint32_t tid = threadIdx.x, j0 = blockIdx.x * kThreads + tid;
    if (tid == 0) {
        s_rect[0] = s_rect[2] = 0xffffu;
        s_rect[1] = s_rect[3] = 0u;
    }
    __syncthreads();
    if (j0 < *live_count) {
        const uint2 q = brect[live[j0]];
        const uint32_t bx0 = q.x & 0xffffu, bx1 = q.x >> 16, by0 = q.y & 0xffffu, by1 = q.y >> 16;
        if (bx0 <= bx1) {
            atomicMin(&s_rect[0], bx0);
            atomicMax(&s_rect[1], bx1);
            atomicMin(&s_rect[2], by0);
            atomicMax(&s_rect[3], by1);
        }
    }
    __syncthreads();
    const uint32_t rx0 = s_rect[0], rx1 = s_rect[1], ry0 = s_rect[2], ry1 = s_rect[3];
    const uint32_t rw = rx1 - rx0 + 1;
    const bool use_lds = rx0 <= rx1 && (uint64_t)rw * (ry1 - ry0 + 1) <= kBlockTiles;   // block-uniform
    const uint32_t rarea = use_lds ? rw * (ry1 - ry0 + 1) : 0u;
    // bucket q of tile b starts at off[b] + the counts of buckets 0 .. q-1
    auto bucket_start = [&](uint32_t b, uint32_t q) {
        uint32_t st = off[b];
        for (uint32_t k = 0; k < q; ++k) st += cntq[(kBuckets - 1ull) * b + k];
        return st;
    };
    if (use_lds) {
        for (uint32_t k = tid; k < rarea; k += kThreads) {
            const unsigned long long c = blkcnt[(uint64_t)blockIdx.x * kBlockTiles + k];   // k_bin_count's
            if (c) {
                const uint32_t b = (ry0 + k / rw) * bins_x + rx0 + k % rw;
                uint32_t st = off[b];
                for (uint32_t q = 0; q < kBuckets; ++q) {
                    const uint32_t cq = (uint32_t)((c >> (kBucketBits * q)) & kBucketMask);
                    s_base[q][k] = cq ? st + atomicAdd(cur + (unsigned long long)kBuckets * b + q, cq) : 0u;
                    if (q < kBuckets - 1u) st += cntq[(kBuckets - 1ull) * b + q];
                }
            }
            s_cnt[k] = 0ull;
        }
        __syncthreads();
    }
    auto reserve = [&](uint32_t) { return pres ? pbase_in[blockIdx.x] : ~0u; };
    for_block_pairs(brect, live, live_count, L, reserve, [&](uint32_t i, uint32_t bx, uint32_t by, uint32_t pb,
                                                             uint32_t p) {
        // the pair's class, pixel mask and bucket: k_bin_count's result when
        // its block had room in the pair buffer, else computed again
        uint32_t pm, q;
        if (pb != ~0u) {
            const uint32_t r = pres[pb + p];
            if (!(r >> 31)) return;
            pm = (r >> 8) & 0xFFFFu;
            q = r & 0xFFu;
        } else {
            const float4 r0 = binrec[4ull * i], r1 = binrec[4ull * i + 1], r2 = binrec[4ull * i + 2];
            const int cls = tile_class(r0, r1, r2, bx, by, w, h, tw, th);
            if (!cls) return;
            pm = cls == 2 ? 0xFFFFu : pixel_mask(r0, r1, r2, bx, by, w, h, tw, th);
            q = entry_bucket(cls, pm);
        }
        const float4 r0 = binrec[4ull * i], r1 = binrec[4ull * i + 1], r2 = binrec[4ull * i + 2];
        // the entry's word 11: plan meta (bits 0-13) | pixel mask << 16
        uint32_t pos;
        if (use_lds) {
            const uint32_t k = (by - ry0) * rw + (bx - rx0);
            const unsigned long long r = atomicAdd(&s_cnt[k], 1ull << (kBucketBits * q));
            pos = s_base[q][k] + (uint32_t)((r >> (kBucketBits * q)) & kBucketMask);
        } else {
            const uint32_t b = by * bins_x + bx;
            pos = bucket_start(b, q) + atomicAdd(cur + (unsigned long long)kBuckets * b + q, 1u);
        }
        float4 *o = list + (uint64_t)kBinEntryF4 * pos;
        o[0] = r0;
        o[1] = r1;
        o[2] = make_float4(r2.x, r2.y, r2.z, __uint_as_float((__float_as_uint(r2.w) & 0xFFFFu) | (pm << 16)));
    });
}

// The global list's entries (the same 48-byte entries); gstat as k_bin_status
// left it (a grid over kBinGlobalMax entries: no host copy of the count).
__global__ void __launch_bounds__(kThreads) k_bin_gfill(const uint32_t *__restrict__ gstat,
                                                        const uint32_t *__restrict__ glist,
                                                        const float4 *__restrict__ binrec,
                                                        float4 *__restrict__ gent) {
    const uint32_t j = blockIdx.x * kThreads + threadIdx.x;
    const uint32_t gn = *gstat;
    if (gn == kBinsUnusable || j >= gn) return;
    const uint32_t i = glist[j];
    for (uint32_t k = 0; k < 2; ++k) gent[(uint64_t)kBinEntryF4 * j + k] = binrec[4ull * i + k];
    const float4 r2 = binrec[4ull * i + 2];   // every pixel of every tile
    gent[(uint64_t)kBinEntryF4 * j + 2] =
        make_float4(r2.x, r2.y, r2.z, __uint_as_float(__float_as_uint(r2.w) | 0xFFFF0000u));
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
// others): per band the tiles with a non-empty list, longest processing time
// first, then the tiles no triangle touches (background).  Without measured
// costs the order is by power-of-two classes of the list length; with them
// (the cycles per frame an earlier launch of this camera measured for each
// tile, RenderArgs::bin_cost) by quarter-power-of-two classes of the cost,
// and each band's tiles costing at least kHeavyFactor x the mean -- their
// items would otherwise run for most of a multi-frame launch on one wave --
// come first and are counted (qw[kQHeavy + band]) for the kernel to split over
// frame ranges.  Built once per camera, image, row set and cost state.
constexpr uint32_t kQBands = 8, kQClasses = 65;   // live classes 0..63 (costliest first), 64: background
constexpr uint32_t kQCount = 0, kQStart = kQBands * kQClasses, kQCur = 2 * kQBands * kQClasses,
                   kQHdr = 3 * kQBands * kQClasses, kQHeavy = kQHdr + 4 * kQBands, kQWords = 2048;
static_assert(kQHeavy + kQBands <= kQWords, "queue words");
#ifndef BIH_HEAVY_FACTOR
#define BIH_HEAVY_FACTOR 2.0f
#endif
constexpr float kHeavyFactor = BIH_HEAVY_FACTOR;
__device__ __forceinline__ uint32_t queue_bin(uint32_t t, uint32_t tiles_x, uint32_t row0,
                                              uint32_t band_h, uint32_t band_step, uint32_t th,
                                              uint32_t bins_x) {
    const uint32_t ty = t / tiles_x, tx = t - ty * tiles_x;
    const uint32_t lr = ty * th;
    const uint32_t gy = row0 + (lr / band_h) * band_h * band_step + (lr % band_h);
    return (gy / th) * bins_x + tx;
}
// cost -> class: key = 4 log2(cost) (two fraction bits), class 95 - key
// clamped to [0, 63]: the costliest first, a quarter power of two apart
// (k_render_bins' cost = 256 x (entries pre-tested + 4 x intersector calls)
// per frame, ~2^11 .. 2^16: classes ~31 .. 51)
__device__ __forceinline__ uint32_t cost_class(uint32_t cost) {
    const uint32_t c = cost | 1u, lz = __clz(c);
    const uint32_t frac = (lz < 30u) ? ((c << (lz + 1u)) >> 30) : 0u;
    const int key = (int)(31u - lz) * 4 + (int)frac;
    const int k = 95 - key;
    return (uint32_t)(k < 0 ? 0 : (k > 63 ? 63 : k));
}
// the class's representative cost (the low end of its range)
__device__ __forceinline__ float class_cost(uint32_t k) { return exp2f((float)(95 - (int)k) * 0.25f); }
// qw: class counts, class starts, fill cursors (kQBands x kQClasses each),
// per band {start, live, background, items}, per band heavy count
__global__ void __launch_bounds__(kThreads) k_queue_class(const uint32_t *__restrict__ off,
                                                          const uint32_t *__restrict__ gstat,
                                                          uint32_t ntiles, uint32_t tiles_x,
                                                          uint32_t tiles_y, uint32_t row0,
                                                          uint32_t band_h, uint32_t band_step,
                                                          uint32_t th, uint32_t bins_x, uint32_t lpt,
                                                          const uint32_t *__restrict__ cost,
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
        const uint32_t lc = !lpt ? 0u : (cost ? cost_class(cost[b]) : (uint32_t)__clz(len));
        const uint32_t k = band * kQClasses + (len ? lc : kQClasses - 1);
        cls[t] = (uint16_t)k;
        atomicAdd(&hist[k], 1u);
    }
    __syncthreads();
    for (uint32_t k = threadIdx.x; k < kQBands * kQClasses; k += kThreads)
        if (hist[k]) atomicAdd(qw + kQCount + k, hist[k]);
}
__global__ void __launch_bounds__(kThreads) k_queue_scan(uint32_t *__restrict__ qw, uint32_t heavy) {
    // one block: the counts to LDS in one parallel load, band totals and
    // starts from LDS, then each band's class starts (a serial chain of
    // global loads took 19 us)
    __shared__ uint32_t c[kQBands * kQClasses], bstart[kQBands + 1];
    __shared__ uint32_t hthr;
    const uint32_t t = threadIdx.x;
    for (uint32_t k = t; k < kQBands * kQClasses; k += kThreads) c[k] = qw[kQCount + k];
    __syncthreads();
    if (t == 0) {
        uint32_t acc = 0;
        for (uint32_t b = 0; b < kQBands; ++b) {
            bstart[b] = acc;
            for (uint32_t k = 0; k < kQClasses; ++k) acc += c[b * kQClasses + k];
        }
        bstart[kQBands] = acc;
        // heavy tiles (measured costs only): classes whose cost reaches
        // kHeavyFactor x the mean live cost
        uint32_t thr = 0;
        if (heavy) {
            float n = 0.f, sum = 0.f;
            for (uint32_t k = 0; k + 1 < kQClasses; ++k) {
                float m = 0.f;
                for (uint32_t b = 0; b < kQBands; ++b) m += (float)c[b * kQClasses + k];
                n += m;
                sum += m * class_cost(k);
            }
            const float lim = n > 0.f ? kHeavyFactor * sum / n : 0.f;
            while (thr + 1 < kQClasses && class_cost(thr) >= lim) ++thr;   // classes [0, thr) are heavy
        }
        hthr = thr;
    }
    __syncthreads();
    if (t < kQBands) {
        const uint32_t b = t, start = bstart[b];
        uint32_t acc = start, hv = 0;
        for (uint32_t k = 0; k < kQClasses; ++k) {
            qw[kQStart + b * kQClasses + k] = acc;
            qw[kQCur + b * kQClasses + k] = 0;
            acc += c[b * kQClasses + k];
            if (k < hthr) hv += c[b * kQClasses + k];
        }
        const uint32_t bg = c[b * kQClasses + kQClasses - 1];
        const uint32_t live = acc - start - bg;
        qw[kQHdr + 4 * b] = start;
        qw[kQHdr + 4 * b + 1] = live;
        qw[kQHdr + 4 * b + 2] = bg;
        qw[kQHdr + 4 * b + 3] = live + (bg + 63u) / 64u;
        qw[kQHeavy + b] = hv;
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
        if (hist[j]) base[j] = qw[kQStart + j] + atomicAdd(qw + kQCur + j, hist[j]);
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

int launch_bin_footprints(const float *tris, uint32_t n, const uint4 *nodes, uint32_t m, const float origin[3],
                          float *prim, const TreeHeader *hdr, const uint32_t *tri_leaf,
                          const int32_t *leaf_parent, const int32_t *parent, const BinCamera &c,
                          const BinBuffers &b, void *stream) {
    const hipStream_t st = (hipStream_t)stream;
    const uint32_t nb = b.bins_x * b.bins_y;
    const uint4 *node_prim = reinterpret_cast<const uint4 *>(prim + 16ull * n);
    if (n > 0) {
        // gcount[0] = global list length, gcount[3] = alive triangles,
        // gcount[4..5] = the list total as a 64-bit sum (k_bin_count); cnt,
        // cntq and cur (adjacent) zeroed
        const dim3 g((n + kThreads - 1) / kThreads);
        const uint32_t zero_words = (uint32_t)((reinterpret_cast<const char *>(b.cur + (size_t)kBuckets * nb) -
                                                reinterpret_cast<const char *>(b.cnt)) / 4);
        hipLaunchKernelGGL(k_cam_tris, g, dim3(kThreads), 0, st, tris, n, origin[0], origin[1], origin[2], prim,
                           nodes, m, reinterpret_cast<uint4 *>(prim + 16ull * n),
                           reinterpret_cast<unsigned long long *>(b.bmask), b.bcnt, b.cnt, zero_words, b.gcount);
        hipError_t e = (hipError_t)scan_exclusive(b.bcnt, b.boff, g.x, b.bpart, b.gcount + 3, stream);
        if (e != hipSuccess) return (int)e;
        hipLaunchKernelGGL(k_live_compact, g, dim3(kThreads), 0, st,
                           reinterpret_cast<const unsigned long long *>(b.bmask), b.boff, b.live);
        hipLaunchKernelGGL(k_bin_fp, g, dim3(kThreads), 0, st, prim, n, c, hdr, node_prim, tri_leaf, leaf_parent,
                           parent, b.path, b.brect, b.binrec, b.gcount,
                           b.glist, b.live, b.gcount + 3);
        if (BIH_FP_SPLIT)
            hipLaunchKernelGGL(k_bin_plan, g, dim3(kThreads), 0, st, prim, c, hdr, node_prim, tri_leaf, leaf_parent,
                               parent, b.path, b.binrec, b.live, b.gcount + 3);
        hipLaunchKernelGGL(k_bin_count, g, dim3(kThreads), 0, st, b.brect, b.live, b.gcount + 3, b.bins_x,
                           reinterpret_cast<const float4 *>(b.binrec), c.w, c.h, c.tw, c.th, b.cnt, b.cntq,
                           reinterpret_cast<unsigned long long *>(b.blkcnt),
                           reinterpret_cast<unsigned long long *>(b.gcount + 4), b.pres, b.pres_cap,
                           reinterpret_cast<unsigned long long *>(b.gcount + 6),
                           b.pbase);
    }
    const hipError_t e = hipGetLastError();
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
    (void)nb;   // the cursors were zeroed by k_cam_tris
    if (n > 0)
        hipLaunchKernelGGL(k_bin_fill, dim3((n + kThreads - 1) / kThreads), dim3(kThreads), 0, st,
                           b.brect, b.live, b.gcount + 3, b.bins_x, c.w, c.h, c.tw, c.th, b.off, b.cntq,
                           reinterpret_cast<const unsigned long long *>(b.blkcnt), b.cur,
                           reinterpret_cast<const float4 *>(b.binrec), gstat, reinterpret_cast<float4 *>(list),
                           b.pres, b.pbase);
    if (n > 0)
        hipLaunchKernelGGL(k_bin_gfill, dim3((kBinGlobalMax + kThreads - 1) / kThreads), dim3(kThreads), 0, st,
                           gstat, b.glist, reinterpret_cast<const float4 *>(b.binrec),
                           reinterpret_cast<float4 *>(gent));
    return (int)hipGetLastError();
}

size_t bin_queue_bytes(uint32_t ntiles) {
    return ((size_t)ntiles * 6 + kQWords * 4 + 255) & ~(size_t)255;
}

int launch_bin_queue(const uint32_t *off, const uint32_t *gstat, uint32_t bins_x, uint32_t tiles_x, uint32_t ntiles,
                     uint32_t row0, uint32_t band_h, uint32_t band_step, uint32_t th, void *mem,
                     uint32_t **queue, uint32_t **qhdr, void *stream, const uint32_t *cost, uint32_t **qheavy) {
    const hipStream_t st = (hipStream_t)stream;
    uint32_t *qw = reinterpret_cast<uint32_t *>(mem);
    uint32_t *q = qw + kQWords;
    uint16_t *cls = reinterpret_cast<uint16_t *>(q + ntiles);
    *queue = q;
    *qhdr = qw + kQHdr;
    if (qheavy) *qheavy = qw + kQHeavy;
    hipError_t e = hipMemsetAsync(qw, 0, kQWords * sizeof(uint32_t), st);
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
                           band_h, band_step, th, bins_x, lpt, cost, cls, qw);
    }
    hipLaunchKernelGGL(k_queue_scan, dim3(1), dim3(kThreads), 0, st, qw, (cost && lpt) ? 1u : 0u);
    if (ntiles > 0)
        hipLaunchKernelGGL(k_queue_fill, dim3((ntiles + kThreads - 1) / kThreads), dim3(kThreads), 0, st, cls,
                           ntiles, qw, q);
    return (int)hipGetLastError();
}

}  // namespace bih
