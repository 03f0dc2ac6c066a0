// bih_whitted.hip -- config C4 (BASELINE.json configs[3]): 8-bounce Whitted
// mirror rays at 3840x2160 on gfx950, as a wavefront of compacted ray queues.
//
// The reference has primary rays only (cudaRender, CUDAKernels.cu:391-423;
// Color :370-389 is binary).  C4's semantics are the build's own, defined in
// the test oracle (ob_render_whitted) and DESIGN.md section 4.5:
//   closest hit = min (t, sorted position) over the triangles the reference
//   walk visits (TraverseTree's decisions, :227-368, RayTriangleIntersection
//   :17-50), t_lo < t < FLT_MAX (t_lo = 0 for primary rays, 1e-4 after; a
//   bounce's walk interval starts at max(box entry, t_lo));
//   P = O + t*D, n = cross(e1, e2), k = (2*dot(D, n)) / dot(n, n), R = D - k*n;
//   shade(d) = miss ? (20,20,40) : d == 8 ? (255,255,0) : 0.5*Y + 0.5*shade(d+1).
// The (t, i) rule is order-independent, so any walk order over the same visit
// set gives the oracle's hit; every f32 expression is the oracle's, in its
// order (-ffp-contract=off): bit-exact RGBA.
//
// Kernels (one frame, all on the caller's stream, no host round trip):
//   k_wh_gen    one thread per sample: the XORWOW jitter (cudaRender's draws)
//               and camera direction into ray queue 0; zeroes the counters.
//   k_wh_trace  bounce d (9 launches): persistent waves drain queue d%2
//               (length counts[d]); each lane walks its ray's BIH visit set
//               for the closest hit; hits reflect and are appended to queue
//               (d+1)%2 with one ballot + mbcnt per wave and one atomic per
//               wave (wavefront compaction: the next bounce's waves are full).
//   k_wh_shade  one thread per pixel: the samples' shades -> rgbToInt.
#include <hip/hip_runtime.h>
#include <float.h>

#include "bih_device.h"
#include "bih_internal.h"

namespace bih {
namespace {

using dev::camera_dir;
using dev::global_row;
using dev::kDetEps;
using dev::rgb_to_int;
using dev::xorwow_uniform;

constexpr uint32_t kWT = 64;            // threads per block: one wave
constexpr int kWStack = kStackDepth;    // Karras path length <= 30 (bih_internal.h)
#ifndef BIH_WH_LDS
#define BIH_WH_LDS 10   // (A/B r04r/s, ms per C4 frame: 6 958, 8 725, 10 683, 12 752, 16 877)
#endif
constexpr int kWLds = BIH_WH_LDS;       // stack slots per lane in LDS; deeper ones in HBM
constexpr uint32_t kWBlocksPerCU = 32;  // persistent grid of k_wh_trace
constexpr uint32_t kNoHit = 0xFFFFFFFFu;
constexpr float kBounceTLo = 1e-4f;     // t_lo of secondary rays (oracle: 1e-4f)
constexpr uint32_t kWCounts = 32;       // counter words: [0..9] rays per queue, [16..25] rays taken (k_wh_trace_dyn)
constexpr uint32_t kWFetch = 16;
#ifndef BIH_WH_SORT_BITS
#define BIH_WH_SORT_BITS 5   // origin cells per axis 2^bits (3: LDS-aggregated counts; more: global atomics;
                             // A/B r04zo per 4K frame: 3 0.636 s, 4 0.644, 5 0.620, 6 0.623)
#endif
#ifndef BIH_WH_SORT_DIR
#define BIH_WH_SORT_DIR 0    // 1: the direction's dominant axis joins the key (x 4 buckets; r04zp: 0.617 vs 0.621 s, noise)
#endif
constexpr uint32_t kWSortBucketsGen = (8u << (3 * BIH_WH_SORT_BITS)) << (BIH_WH_SORT_DIR ? 2 : 0);   // = kWSortBuckets
constexpr uint32_t kWWorkWords = 18;    // work counters: {nodes, triangles} per bounce, u64 (k_wh_trace_dyn<true>)

struct WScene {
    const uint4 *nodes;
    const float *tris;          // sorted {v0, e1, e2}
    const uint32_t *dup;
    float slo[3], shi[3];
    uint32_t U, N;
};

__device__ __forceinline__ WScene load_wscene(const RenderArgs &a) {
    WScene s;
    s.nodes = a.nodes;
    s.tris = a.tris;
    s.dup = a.dup_cnt;
    for (int k = 0; k < 3; ++k) {
        s.slo[k] = a.hdr->scene_lo[k];
        s.shi[k] = a.hdr->scene_hi[k];
    }
    s.U = a.hdr->n_unique;
    s.N = a.hdr->n_tris;
    return s;
}

__device__ __forceinline__ float pick3(uint32_t ax, float a, float b, float c) {
    return ax == 0 ? a : (ax == 1 ? b : c);
}

// RayTriangleIntersection (CUDAKernels.cu:17-50) on a {v0, e1, e2} record,
// returning t; with the C4 acceptance t_lo < t < FLT_MAX.
__device__ __forceinline__ bool mt_t(const float *__restrict__ tp, float ox, float oy, float oz, float dx,
                                     float dy, float dz, float t_lo, float &t) {
    const float v0x = tp[0], v0y = tp[1], v0z = tp[2];
    const float e1x = tp[3], e1y = tp[4], e1z = tp[5];
    const float e2x = tp[6], e2y = tp[7], e2z = tp[8];
    const float px = dy * e2z - e2y * dz;                  // pvec = cross(D, e2)
    const float py = dz * e2x - e2z * dx;
    const float pz = dx * e2y - e2x * dy;
    const float det = (e1x * px + e1y * py) + e1z * pz;
    if (det <= kDetEps) return false;                      // det < 0.000001 (double); NaN passes
    const float inv = 1.0f / det;
    const float sx = ox - v0x, sy = oy - v0y, sz = oz - v0z;
    const float u = ((sx * px + sy * py) + sz * pz) * inv;
    if (u < 0.0f || u > 1.0f) return false;
    const float qx = sy * e1z - e1y * sz;                  // qvec = cross(tvec, e1)
    const float qy = sz * e1x - e1z * sx;
    const float qz = sx * e1y - e1x * sy;
    const float v = ((dx * qx + dy * qy) + dz * qz) * inv;
    if (v < 0.0f || u + v > 1.0f) return false;
    t = ((e2x * qx + e2y * qy) + e2z * qz) * inv;
    return t > t_lo && t < FLT_MAX;
}

// Per-lane stack: slots [0, kWLds) in LDS at [slot * kWT] from this lane's
// base, deeper slots in this thread's HBM area (slot-major, grid-interleaved).
struct WStack {
    uint32_t *sn;
    float *smin, *smax;
    uint32_t *spill;           // + gtid; slot k >= kWLds at ((k - kWLds) * 3) * gthreads
    uint64_t gthreads;
    __device__ __forceinline__ void push(uint32_t sp, uint32_t n, float lo, float hi) const {
        if (sp < (uint32_t)kWLds) {
            sn[sp * kWT] = n; smin[sp * kWT] = lo; smax[sp * kWT] = hi;
        } else {
            uint32_t *q = spill + (uint64_t)(sp - kWLds) * 3 * gthreads;
            q[0] = n; q[gthreads] = __float_as_uint(lo); q[2 * gthreads] = __float_as_uint(hi);
        }
    }
    __device__ __forceinline__ void pop(uint32_t sp, uint32_t &n, float &lo, float &hi) const {
        if (sp < (uint32_t)kWLds) {
            n = sn[sp * kWT]; lo = smin[sp * kWT]; hi = smax[sp * kWT];
        } else {
            const uint32_t *q = spill + (uint64_t)(sp - kWLds) * 3 * gthreads;
            n = q[0]; lo = __uint_as_float(q[gthreads]); hi = __uint_as_float(q[2 * gthreads]);
        }
    }
};

// The C4 closest hit (the oracle's traverse_closest): the reference walk's
// decisions and order, min (t, i) at its leaves, and once a hit is known a
// node entered beyond it is popped and tMax is clamped to it.  bi = kNoHit on
// a miss.
__device__ void closest_walk(const WScene &s, float ox, float oy, float oz, float dx, float dy, float dz,
                             float t_lo, float &bt, uint32_t &bi, const WStack &stk) {
    bt = FLT_MAX;
    bi = kNoHit;
    const float ix = 1.0f / dx, iy = 1.0f / dy, iz = 1.0f / dz;
    const uint32_t sg = (ix < 0.0f ? 1u : 0u) | (iy < 0.0f ? 2u : 0u) | (iz < 0.0f ? 4u : 0u);
    // scene-AABB slab test, CUDAKernels.cu:237-262 (tMin may be negative)
    float tMin = (((sg & 1) ? s.shi[0] : s.slo[0]) - ox) * ix;
    float tMax = (((sg & 1) ? s.slo[0] : s.shi[0]) - ox) * ix;
    const float tymin = (((sg & 2) ? s.shi[1] : s.slo[1]) - oy) * iy;
    const float tymax = (((sg & 2) ? s.slo[1] : s.shi[1]) - oy) * iy;
    if ((tMin > tymax) || (tymin > tMax)) return;
    if (tymin > tMin) tMin = tymin;
    if (tymax < tMax) tMax = tymax;
    const float tzmin = (((sg & 4) ? s.shi[2] : s.slo[2]) - oz) * iz;
    const float tzmax = (((sg & 4) ? s.slo[2] : s.shi[2]) - oz) * iz;
    if ((tMin > tzmax) || (tzmin > tMax)) return;
    if (tzmin > tMin) tMin = tzmin;
    if (tzmax < tMax) tMax = tzmax;
    if (t_lo > 0.0f && tMin < t_lo) tMin = t_lo;   // a bounce's walk starts at its origin (oracle)
    if (s.U == 0) return;
    auto leaf = [&](uint32_t b, uint32_t e) {
        for (uint32_t i = b; i < e; ++i) {
            float t;
            if (mt_t(s.tris + 9ull * i, ox, oy, oz, dx, dy, dz, t_lo, t) && (t < bt || (t == bt && i < bi))) {
                bt = t;
                bi = i;
            }
        }
    };
    if (s.U == 1) {   // single leaf (reference: UB; defined as the oracle's)
        leaf(0, s.N);
        return;
    }
    uint32_t cur = 0, sp = 0;
    for (;;) {
        const float best = bi != kNoHit ? bt : __builtin_inff();
        if (tMin > best) {                           // entered beyond the best hit: skip
            if (sp == 0) return;
            --sp;
            stk.pop(sp, cur, tMin, tMax);
            continue;
        }
        if (best < tMax) tMax = best;
        const uint4 nd = s.nodes[cur];
        const uint32_t ax = (nd.z >> 27) & 3u;
        const float org = pick3(ax, ox, oy, oz), inv = pick3(ax, ix, iy, iz);
        const uint32_t nr = (sg >> ax) & 1u;
        const float t0 = (__uint_as_float(nd.x) - org) * inv;
        const float t1 = (__uint_as_float(nd.y) - org) * inv;
        const float tn = nr ? t1 : t0, tf = nr ? t0 : t1;
        const bool A = tMin < tn, B = tMax < tf;
        const uint32_t split = nd.z & kIdxMask, mid = nd.w & kIdxMask;
        const bool leafL = (nd.z >> 29) & 1u, leafR = (nd.z >> 30) & 1u;
        const bool leafN = nr ? leafR : leafL, leafF = nr ? leafL : leafR;
        uint32_t cL = (nd.w >> 27) & 3u, cR = (nd.w >> 29) & 3u;
        if (leafL && cL == 0) cL = s.dup[split];
        if (leafR && cR == 0) cR = s.dup[split + 1];
        const uint32_t nb = nr ? mid : mid - cL, ne = nr ? mid + cR : mid;
        const uint32_t fb = nr ? mid - cL : mid, fe = nr ? mid : mid + cR;
        const uint32_t nearc = split + nr, farc = split + 1u - nr;
        bool pop = false;
        if (!A && B) {
            pop = true;
        } else if (A && B) {
            if (leafN) { leaf(nb, ne); pop = true; }
            else { cur = nearc; tMax = tn; }
        } else if (!A && !B) {
            if (leafF) { leaf(fb, fe); pop = true; }
            else { cur = farc; tMin = tf; }
        } else {
            if (leafN && leafF) {
                leaf(nb, ne);
                leaf(fb, fe);
                pop = true;
            } else if (!leafN && leafF) {
                leaf(fb, fe);
                cur = nearc; tMax = tn;
            } else if (leafN && !leafF) {
                leaf(nb, ne);
                cur = farc; tMin = tf;
            } else {
                stk.push(sp, farc, tf, tMax);
                ++sp;
                cur = nearc; tMax = tn;
            }
        }
        if (pop) {
            if (sp == 0) return;
            --sp;
            stk.pop(sp, cur, tMin, tMax);
        }
    }
}

// Ray queue: 7 planes of `cap` words {ox, oy, oz, dx, dy, dz, sample}.
struct WQueue {
    float *p;
    uint64_t cap;
    __device__ __forceinline__ void put(uint64_t i, const float o[3], const float d[3], uint32_t sid) const {
        for (int k = 0; k < 3; ++k) {
            p[k * cap + i] = o[k];
            p[(3 + k) * cap + i] = d[k];
        }
        reinterpret_cast<uint32_t *>(p)[6 * cap + i] = sid;
    }
};

// counts[0..9]: rays in queue d (d = bounce depth).  With hit_mask (the
// primary samples' any-hit result from the frustum bins, one u64 per tile of
// TW x TH pixels, lane = pixel * spp + sample): only the samples that hit are
// queued for bounce 0, compacted per wave (ballot + mbcnt, one atomic on
// counts[0], zeroed before the launch); a sample the bins prove to miss has no
// closest hit either (the same visit set and test), so its depth stays 0.
__global__ void __launch_bounds__(kWT) k_wh_gen(const RenderArgs a, WQueue q, uint32_t *counts,
                                                uint8_t *hits, uint32_t *sort_hist,
                                                const unsigned long long *hit_mask, uint32_t tiles_x,
                                                uint32_t log2spp) {
    const uint64_t P = (uint64_t)a.nrows * a.w;
    const uint64_t rays = P * a.spp;
    const uint64_t gid = (uint64_t)blockIdx.x * kWT + threadIdx.x;
    // k_wh_sort_*'s histogram (zeroed again by each scan), whatever the grid
    for (uint64_t k = gid; k < kWSortBucketsGen; k += (uint64_t)gridDim.x * kWT) sort_hist[k] = 0u;
    if (gid == 0 && !hit_mask) {
        counts[0] = (uint32_t)rays;
        for (uint32_t k = 1; k < kWCounts; ++k) counts[k] = 0u;
    }
    const bool in = gid < rays;
    const uint64_t lp = in ? gid / a.spp : 0;
    const uint32_t s = (uint32_t)(gid % a.spp);
    const uint32_t lr = (uint32_t)(lp / a.w), x = (uint32_t)(lp % a.w);
    bool hit = in;
    if (hit_mask && in) {
        // TileShape: TW x TH pixels, TW * TH = 64 >> log2(spp)
        const uint32_t lpx = 6 - log2spp, tw = 1u << ((lpx + 1) / 2), th = 1u << (lpx / 2);
        const uint32_t tile = (lr / th) * tiles_x + x / tw;
        const uint32_t bit = (((lr % th) * tw + (x % tw)) << log2spp) + s;
        hit = (hit_mask[tile] >> bit) & 1ull;
    }
    uint64_t slot = gid;
    if (hit_mask) {
        const unsigned long long b = __ballot(hit);
        uint32_t base = 0;
        if (threadIdx.x == 0 && b) base = atomicAdd(counts, (uint32_t)__popcll(b));
        base = __builtin_amdgcn_readfirstlane(base);
        slot = base + __builtin_amdgcn_mbcnt_hi((uint32_t)(b >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)b, 0u));
    }
    if (in) hits[gid] = 0;
    if (!hit) return;
    // draws 2s, 2s+1 of this pixel's frame (cudaRender :413-415)
    uint32_t v[5];
    for (int i = 0; i < 5; ++i) v[i] = a.rng_in[(uint64_t)i * P + lp];
    uint32_t d = a.d_base;
    float ru = 0.f, rv = 0.f;
    for (uint32_t k = 0; k <= s; ++k) {
        ru = xorwow_uniform(v, d);
        rv = xorwow_uniform(v, d);
    }
    const uint32_t y = global_row(lr, a.row0, a.band_h, a.band_step);
    float dir[3];
    camera_dir(a, ((float)x + ru) / (float)a.w, ((float)y + rv) / (float)a.h, dir[0], dir[1], dir[2]);
    q.put(slot, a.cam, dir, (uint32_t)gid);
}

__global__ void __launch_bounds__(kWT) k_wh_trace(const RenderArgs a, uint32_t depth, WQueue qin, WQueue qout,
                                                  uint32_t *counts, uint8_t *hits, uint32_t *spill) {
    __shared__ uint32_t s_node[kWLds * kWT];
    __shared__ float s_min[kWLds * kWT];
    __shared__ float s_max[kWLds * kWT];
    const uint32_t lane = threadIdx.x;
    WStack stk;
    stk.sn = s_node + lane;
    stk.smin = s_min + lane;
    stk.smax = s_max + lane;
    stk.gthreads = (uint64_t)gridDim.x * kWT;
    stk.spill = spill + (uint64_t)blockIdx.x * kWT + lane;
    const WScene sc = load_wscene(a);
    const uint32_t n = counts[depth];
    const float t_lo = depth ? kBounceTLo : 0.0f;
    const uint32_t *sid_in = reinterpret_cast<const uint32_t *>(qin.p) + 6 * qin.cap;
    // wave-uniform loop over the queue (every lane takes part in the ballot)
    for (uint64_t base = (uint64_t)blockIdx.x * kWT; base < n; base += (uint64_t)gridDim.x * kWT) {
        const uint64_t i = base + lane;
        const bool valid = i < n;
        float o[3] = {0.f, 0.f, 0.f}, d[3] = {0.f, 0.f, 1.f};
        uint32_t sid = 0;
        float bt = FLT_MAX;
        uint32_t bi = kNoHit;
        if (valid) {
            for (int k = 0; k < 3; ++k) {
                o[k] = qin.p[k * qin.cap + i];
                d[k] = qin.p[(3 + k) * qin.cap + i];
            }
            sid = sid_in[i];
            closest_walk(sc, o[0], o[1], o[2], d[0], d[1], d[2], t_lo, bt, bi, stk);
        }
        const bool hit = valid && bi != kNoHit;
        if (hit) hits[sid] = (uint8_t)(depth + 1);
        // the mirror ray (oracle whitted_path), then compaction into qout
        const bool next = hit && depth < 8u;
        float po[3], rd[3];
        if (next) {
            const float *v = sc.tris + 9ull * bi;
            const float e1x = v[3], e1y = v[4], e1z = v[5], e2x = v[6], e2y = v[7], e2z = v[8];
            const float nx = e1y * e2z - e2y * e1z;        // n = cross(e1, e2), glm order
            const float ny = e1z * e2x - e2z * e1x;
            const float nz = e1x * e2y - e2x * e1y;
            const float dn = (d[0] * nx + d[1] * ny) + d[2] * nz;
            const float nn = (nx * nx + ny * ny) + nz * nz;
            const float kk = (2.0f * dn) / nn;
            const float nv[3] = {nx, ny, nz};
            for (int k = 0; k < 3; ++k) {
                const float td = bt * d[k];
                po[k] = o[k] + td;
                const float kn = kk * nv[k];
                rd[k] = d[k] - kn;
            }
        }
        const unsigned long long m = __ballot(next);
        if (m) {
            uint32_t first = 0;
            if (lane == 0) first = atomicAdd(counts + depth + 1, (uint32_t)__popcll(m));
            first = __builtin_amdgcn_readfirstlane(first);
            if (next) {
                const uint32_t r = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                                             __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
                qout.put((uint64_t)first + r, po, rd, sid);
            }
        }
    }
}

// k_wh_trace with per-lane ray fetching (U >= 2): a lane whose walk has
// ended takes the next ray of the queue while the other lanes of its wave
// keep walking, so a wave no longer waits for its slowest ray before taking
// 64 new ones (secondary rays trapped in the soup walk very unequal visit
// sets).  Each lane's walk is closest_walk's, step for step: one iteration of
// its loop per wave iteration, the same decisions, intervals, stack and (t, i)
// rule -- the same hit.  Idle lanes are refilled with one atomic per wave
// when a quarter of the wave is idle (or all of it).
#ifndef BIH_WH_REFILL
#define BIH_WH_REFILL 16   // idle lanes of a wave that trigger a refill
#endif
#ifndef BIH_WH_STEPS
#define BIH_WH_STEPS 256   // walk steps per lane between refill checks (A/B r03: 1 1.792 s, 2 1.777, 4 1.755 per 4K frame;
                           // r04y-zg after the one-round-trip step: 2 0.698, 4 0.680, 8 0.669, 16 0.660, 32 0.653,
                           // 64 0.645, 128 0.639, 256 0.635, 512 0.636, 1024 0.647: a refill stalls the whole wave
                           // on the new rays' loads, so fewer, larger refills pay until idle lanes wait too long)
#endif
// BIH_WH_PREFETCH: a step requests the next node's record before it tests
// the leaves it decided to visit, so the node load and the leaves' triangle
// loads are in flight together (one memory round trip per step instead of
// two); the record waits in the ray state for the next step.  The leaves are
// still tested before the next node's decisions read the best hit: the same
// decisions, the same hit.
#ifndef BIH_WH_MAXDIAG
#define BIH_WH_MAXDIAG 0   // diagnostic build: bih_whitted_work's triangles = the longest walk per bounce
#endif
#ifndef BIH_WH_PREFETCH
#define BIH_WH_PREFETCH 1
#endif
struct WRay {
    float o[3], d[3], ix, iy, iz, tMin, tMax, bt;
    uint32_t sg, cur, sp, bi, sid;
#if BIH_WH_PREFETCH
    uint4 nd;                  // the record of node cur (requested by the previous step)
#endif
};
__device__ __forceinline__ bool wray_start(const WScene &s, WRay &r, float t_lo) {
    r.bt = FLT_MAX;
    r.bi = kNoHit;
    r.cur = 0;
    r.sp = 0;
    r.ix = 1.0f / r.d[0];
    r.iy = 1.0f / r.d[1];
    r.iz = 1.0f / r.d[2];
    r.sg = (r.ix < 0.0f ? 1u : 0u) | (r.iy < 0.0f ? 2u : 0u) | (r.iz < 0.0f ? 4u : 0u);
    // scene-AABB slab test, CUDAKernels.cu:237-262 (as closest_walk)
    float tMin = (((r.sg & 1) ? s.shi[0] : s.slo[0]) - r.o[0]) * r.ix;
    float tMax = (((r.sg & 1) ? s.slo[0] : s.shi[0]) - r.o[0]) * r.ix;
    const float tymin = (((r.sg & 2) ? s.shi[1] : s.slo[1]) - r.o[1]) * r.iy;
    const float tymax = (((r.sg & 2) ? s.slo[1] : s.shi[1]) - r.o[1]) * r.iy;
    if ((tMin > tymax) || (tymin > tMax)) return false;
    if (tymin > tMin) tMin = tymin;
    if (tymax < tMax) tMax = tymax;
    const float tzmin = (((r.sg & 4) ? s.shi[2] : s.slo[2]) - r.o[2]) * r.iz;
    const float tzmax = (((r.sg & 4) ? s.slo[2] : s.shi[2]) - r.o[2]) * r.iz;
    if ((tMin > tzmax) || (tzmin > tMax)) return false;
    if (tzmin > tMin) tMin = tzmin;
    if (tzmax < tMax) tMax = tzmax;
    if (t_lo > 0.0f && tMin < t_lo) tMin = t_lo;   // a bounce's walk starts at its origin (oracle)
    r.tMin = tMin;
    r.tMax = tMax;
#if BIH_WH_PREFETCH
    r.nd = s.nodes[0];
#endif
    return true;
}
// one iteration of closest_walk's loop; true when the walk has ended.
// COUNT: nodes entered (cn) and triangles tested (ct) for the work counters.
template <bool COUNT>
__device__ __forceinline__ bool wray_step(const WScene &s, WRay &r, float t_lo, const WStack &stk, uint32_t &cn,
                                          uint32_t &ct) {
    auto leaf = [&](uint32_t b, uint32_t e) {
        if (COUNT) ct += e - b;
        for (uint32_t i = b; i < e; ++i) {
            float t;
            if (mt_t(s.tris + 9ull * i, r.o[0], r.o[1], r.o[2], r.d[0], r.d[1], r.d[2], t_lo, t) &&
                (t < r.bt || (t == r.bt && i < r.bi))) {
                r.bt = t;
                r.bi = i;
            }
        }
    };
    const float best = r.bi != kNoHit ? r.bt : __builtin_inff();
    if (r.tMin > best) {                          // entered beyond the best hit: skip
        if (r.sp == 0) return true;
        --r.sp;
        stk.pop(r.sp, r.cur, r.tMin, r.tMax);
#if BIH_WH_PREFETCH
        r.nd = s.nodes[r.cur];
#endif
        return false;
    }
    if (best < r.tMax) r.tMax = best;
    if (COUNT) ++cn;
#if BIH_WH_PREFETCH
    const uint4 nd = r.nd;
#else
    const uint4 nd = s.nodes[r.cur];
#endif
    const uint32_t ax = (nd.z >> 27) & 3u;
    const float org = pick3(ax, r.o[0], r.o[1], r.o[2]), inv = pick3(ax, r.ix, r.iy, r.iz);
    const uint32_t nr = (r.sg >> ax) & 1u;
    const float t0 = (__uint_as_float(nd.x) - org) * inv;
    const float t1 = (__uint_as_float(nd.y) - org) * inv;
    const float tn = nr ? t1 : t0, tf = nr ? t0 : t1;
    const bool A = r.tMin < tn, B = r.tMax < tf;
    const uint32_t split = nd.z & kIdxMask, mid = nd.w & kIdxMask;
    const bool leafL = (nd.z >> 29) & 1u, leafR = (nd.z >> 30) & 1u;
    const bool leafN = nr ? leafR : leafL, leafF = nr ? leafL : leafR;
    uint32_t cL = (nd.w >> 27) & 3u, cR = (nd.w >> 29) & 3u;
    if (leafL && cL == 0) cL = s.dup[split];
    if (leafR && cR == 0) cR = s.dup[split + 1];
    const uint32_t nb = nr ? mid : mid - cL, ne = nr ? mid + cR : mid;
    const uint32_t fb = nr ? mid - cL : mid, fe = nr ? mid : mid + cR;
    const uint32_t nearc = split + nr, farc = split + 1u - nr;
    // the leaves this step visits, in the walk's order: [l0b, l0e) then [l1b, l1e)
    uint32_t l0b = 0, l0e = 0, l1b = 0, l1e = 0;
    bool pop = false;
    if (!A && B) {
        pop = true;
    } else if (A && B) {
        if (leafN) { l0b = nb; l0e = ne; pop = true; }
        else { r.cur = nearc; r.tMax = tn; }
    } else if (!A && !B) {
        if (leafF) { l0b = fb; l0e = fe; pop = true; }
        else { r.cur = farc; r.tMin = tf; }
    } else {
        if (leafN && leafF) {
            l0b = nb; l0e = ne;
            l1b = fb; l1e = fe;
            pop = true;
        } else if (!leafN && leafF) {
            l0b = fb; l0e = fe;
            r.cur = nearc; r.tMax = tn;
        } else if (leafN && !leafF) {
            l0b = nb; l0e = ne;
            r.cur = farc; r.tMin = tf;
        } else {
            stk.push(r.sp, farc, tf, r.tMax);
            ++r.sp;
            r.cur = nearc; r.tMax = tn;
        }
    }
    bool fin = false;
    if (pop) {
        if (r.sp == 0) {
            fin = true;
        } else {
            --r.sp;
            stk.pop(r.sp, r.cur, r.tMin, r.tMax);
        }
    }
#if BIH_WH_PREFETCH
    if (!fin) r.nd = s.nodes[r.cur];
#endif
    leaf(l0b, l0e);
    leaf(l1b, l1e);
    return fin;
}
template <bool COUNT>
#ifndef BIH_WH_WAVES
#define BIH_WH_WAVES 0   // waves per SIMD forced on k_wh_trace_dyn (0: the compiler's choice)
#endif
#if BIH_WH_WAVES
#define BIH_WH_OCC __attribute__((amdgpu_waves_per_eu(BIH_WH_WAVES, BIH_WH_WAVES)))
#else
#define BIH_WH_OCC
#endif
__global__ void __launch_bounds__(kWT) BIH_WH_OCC k_wh_trace_dyn(const RenderArgs a, uint32_t depth, WQueue qin, WQueue qout,
                                                      uint32_t *counts, uint8_t *hits, uint32_t *spill,
                                                      unsigned long long *work) {
    uint32_t cn = 0, ct = 0;   // COUNT: nodes entered, triangles tested by this lane
#if BIH_WH_MAXDIAG
    uint32_t cn_ray0 = 0, cmax = 0;   // (diagnostic build: the longest walk, in nodes, reported as 'tris')
#endif
    __shared__ uint32_t s_node[kWLds * kWT];
    __shared__ float s_min[kWLds * kWT];
    __shared__ float s_max[kWLds * kWT];
    const uint32_t lane = threadIdx.x;
    WStack stk;
    stk.sn = s_node + lane;
    stk.smin = s_min + lane;
    stk.smax = s_max + lane;
    stk.gthreads = (uint64_t)gridDim.x * kWT;
    stk.spill = spill + (uint64_t)blockIdx.x * kWT + lane;
    const WScene sc = load_wscene(a);
    const uint32_t n = counts[depth];
    uint32_t *fetch = counts + kWFetch + depth;   // rays of queue `depth` taken so far
    const float t_lo = depth ? kBounceTLo : 0.0f;
    const uint32_t *sid_in = reinterpret_cast<const uint32_t *>(qin.p) + 6 * qin.cap;
    WRay r;
    bool has = false;          // this lane walks a ray
    bool more = true;          // (wave-uniform) the queue may still hold rays
    for (;;) {
        const unsigned long long idle = __ballot(!has);
        if (more && (__popcll(idle) >= BIH_WH_REFILL || idle == ~0ull)) {
            const uint32_t k = (uint32_t)__popcll(idle);
            uint32_t first = 0;
            if (lane == 0) first = atomicAdd(fetch, k);
            first = __builtin_amdgcn_readfirstlane(first);
            if ((uint64_t)first + k >= n) more = false;   // u64: no wrap of first + k
            if (!has) {
                const uint32_t rk = __builtin_amdgcn_mbcnt_hi((uint32_t)(idle >> 32),
                                                             __builtin_amdgcn_mbcnt_lo((uint32_t)idle, 0u));
                const uint64_t i = (uint64_t)first + rk;
                if (i < n) {
                    for (int c = 0; c < 3; ++c) {
                        r.o[c] = qin.p[c * qin.cap + i];
                        r.d[c] = qin.p[(3 + c) * qin.cap + i];
                    }
                    r.sid = sid_in[i];
                    has = wray_start(sc, r, t_lo);   // a ray that misses the scene box ends here: no hit
#if BIH_WH_MAXDIAG
                    cn_ray0 = cn;
#endif
                }
            }
        }
        if (!__ballot(has)) {
            if (!more) break;
            continue;
        }
        bool fin = false;
        if (has)
            for (int k = 0; k < BIH_WH_STEPS && !fin; ++k) fin = wray_step<COUNT>(sc, r, t_lo, stk, cn, ct);
#if BIH_WH_MAXDIAG
        if (fin && cn - cn_ray0 > cmax) cmax = cn - cn_ray0;
#endif
        const bool hit = fin && r.bi != kNoHit;
        if (hit) hits[r.sid] = (uint8_t)(depth + 1);
        // the mirror ray (oracle whitted_path), then compaction into qout
        const bool next = hit && depth < 8u;
        float po[3], rd[3];
        if (next) {
            const float *v = sc.tris + 9ull * r.bi;
            const float e1x = v[3], e1y = v[4], e1z = v[5], e2x = v[6], e2y = v[7], e2z = v[8];
            const float nx = e1y * e2z - e2y * e1z;        // n = cross(e1, e2), glm order
            const float ny = e1z * e2x - e2z * e1x;
            const float nz = e1x * e2y - e2x * e1y;
            const float dn = (r.d[0] * nx + r.d[1] * ny) + r.d[2] * nz;
            const float nn = (nx * nx + ny * ny) + nz * nz;
            const float kk = (2.0f * dn) / nn;
            const float nv[3] = {nx, ny, nz};
            for (int k = 0; k < 3; ++k) {
                const float td = r.bt * r.d[k];
                po[k] = r.o[k] + td;
                const float kn = kk * nv[k];
                rd[k] = r.d[k] - kn;
            }
        }
        const unsigned long long m = __ballot(next);
        if (m) {
            uint32_t first = 0;
            if (lane == 0) first = atomicAdd(counts + depth + 1, (uint32_t)__popcll(m));
            first = __builtin_amdgcn_readfirstlane(first);
            if (next) {
                const uint32_t rk = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                                             __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
                qout.put((uint64_t)first + rk, po, rd, r.sid);
            }
        }
        if (fin) has = false;
    }
    if (COUNT) {   // work[2 depth] += nodes, work[2 depth + 1] += triangles (per wave, u64)
        unsigned long long n64 = cn, t64 = ct;
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) {
            n64 += __shfl_xor(n64, off, 64);
            t64 += __shfl_xor(t64, off, 64);
        }
#if BIH_WH_MAXDIAG
        unsigned long long m64 = cmax;
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) {
            const unsigned long long o = __shfl_xor(m64, off, 64);
            m64 = o > m64 ? o : m64;
        }
        if (lane == 0) {
            atomicAdd(work + 2 * depth, n64);
            atomicMax(work + 2 * depth + 1, m64);
        }
#else
        if (lane == 0) {
            atomicAdd(work + 2 * depth, n64);
            atomicAdd(work + 2 * depth + 1, t64);
        }
#endif
    }
}

// Ray order of a bounce queue (round 4).  The rays of queue d+1 arrive in the
// order their waves finished, so neighbouring lanes start unrelated walks.
// Before bounce d+1 the queue is reordered by a key of origin cell (3 bits of
// the scene box per axis, Morton-interleaved) x direction octant: lanes and
// waves of one XCD then walk neighbouring subtrees, and the node / triangle
// lines they share stay in that XCD's L2.  A counting sort (k_wh_sort_count,
// k_wh_sort_scan, k_wh_sort_scatter); the order within a bucket is arbitrary.
// No result depends on the queue order (each ray carries its sample id and
// its walk is its own), so the pixels and hit counts are unchanged.
constexpr uint32_t kWSortBits = BIH_WH_SORT_BITS;              // cells per axis: 2^bits
constexpr uint32_t kWSortBuckets = (8u << (3 * kWSortBits)) << (BIH_WH_SORT_DIR ? 2 : 0);   // x 8 octants (3 bits: 4096)
constexpr bool kWSortLds = kWSortBuckets == 4096;               // counts aggregated in LDS per block
constexpr uint32_t kWSortChunk = 4096;                          // rays per sort block (16 per thread)
__device__ __forceinline__ uint32_t wh_cell(float o, float lo, float hi) {
    const float q = (o - lo) / (hi - lo) * (float)(1u << kWSortBits);
    // NaN and out-of-box origins clamp (any key is correct, only the order changes)
    return q >= 1.0f ? (q < (float)((1u << kWSortBits) - 1u) ? (uint32_t)q : (1u << kWSortBits) - 1u) : 0u;
}
__device__ __forceinline__ uint32_t wh_sort_key(const WScene &s, const WQueue &q, uint64_t i) {
    uint32_t cell = 0;
    for (int c = 0; c < 3; ++c) {
        const uint32_t v = wh_cell(q.p[c * q.cap + i], s.slo[c], s.shi[c]);
        for (uint32_t b = 0; b < kWSortBits; ++b) cell |= ((v >> b) & 1u) << (3 * b + (2 - c));
    }
    const float dx = q.p[3 * q.cap + i], dy = q.p[4 * q.cap + i], dz = q.p[5 * q.cap + i];
    const uint32_t oct = (dx < 0.0f ? 1u : 0u) | (dy < 0.0f ? 2u : 0u) | (dz < 0.0f ? 4u : 0u);
#if BIH_WH_SORT_DIR
    const float ax = fabsf(dx), ay = fabsf(dy), az = fabsf(dz);
    const uint32_t dom = (ax >= ay && ax >= az) ? 0u : (ay >= az ? 1u : 2u);
    return (((cell << 3) | oct) << 2) | dom;
#else
    return (cell << 3) | oct;
#endif
}
// Per-block bucket counts of queue q's rays [blockIdx.x * chunk, +chunk) into
// LDS; SCATTER = false adds them to the global histogram, true reserves each
// non-zero bucket's range at its cursor and copies the rays to qout.
template <bool SCATTER>
__global__ void __launch_bounds__(256) k_wh_sort_pass(const RenderArgs a, uint32_t depth, WQueue qin, WQueue qout,
                                                      const uint32_t *counts, uint32_t *hist) {
    __shared__ uint32_t s_cnt[kWSortLds ? kWSortBuckets : 1];
    __shared__ uint32_t s_base[(SCATTER && kWSortLds) ? kWSortBuckets : 1];
    const uint32_t n = counts[depth];
    const uint64_t c0 = (uint64_t)blockIdx.x * kWSortChunk;
    if (c0 >= n) return;
    if (!kWSortLds) {
        // finer keys: one global atomic per ray (count, then the ray's slot)
        const WScene sc = load_wscene(a);
        const uint32_t *sid_in = reinterpret_cast<const uint32_t *>(qin.p) + 6 * qin.cap;
        uint32_t *cur = hist + kWSortBuckets;
        for (uint32_t r = 0; r < kWSortChunk / 256; ++r) {
            const uint64_t i = c0 + r * 256 + threadIdx.x;
            if (i >= n) continue;
            const uint32_t key = wh_sort_key(sc, qin, i);
            if (!SCATTER) {
                atomicAdd(hist + key, 1u);
            } else {
                const uint64_t j = atomicAdd(cur + key, 1u);
                float o[3], d[3];
                for (int c = 0; c < 3; ++c) {
                    o[c] = qin.p[c * qin.cap + i];
                    d[c] = qin.p[(3 + c) * qin.cap + i];
                }
                qout.put(j, o, d, sid_in[i]);
            }
        }
        return;
    }
    for (uint32_t k = threadIdx.x; k < kWSortBuckets; k += 256) s_cnt[k] = 0u;
    __syncthreads();
    const WScene sc = load_wscene(a);
    uint32_t key[kWSortChunk / 256], rank[kWSortChunk / 256];
#pragma unroll
    for (uint32_t r = 0; r < kWSortChunk / 256; ++r) {
        const uint64_t i = c0 + r * 256 + threadIdx.x;
        key[r] = i < n ? wh_sort_key(sc, qin, i) : 0u;
        rank[r] = i < n ? atomicAdd(&s_cnt[key[r]], 1u) : 0u;
    }
    __syncthreads();
    uint32_t *cur = hist + kWSortBuckets;   // [kWSortBuckets, 2 kWSortBuckets): scatter cursors
    for (uint32_t k = threadIdx.x; k < kWSortBuckets; k += 256) {
        const uint32_t c = s_cnt[k];
        if (SCATTER) s_base[k] = c ? atomicAdd(cur + k, c) : 0u;
        else if (c) atomicAdd(hist + k, c);
    }
    if (!SCATTER) return;
    __syncthreads();
    const uint32_t *sid_in = reinterpret_cast<const uint32_t *>(qin.p) + 6 * qin.cap;
#pragma unroll
    for (uint32_t r = 0; r < kWSortChunk / 256; ++r) {
        const uint64_t i = c0 + r * 256 + threadIdx.x;
        if (i >= n) continue;
        const uint64_t j = s_base[key[r]] + rank[r];
        float o[3], d[3];
        for (int c = 0; c < 3; ++c) {
            o[c] = qin.p[c * qin.cap + i];
            d[c] = qin.p[(3 + c) * qin.cap + i];
        }
        qout.put(j, o, d, sid_in[i]);
    }
}
// Bucket starts: cursors = exclusive scan of the histogram; the histogram is
// zeroed for the next bounce's count (one block of 1024 threads, kPer buckets each).
constexpr uint32_t kWSortPer = kWSortBuckets / 1024;
__global__ void __launch_bounds__(1024) k_wh_sort_scan(uint32_t *hist) {
    __shared__ uint32_t s_w[16];
    const uint32_t t = threadIdx.x, lane = t & 63u, w = t >> 6;
    uint32_t v[kWSortPer], sum = 0;
    for (uint32_t k = 0; k < kWSortPer; ++k) {
        v[k] = hist[kWSortPer * t + k];
        sum += v[k];
    }
    uint32_t inc = sum;
    for (uint32_t d = 1; d < 64u; d <<= 1) {
        const uint32_t y = __shfl_up(inc, d, 64);
        if (lane >= d) inc += y;
    }
    if (lane == 63u) s_w[w] = inc;
    __syncthreads();
    uint32_t run = inc - sum;
    for (uint32_t k = 0; k < w; ++k) run += s_w[k];
    for (uint32_t k = 0; k < kWSortPer; ++k) {
        hist[kWSortBuckets + kWSortPer * t + k] = run;
        hist[kWSortPer * t + k] = 0u;
        run += v[k];
    }
}
static_assert(kWSortBuckets % 1024 == 0, "k_wh_sort_scan: 1024 threads x kWSortPer buckets");
static_assert(kWSortBuckets == kWSortBucketsGen, "k_wh_gen zeroes every bucket");

// shade of a sample with h hits (oracle whitted_shade), f32
__device__ __forceinline__ void wh_shade(uint32_t h, float &r, float &g, float &b) {
    if (h > 8u) { r = 255.0f; g = 255.0f; b = 0.0f; h = 8u; }
    else { r = 20.0f; g = 20.0f; b = 40.0f; }
    for (uint32_t k = 0; k < h; ++k) {
        r = 0.5f * 255.0f + 0.5f * r;
        g = 0.5f * 255.0f + 0.5f * g;
        b = 0.5f * 0.0f + 0.5f * b;
    }
}

__global__ void __launch_bounds__(256) k_wh_shade(const RenderArgs a, const uint8_t *hits, uint32_t *d_hits) {
    const uint64_t P = (uint64_t)a.nrows * a.w;
    const uint64_t lp = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (lp >= P) return;
    float cr = 0.f, cg = 0.f, cb = 0.f;
    for (uint32_t s = 0; s < a.spp; ++s) {
        const uint32_t h = hits[lp * a.spp + s];
        if (d_hits) d_hits[lp * a.spp + s] = h;
        float r, g, b;
        wh_shade(h, r, g, b);
        cr += r; cg += g; cb += b;                     // col += Color(...), sample order
    }
    const float fs = (float)a.spp;
    a.out[lp] = rgb_to_int(cr / fs, cg / fs, cb / fs);
}

}  // namespace

static uint32_t whitted_grid(uint64_t rays) {
    int dev = 0, cus = 256;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    const uint64_t need = (rays + kWT - 1) / kWT, cap = (uint64_t)(cus > 0 ? cus : 256) * kWBlocksPerCU;
    return (uint32_t)(need < cap ? need : cap);
}

// two queues of 7 planes, 16 counters, per-sample hits (u8), the stack
// spill, the ray-order histogram and cursors
static uint64_t whitted_spill_words(uint64_t rays) {
    return (uint64_t)whitted_grid(rays) * kWT * (kWStack - kWLds) * 3;
}
size_t whitted_bytes(uint64_t rays) {
    const uint64_t q = 2 * 7 * rays * 4, hits = (rays + 255) & ~255ull;
    return q + kWCounts * 4 + hits + whitted_spill_words(rays) * 4 + 2 * kWSortBuckets * 4 + kWWorkWords * 8;
}
// the work counters of the last launch_whitted with counters on (u64[2 x 9]:
// nodes, triangles per bounce) and its rays per bounce (u32[9])
int whitted_work(const void *mem, uint64_t rays, uint32_t ray_counts[9], unsigned long long work[18],
                 void *stream) {
    const hipStream_t st = (hipStream_t)stream;
    const char *base = reinterpret_cast<const char *>(mem);
    const uint32_t *counts = reinterpret_cast<const uint32_t *>(base + 14 * rays * 4);
    const uint8_t *hits = reinterpret_cast<const uint8_t *>(counts + kWCounts);
    const uint32_t *spill = reinterpret_cast<const uint32_t *>(hits + ((rays + 255) & ~255ull));
    const unsigned long long *w =
        reinterpret_cast<const unsigned long long *>(spill + whitted_spill_words(rays) + 2 * kWSortBuckets);
    hipError_t e = hipMemcpyAsync(ray_counts, counts, 9 * 4, hipMemcpyDeviceToHost, st);
    if (e == hipSuccess) e = hipMemcpyAsync(work, w, 18 * 8, hipMemcpyDeviceToHost, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    return (int)e;
}

int launch_whitted(const RenderArgs &a, void *mem, uint64_t rays, uint32_t *d_hits, void *stream, void *ev_k0,
                   void *ev_k1, bool count, const unsigned long long *hit_mask, uint32_t tiles_x) {
    const hipStream_t st = (hipStream_t)stream;
    if (rays == 0) return 0;
    float *base = reinterpret_cast<float *>(mem);
    WQueue q0{base, rays}, q1{base + 7 * rays, rays};
    uint32_t *counts = reinterpret_cast<uint32_t *>(base + 14 * rays);
    uint8_t *hits = reinterpret_cast<uint8_t *>(counts + kWCounts);
    uint32_t *spill = reinterpret_cast<uint32_t *>(hits + ((rays + 255) & ~255ull));
    uint32_t *hist = spill + whitted_spill_words(rays);
    unsigned long long *work = reinterpret_cast<unsigned long long *>(hist + 2 * kWSortBuckets);
    if (count) {
        const hipError_t ez = hipMemsetAsync(work, 0, kWWorkWords * 8, st);
        if (ez != hipSuccess) return (int)ez;
    }
    if (hit_mask) {
        // k_wh_gen appends the primary samples that hit to queue 0
        const hipError_t ez = hipMemsetAsync(counts, 0, kWCounts * 4, st);
        if (ez != hipSuccess) return (int)ez;
    }
    hipLaunchKernelGGL(k_wh_gen, dim3((uint32_t)((rays + kWT - 1) / kWT)), dim3(kWT), 0, st, a, q0, counts, hits,
                       hist, hit_mask, tiles_x, (uint32_t)__builtin_ctz(a.spp));
    hipError_t e = ev_k0 ? hipEventRecord((hipEvent_t)ev_k0, st) : hipSuccess;
    if (e != hipSuccess) return (int)e;
    const uint32_t grid = whitted_grid(rays);
    // per-lane ray fetching (k_wh_trace_dyn) needs internal nodes; a one-leaf
    // tree (or BIH_WH_STATIC=1, A/B) takes the wave-per-64-rays kernel
    static const bool dyn_on = [] {
        const char *e = getenv("BIH_WH_STATIC");
        return !(e && e[0] == '1');
    }();
    const bool dyn = dyn_on && a.n_nodes > 0;
    // ray order (k_wh_sort_*; BIH_WH_SORT=0 for A/B): queue d+1 is written to
    // q1 and sorted back into q0, so every bounce reads q0
    static const bool sort_on = [] {
        const char *e = getenv("BIH_WH_SORT");
        return !(e && e[0] == '0');
    }();
    const bool srt = sort_on && a.n_nodes > 0;
    const uint32_t sort_blocks = (uint32_t)((rays + kWSortChunk - 1) / kWSortChunk);
    for (uint32_t d = 0; d <= 8; ++d) {
        const WQueue &qi = (srt || !(d & 1)) ? q0 : q1, &qo = (srt || !(d & 1)) ? q1 : q0;
        if (dyn && count)
            hipLaunchKernelGGL(k_wh_trace_dyn<true>, dim3(grid), dim3(kWT), 0, st, a, d, qi, qo, counts, hits, spill,
                               work);
        else if (dyn)
            hipLaunchKernelGGL(k_wh_trace_dyn<false>, dim3(grid), dim3(kWT), 0, st, a, d, qi, qo, counts, hits, spill,
                               work);
        else
            hipLaunchKernelGGL(k_wh_trace, dim3(grid), dim3(kWT), 0, st, a, d, qi, qo, counts, hits, spill);
        if (srt && d < 8) {
            hipLaunchKernelGGL(k_wh_sort_pass<false>, dim3(sort_blocks), dim3(256), 0, st, a, d + 1, q1, q0,
                               counts, hist);
            hipLaunchKernelGGL(k_wh_sort_scan, dim3(1), dim3(1024), 0, st, hist);
            hipLaunchKernelGGL(k_wh_sort_pass<true>, dim3(sort_blocks), dim3(256), 0, st, a, d + 1, q1, q0,
                               counts, hist);
        }
    }
    e = ev_k1 ? hipEventRecord((hipEvent_t)ev_k1, st) : hipSuccess;
    if (e != hipSuccess) return (int)e;
    const uint64_t P = (uint64_t)a.nrows * a.w;
    hipLaunchKernelGGL(k_wh_shade, dim3((uint32_t)((P + 255) / 256)), dim3(256), 0, st, a, hits, d_hits);
    return (int)hipGetLastError();
}

}  // namespace bih
