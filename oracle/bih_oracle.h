/*
 * bih_oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * Strict-IEEE binary32 CPU restatement of the reference hot path
 * (rehakvoj1/BIH-GPU-Raytracer: per-frame BIH build + cudaRender).  Only
 * tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load
 * this library, and only as the checker / CPU baseline -- never as the
 * product path.  The product is bih-gpu-raytracer_amd/ (HIP, gfx950).
 *
 * Parity status: pinned structurally by the reference's only fixture
 * (BIH1.txt tree dump, see tests/test_oracle_fixture.py); the cuRAND XORWOW
 * constants are restated from cuRAND's public headers and are "parity
 * unpinned" at that boundary.
 */
#ifndef BIH_ORACLE_H
#define BIH_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Canonical tree arrays, same meaning as the reference's GPUArrayManager
 * buffers (src/GPUArrayManager.h:46-55, src/Tree.cuh:16-24).  Node arrays
 * have U-1 entries (reference allocates N-1, App.cpp:83; only U-1 are live). */
typedef struct ob_tree {
    int32_t n_tris;
    int32_t n_unique;            /* U */
    float scene_lo[3], scene_hi[3];
    float *lo, *hi, *center, *norm;   /* n*3 each (AABBs arrays, AABB.h:14-21) */
    uint32_t *morton;            /* n, sorted codes (Renderer.cpp:441-445)      */
    uint32_t *tri_idx;           /* n, trisIndexes after stable sort             */
    uint32_t *unique_mc;         /* U */
    uint32_t *dup_cnt;           /* U */
    int32_t *first_idx;          /* U */
    int32_t *leaf_parent;        /* U */
    float *clip;                 /* 2*(U-1) */
    int32_t *axis;               /* U-1 */
    int32_t *children;           /* 2*(U-1) */
    uint8_t *is_leaf;            /* 2*(U-1) */
    int32_t *parent;             /* U-1 */
    float *tris;                 /* n*9 copy of the input soup (Triangle[])     */
} ob_tree;

/* traversal modes */
#define OB_MODE_GPU_REF      0  /* cudaRender/TraverseTree, CUDAKernels.cu:227-368   */
#define OB_MODE_BRUTE        1  /* all triangles, TraverseTriangles-style check     */
#define OB_MODE_HOST_DEBUG   2  /* CPUTraverseTree, Renderer.cpp:202-349             */
#define OB_MODE_GPU_ANYHIT   3  /* mode 0 stopped at the first valid hit (same RGBA) */

typedef struct ob_stats {
    uint64_t rays, rays_hit;
    uint64_t node_visits;        /* iterations of the traversal loop */
    uint64_t leaf_visits;        /* FindNearestTriangle calls        */
    uint64_t tri_tests;          /* RayTriangleIntersection calls    */
    uint64_t slab_miss;          /* rays rejected by the scene slab  */
    int32_t max_stack;           /* deepest stack (excluding sentinel) */
    int32_t threads;
    double render_seconds;       /* wall time of the traversal loop only */
    uint64_t push_at[33];        /* stack pushes by slot index (32 = deeper)  */
} ob_stats;

int  ob_build(const float *v, int32_t n, ob_tree **out);
void ob_free(ob_tree *t);

/* Camera::Camera(origin=(2,0,-2), aspect=(float)W/H), Renderer.cpp:99,
 * Camera.cu:5-9.  cam = origin, lower_left, horizontal, vertical (12 f32). */
void ob_camera_reference(uint32_t w, uint32_t h, float cam[12]);

/* XORWOW (cuRAND curand_init(seed, subseq, 0) + skip) state for one pixel. */
void ob_rng_state(uint64_t seed, uint64_t subsequence, uint64_t skip,
                  uint32_t v[5], uint32_t *d);
uint32_t ob_rng_next(uint32_t v[5], uint32_t *d);
float ob_rng_uniform(uint32_t v[5], uint32_t *d);

/* Renders rows y = row0 + k*row_step, k < nrows, of a w*h frame into
 * out[k*w + x] (0x00BBGGRR, row 0 = bottom).  frame f consumes RNG draws
 * [2*spp*f, 2*spp*(f+1)) of each pixel's subsequence (pixel = y*w + x).
 * ray_counts (optional) receives {node visits, leaf visits, triangle tests}
 * per ray at [3*((k*w + x)*spp + s)]. */
int ob_render(const ob_tree *t, const float cam[12], uint32_t w, uint32_t h,
              uint32_t spp, uint32_t frame, uint64_t seed,
              uint32_t row0, uint32_t nrows, uint32_t row_step,
              uint32_t *out, int mode, int nthreads, ob_stats *stats,
              uint32_t *ray_counts);

/* Config C4 (BASELINE.json configs[3]): 8-bounce Whitted mirror rays.  A
 * build-defined extension (the reference has no secondary rays,
 * CUDAKernels.cu:370-389); semantics, all f32 without contraction:
 *   closest hit of a ray = min (t, sorted position i) over the triangles the
 *     reference walk tests (TraverseTree's decisions and order,
 *     CUDAKernels.cu:227-368; RayTriangleIntersection :17-50) with
 *     t_lo < t < FLT_MAX (depth 0: t > 0 as FindNearestTriangle :212;
 *     bounces: t > 1e-4), where the walk culls front to back once it has a
 *     hit: before each node, pop if tMin > best, else tMax = min(tMax, best);
 *     a bounce's walk interval starts at max(scene-box entry, 1e-4), not at
 *     the box entry behind its origin (round 4);
 *   hit point P = O + t*D; n = cross(e1, e2) (glm order, e = v - v0 of the
 *     original triangle); k = (2*dot(D, n)) / dot(n, n); R = D - k*n;
 *   shade(d) = miss ? (20,20,40) : d == 8 ? (255,255,0)
 *              : 0.5*(255,255,0) + 0.5*shade(d+1)   (d = 0 primary .. 8)
 *   pixel = rgbToInt(sum of the spp samples / spp) as cudaRender (:420-422).
 * The shades are dyadic, so the pixel depends only on each sample's hit
 * count h (0..9): bit-exact.  depth_out (optional) receives h per sample at
 * [(k*w + x)*spp + s]. */
#define OB_WHITTED_BOUNCES 8
int ob_render_whitted(const ob_tree *t, const float cam[12], uint32_t w, uint32_t h,
                      uint32_t spp, uint32_t frame, uint64_t seed,
                      uint32_t row0, uint32_t nrows, uint32_t row_step,
                      uint32_t *out, int nthreads, ob_stats *stats, uint8_t *depth_out);
/* One closest-hit query with the C4 rule (tests): *t_out, *idx_out (sorted
 * position, -1 on a miss) for ray (o, d) accepting t_lo < t < FLT_MAX. */
int ob_closest(const ob_tree *t, const float o[3], const float d[3], float t_lo,
               float *t_out, int32_t *idx_out);

/* Per-ray hit flag + counters for a list of explicit rays (tests). */
int ob_trace_rays(const ob_tree *t, const float *orig, const float *dir, int32_t n,
                  int mode, uint8_t *hit, uint32_t *nodes, uint32_t *tris);

/* Möller–Trumbore exactly as RayTriangleIntersection (CUDAKernels.cu:17-50). */
int ob_mt(const float tri[9], const float o[3], const float d[3], float *t_out);

uint32_t ob_morton3d(float x, float y, float z);

#ifdef __cplusplus
}
#endif
#endif
