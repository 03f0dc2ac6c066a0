/*
 * bih.h -- C ABI of the MI355X-native BIH ray tracer (libbih_amd.so).
 *
 * Drop-in boundary for the reference's hot path (rehakvoj1/BIH-GPU-Raytracer,
 * paths relative to BIH_Raytracer/BIH_Raytracer/):
 *
 *   bih_build   replaces Renderer::Render steps 1-7 (src/Renderer.cpp:422-503:
 *               Morton transform, stable_sort_by_key, reduce_by_key,
 *               unique_by_key_copy, Launch_BuildTree, Launch_FindClipPlanes)
 *               plus the host scene prep of App::LoadModels (src/App.cpp:95-164).
 *   bih_render  replaces Renderer::Launch_cudaRender (src/Renderer.h:27,
 *               src/CUDAKernels.cu:425-447 -> cudaRender :391-423) including the
 *               persistent cuRAND state of InitRandGPU (:450-463) and the
 *               framebuffer writeback g_odata[j*W+i] = rgbToInt(col) (:420-422).
 *   bih_camera_reference  replaces `new Camera(vec3(2,0,-2), (float)W/H)`
 *               (src/Renderer.cpp:99, src/Camera.cu:5-9).
 *
 * Conventions: every call is synchronous, returns 0 or a negative BIH_ERR_*
 * code (never exits; the reference's checkCudaErrors calls exit(99),
 * src/Renderer.cpp:63-73), and touches exactly one device (the one the tree
 * was built on).  The caller owns scenes and host framebuffers; the library
 * owns device memory (scene, tree, per-pixel RNG state).  Distinct trees may
 * be used concurrently from distinct host threads.  No HIP/torch types cross
 * this boundary: streams are passed as void* (hipStream_t), device buffers as
 * plain pointers.
 */
#ifndef BIH_H
#define BIH_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define BIH_ABI_VERSION 4   /* 2: bih_tree_info.device_allocs, bih_reserve, bih_tree_set_param;
                               3: bih_whitted_work, BIH_PARAM_WHITTED_COUNTERS;
                               4: bih_host_register / bih_host_unregister, bih_render_history */

/* error codes */
#define BIH_OK               0
#define BIH_ERR_INVALID     -1   /* bad argument / shape                     */
#define BIH_ERR_NO_DEVICE   -2   /* no HIP device, or device index invalid   */
#define BIH_ERR_HIP         -3   /* HIP runtime error                        */
#define BIH_ERR_OOM         -4   /* device or host allocation failed         */
#define BIH_ERR_NONFINITE   -5   /* scene holds a NaN/Inf coordinate         */
#define BIH_ERR_TOO_LARGE   -6   /* more than BIH_MAX_TRIS triangles         */
#define BIH_ERR_MISMATCH    -7   /* scene does not belong to this tree       */
#define BIH_ERR_IO          -8   /* file could not be opened / read          */
#define BIH_ERR_PARSE       -9   /* malformed scene file                     */

#define BIH_MAX_TRIS (1u << 27)

/* Triangle soup, file order (App.cpp:108-121 flattening): v[9*i .. 9*i+8] =
 * v0.xyz, v1.xyz, v2.xyz of triangle i.  Host-owned. */
typedef struct bih_scene {
    uint32_t n_tris;
    const float *v;
} bih_scene;

/* Opaque BIH; built by bih_build*, owned by the library, freed by bih_free. */
typedef struct bih_tree bih_tree;

/* == Camera members m_origin, m_lowerLeftCorner, m_horizontal, m_vertical
 * (src/Camera.h:14-17).  Ray(u,v) = Ray(origin,
 * lower_left + u*horizontal + v*vertical - origin), Camera.cu:18-20. */
typedef struct bih_camera {
    float origin[3], lower_left[3], horizontal[3], vertical[3];
} bih_camera;

/* Host framebuffer: w*h uint32 0x00BBGGRR, row 0 = bottom (GL convention).
 * Frame f consumes cuRAND draws [2*spp*f, 2*spp*(f+1)) of the XORWOW
 * subsequence `pixel = y*w + x` seeded with `seed` (reference: 1984). */
typedef struct bih_framebuffer {
    uint32_t w, h, spp, frame;
    uint64_t seed;
    uint32_t *rgba;
} bih_framebuffer;

/* Traversal flavours; both produce bit-identical RGBA.
 * BIH_TRAVERSE_REFERENCE visits exactly the nodes/leaves/triangles of
 * TraverseTree (CUDAKernels.cu:227-368).  BIH_TRAVERSE_ANYHIT (default)
 * computes only the one bit per sample Color() (:370-389) consumes: does the
 * reference walk reach a triangle that sets rec.triangleIdx.  It answers
 * through the camera's frustum bins (per 4x4-pixel tile the triangles whose
 * proven edge pre-test a sample can pass, each candidate hit verified against
 * the reference walk's decisions on its root path),
 * and whatever a tile list cannot decide -- or a render the bins do not
 * cover -- takes the any-hit BIH walk, which stops at the first such
 * triangle. */
#define BIH_TRAVERSE_ANYHIT     0u
#define BIH_TRAVERSE_REFERENCE  1u

/* Row tiling for bih_render_device: local row r (0 <= r < nrows) is global
 * row y = row0 + (r / band_h) * band_h * band_step + (r % band_h).
 * {row0, nrows, band_h=nrows, band_step=1} = contiguous block;
 * {rank*B, rows_of_rank, B, world} = interleaved bands of B rows. */
typedef struct bih_rows {
    uint32_t row0, nrows, band_h, band_step;
} bih_rows;

typedef struct bih_tree_info {
    uint32_t n_tris, n_unique;            /* N, U (U-1 internal nodes)        */
    float scene_lo[3], scene_hi[3];       /* App.cpp:133-137 scene AABB        */
    int device;
    uint64_t device_bytes;                /* device memory held by the tree    */
    double build_ms;                      /* device time of the last build     */
    uint64_t device_allocs;               /* device allocations the tree made so
                                             far (a steady-state frame loop adds
                                             none: see bih_reserve)              */
} bih_tree_info;

/* Canonical arrays for parity checks (reference buffer names in brackets). */
enum bih_array {
    BIH_ARR_MORTON_SORTED = 0, /* u32[N]  [m_mortonCodes after sort]          */
    BIH_ARR_TRI_INDEX,         /* u32[N]  [m_trisIndexes]                      */
    BIH_ARR_UNIQUE_MC,         /* u32[U]  [m_uniqueMortonCodes]                */
    BIH_ARR_DUP_COUNT,         /* u32[U]  [m_duplicatesCnts]                   */
    BIH_ARR_FIRST_IDX,         /* i32[U]  [m_firstIdxs]                        */
    BIH_ARR_LEAF_PARENT,       /* i32[U]  [m_leafParents]                      */
    BIH_ARR_CLIP,              /* f32[2*(U-1)] [TreeInternalNode::t_clipPlanes]*/
    BIH_ARR_AXIS,              /* i32[U-1]    [t_axis]                         */
    BIH_ARR_CHILDREN,          /* i32[2*(U-1)] [children]                      */
    BIH_ARR_IS_LEAF,           /* u8[2*(U-1)]  [isLeaf]                        */
    BIH_ARR_PARENT,            /* i32[U-1]    [parent]                         */
    BIH_ARR_TRI_LO,            /* f32[3N] [AABBs::arrLo]                       */
    BIH_ARR_TRI_HI,            /* f32[3N] [AABBs::arrHi]                       */
    BIH_ARR_COUNT
};

int bih_device_count(void);
const char *bih_strerror(int code);
int bih_abi_version(void);

int bih_camera_reference(uint32_t w, uint32_t h, bih_camera *out);
/* Host only: an upper bound, per component, of |D| over every primary ray of
 * `camera` as the render kernel evaluates D = ((llc + u*h) + v*vert) - origin
 * in f32 for u, v in [0, 1] (Camera.cu:18-20).  The any-hit walk's miss-proof
 * boxes are sized with it. */
int bih_camera_ray_bound(const bih_camera *camera, float dmax[3]);

/* Scene ingestion (host only, no device): a Wavefront OBJ file flattened to a
 * triangle soup in file order, replacing Model::LoadModel's assimp import
 * (src/Model.cpp:10-95, aiProcess_Triangulate) and the mesh -> triangle walk
 * of App::LoadModels (src/App.cpp:65-121).  On success out->v is allocated by
 * the library (free it with bih_scene_free); on BIH_ERR_PARSE *err_line (may
 * be NULL) holds the 1-based offending line. */
int bih_scene_load_obj(const char *path, bih_scene *out, uint32_t *err_line);
void bih_scene_free(bih_scene *scene);

/* Build from a host soup (copied H2D) or a device-resident soup. */
int bih_build(const bih_scene *scene, int device, bih_tree **out);
int bih_build_device(const float *d_v, uint32_t n_tris, int device, void *stream,
                     bih_tree **out);
/* Rebuild in place (per-frame rebuild as in Renderer::Render).  Renders issued
 * afterwards on any stream see the new tree.  When the soup cannot have
 * changed (BIH_PARAM_STATIC_SOUP) the call does not wait for the device; else
 * it returns after the build, with BIH_ERR_NONFINITE for a non-finite soup. */
int bih_rebuild(bih_tree *tree);
void bih_free(bih_tree *tree);

int bih_tree_get_info(const bih_tree *tree, bih_tree_info *info);
/* Copies one canonical array to host memory; *bytes in/out. */
int bih_tree_export(const bih_tree *tree, int which, void *host_dst, size_t *bytes);

/* Full frame into a host framebuffer (reference render() entry point). */
int bih_render(const bih_scene *scene, const bih_tree *tree, const bih_camera *camera,
               bih_framebuffer *fb);
/* Rows [row0, row0+nrows) into fb->rgba[(y-row0)*w + x]; RNG subsequence and
 * jitter use the GLOBAL pixel index, so tiles reassemble the full frame. */
int bih_render_rows(const bih_scene *scene, const bih_tree *tree, const bih_camera *camera,
                    bih_framebuffer *fb, uint32_t row0, uint32_t nrows);

/* Device-resident render (bench / multi-GPU): writes nrows*w pixels to d_out
 * (device memory on the tree's device) in local row order, on `stream`
 * (NULL = the tree's stream), asynchronously; bih_sync waits for it.
 * traverse = BIH_TRAVERSE_*.  d_ray_stats (optional, device u32[3*rays], ray =
 * (local pixel)*spp + sample) gets per-ray {node visits, leaf visits, triangle
 * tests} for parity checks against the oracle. */
int bih_render_device(const bih_tree *tree, const bih_camera *camera, uint32_t w, uint32_t h,
                      uint32_t spp, uint32_t frame, uint64_t seed, const bih_rows *rows,
                      uint32_t traverse, uint32_t *d_out, uint32_t *d_ray_stats, void *stream);
/* nframes consecutive frames (frame0 .. frame0+nframes-1, any-hit) in one
 * call: frame j's nrows*w pixels at d_out + j*out_stride (out_stride >=
 * nrows*w pixels; 1 <= nframes <= 64).  Each frame is exactly the frame
 * bih_render_device renders at that index; through the frustum bins the
 * frames share one launch of each kernel (the host issue cost and the
 * render's drain are paid once per call -- DESIGN.md section 5), otherwise
 * they are rendered one by one. */
int bih_render_device_frames(const bih_tree *tree, const bih_camera *camera, uint32_t w, uint32_t h,
                             uint32_t spp, uint32_t frame0, uint32_t nframes, uint64_t seed,
                             const bih_rows *rows, uint32_t *d_out, uint64_t out_stride, void *stream);
int bih_sync(const bih_tree *tree, void *stream);

/* Sizes, ahead of time, every per-call device buffer that renders of this
 * shape need (w x h image, spp, rows = NULL for the whole frame, calls of up to
 * max_frames frames through bih_render_device_frames): the XORWOW ring, the
 * per-slot tile-queue state, fallback records and frame-split start states.
 * After it (and after one render with each camera) a frame loop of that shape
 * allocates nothing (bih_tree_info.device_allocs stays put).  The reference
 * allocates these once in Renderer::CreateCUDABuffers (src/Renderer.cpp:
 * 762-797); here they also depend on the call shape, hence the explicit call.
 * Renders of a larger shape still grow the buffers on demand. */
int bih_reserve(bih_tree *tree, uint32_t w, uint32_t h, uint32_t spp, const bih_rows *rows,
                uint32_t max_frames);

/* Per-tree parameters.  None changes a pixel; they only reorder work or
 * force the exact-walk fallback, for A/B runs and tests.  Defaults are read
 * once per process from the environment variable of the same name
 * (BIH_ITEM_TILES, ...), never on the render path. */
#define BIH_PARAM_ITEM_TILES      1  /* tile count below which a multi-frame
                                        launch splits an item's frames (65536);
                                        unset, the render kernel splits by the
                                        launch's live tiles (~16384 items)     */
#define BIH_PARAM_PAIR_CAP        2  /* (triangle, tile) pair-result slots of
                                        the bins build (tests: 0 = recompute)  */
#define BIH_PARAM_BINS_CAP        3  /* cap on bin list entries (tests: force
                                        the overflow path; 0 = none)           */
#define BIH_PARAM_FORCE_FALLBACK  4  /* 1: every live packet of a frustum-bin
                                        render takes the exact walk (tests)    */
#define BIH_PARAM_WHITTED_COUNTERS 5 /* 1: Whitted renders count the nodes and
                                        triangles each bounce's walks visit
                                        (bih_whitted_work; costs time)         */
#define BIH_PARAM_STATIC_SOUP     6  /* 1: the caller does not change the device
                                        soup of a bih_build_device tree between
                                        builds, so bih_rebuild need not read the
                                        new tree's header back: it returns once
                                        the build is enqueued (renders order
                                        after it on the device).  Implied for
                                        bih_build trees (the tree owns its copy) */
#define BIH_PARAM_TEST_ALLOC_FAIL 7  /* tests, one-shot: the next build that
                                        allocates its buffers fails at its k-th
                                        allocation (1..64; BIH_ERR_OOM); the tree
                                        frees what it had allocated and stays
                                        usable (0 = off)                       */
int bih_tree_set_param(bih_tree *tree, int param, uint64_t value);

/* Config C4 (BASELINE.json configs[3]): 8 bounces of mirror (Whitted)
 * reflection per primary ray.  The reference has primary rays only
 * (Color, src/CUDAKernels.cu:370-389), so these semantics are this
 * library's own, stated in DESIGN.md section 4.5 and restated by the oracle
 * (ob_render_whitted): closest hit = min (t, sorted index) over the triangles
 * a front-to-back walk tests -- the reference walk's decisions and order
 * (TraverseTree, :227-368) until the first hit, after which a stacked node
 * entered beyond the best hit (tMin > best) is popped unvisited and tMax is
 * clamped to the best hit; a bounce's walk interval starts at max(scene-box
 * entry, 1e-4) (its origin lies inside the box: nothing behind it can be
 * accepted); P = O + tD, n = cross(e1, e2), R = D - (2 D.n / n.n) n;
 * secondary hits need t > 1e-4; a sample's shade halves towards (255,255,0)
 * per hit and ends at (20,20,40) on a miss (or (255,255,0) after 8 bounces).
 * Same primary rays, RNG draws and framebuffer format as bih_render.
 * d_hits (optional, device u32[rays]): hits along each sample's mirror path
 * (0..9), ray = local pixel * spp + sample. */
#define BIH_WHITTED_BOUNCES 8
int bih_render_whitted_device(const bih_tree *tree, const bih_camera *camera, uint32_t w, uint32_t h,
                              uint32_t spp, uint32_t frame, uint64_t seed, const bih_rows *rows,
                              uint32_t *d_out, uint32_t *d_hits, void *stream);
int bih_render_whitted(const bih_scene *scene, const bih_tree *tree, const bih_camera *camera,
                       bih_framebuffer *fb);
/* Work of the last Whitted render, which must have run with
 * BIH_PARAM_WHITTED_COUNTERS on (else BIH_ERR_INVALID): per bounce d = 0..8
 * the rays traced, the BIH nodes their walks entered and the triangles they
 * tested (the closest-hit walk of section 4.5; no counts for a one-leaf
 * tree, whose walks have no nodes).  Waits for that render. */
int bih_whitted_work(const bih_tree *tree, uint32_t rays[BIH_WHITTED_BOUNCES + 1],
                     uint64_t nodes[BIH_WHITTED_BOUNCES + 1], uint64_t tris[BIH_WHITTED_BOUNCES + 1]);

/* The drop-in host loop (bih_render into a caller's framebuffer) ends in a
 * device-to-host copy of w*h*4 bytes.  Into pageable memory the runtime
 * stages it; page-locking the framebuffer once lets the copy run at DMA rate
 * (the reference copies device-to-device into its GL buffer instead,
 * src/Renderer.cpp:645-655).  Optional: any host buffer works without it.
 * bih_host_unregister undoes it (before the buffer is freed). */
int bih_host_register(void *ptr, size_t bytes);
int bih_host_unregister(void *ptr);

/* Per-render device timing (HIP events on the render stream around the main
 * render kernel and at the end of the render's device work), off by default:
 * the events cost host time on every render call.  bih_last_render_ms gives
 * the main kernel's device time (ms) of the last render, which must have been
 * issued with timing on (else BIH_ERR_INVALID). */
int bih_set_timing(bih_tree *tree, int on);
int bih_last_render_ms(const bih_tree *tree, double *ms);
/* The same render split in two: *kernel_ms as bih_last_render_ms (the main
 * render kernel, the figure rocprofv3 reports for it) and *tail_ms from its
 * end to the end of the render call's device work (k_render_fallback, the
 * exact walk of packets the frustum-bin kernel left undecided). */
int bih_last_render_times(const bih_tree *tree, double *kernel_ms, double *tail_ms);
/* The last n renders (1 <= n <= 3; all issued with timing on), oldest first:
 * t[3*i .. 3*i+2] = {main kernel start, main kernel end, end of the render's
 * device work} in ms after the oldest one's kernel start.  Renders of a frame
 * loop in flight on several streams overlap: the union of their kernel
 * intervals is the loop's kernel time (bench.py's roofline). */
int bih_render_history(const bih_tree *tree, uint32_t n, double *t);

/* The frustum bins of the tree's current camera and image (any-hit renders):
 * usable = 1 when renders walk them; list entries over all tiles, entries of
 * the global list, tiles (TW x TH pixels, one 64-ray packet each). */
typedef struct bih_bins_stats {
    uint32_t usable;
    uint32_t tiles_x, tiles_y;
    uint64_t list_entries;
    uint32_t global_entries;
} bih_bins_stats;
int bih_bins_get_stats(const bih_tree *tree, bih_bins_stats *out);

#ifdef __cplusplus
}
#endif
#endif /* BIH_H */
