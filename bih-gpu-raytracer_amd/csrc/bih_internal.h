// bih_internal.h -- shared host/device definitions of libbih_amd (gfx950).
//
// HBM layout of one built tree (all buffers hipMalloc'd on the tree's device):
//
//   tris_s   f32[9N]    triangles in Morton-sorted order, rewritten as
//                        {v0, e1 = v1-v0, e2 = v2-v0} (36 B; MT's first two
//                        subtractions, CUDAKernels.cu:18-19, done once at build)
//   nodes    u32x4[U-1] render node (16 B): {clip0, clip1, z, w}
//                        z = split | axis<<27 | leafL<<29 | leafR<<30
//                        w = mid | cntL<<27 | cntR<<29, mid = firstIdx[split+1]
//                        left child  = internal node `split` or leaf tris
//                                      [mid - cntL, mid); right child = node
//                                      `split+1` or leaf tris [mid, mid + cntR);
//                        cnt code 0 = escape, read dup_cnt[leaf] (count > 3)
//   canonical arrays (reference names, GPUArrayManager.h:46-55) kept for the
//   builder and for bih_tree_export: morton/tri_idx (sorted), unique_mc,
//   dup_cnt, first_idx, leaf_parent, clip, axis, children, is_leaf, parent.
//   rng      u32[5][P]  XORWOW v[0..4] per pixel, plane-major (the Weyl counter
//                        d is identical for every pixel, so it is not stored).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stddef.h>

#define BIH_HOST_DEVICE __host__ __device__

namespace bih {

constexpr uint32_t kIdxBits = 27;
constexpr uint32_t kIdxMask = (1u << kIdxBits) - 1u;
constexpr int kStackDepth = 32;   // Karras path length <= 30 for distinct 30-bit codes
#ifndef BIH_LDS_STACK
#define BIH_LDS_STACK 10
#endif
// stack entries per lane held in LDS (12 B each); deeper ones spill to HBM.
// 1M-tri soup @1080p: 0.8 % of pushes land in slot >= 10 (12 % at >= 8).
constexpr int kLdsStack = BIH_LDS_STACK;
// work buffer: [0..8) chunk counters (one per image band / XCD); [16..56) walk
// counters of counter builds; [64..64+32*1024) per-CU tile slots (u64, one per
// 128-byte line: no false sharing of the slot atomics between CUs)
constexpr uint32_t kSlotStrideWords = 32;
constexpr uint32_t kWorkWords = 64 + kSlotStrideWords * 1024 + 64;   // + histograms (counter builds)
constexpr uint32_t kHistWord = 64 + kSlotStrideWords * 1024;
constexpr uint32_t kBinGlobalMax = 4096;          // longer global lists: no bins (the shortcut walk)
constexpr uint32_t kBinEntryF4 = 3;               // list entry: 3 x float4 = 48 bytes (bih_bins.hip)
constexpr uint32_t kBinsUnusable = 0xFFFFFFFFu;   // bins status: lists not built (k_bin_status)
constexpr uint32_t kBinSetWords = (16 + 1024) * 32;   // k_render_bins queue state per set
#ifndef BIH_BUCKETS
#define BIH_BUCKETS 6
#endif
constexpr uint32_t kBinBuckets = BIH_BUCKETS;     // list-order buckets per tile (bih_bins.hip)
#ifndef BIH_BLOCK_TILES
#define BIH_BLOCK_TILES 512
#endif
constexpr uint32_t kBinBlockTiles = BIH_BLOCK_TILES;   // tile rectangle of a bins block counted in LDS
#ifndef BIH_PACKET_COUNTERS
#define BIH_PACKET_COUNTERS 0
#endif

// Device-resident header written by the builder.
struct TreeHeader {
    float scene_lo[3];
    float scene_hi[3];
    uint32_t n_tris;
    uint32_t n_unique;
    uint32_t nonfinite;
    uint32_t pad0;
    unsigned long long lo_key[3];   // argmin keys (App.cpp:133-137 tie rules)
    unsigned long long hi_key[3];   // argmax keys
    unsigned long long content;     // hash of the input soup (k_prep, folded in k_morton): the tree is a function of it
};

// Render parameters, passed by value.
struct RenderArgs {
    float cam[12];          // origin, lower_left, horizontal, vertical
    uint32_t w, h, spp;
    uint32_t row0, nrows, band_h, band_step;
    uint32_t d_base;        // XORWOW Weyl counter at the start of this frame
    uint32_t hdr_n_tris;    // host copy of hdr->n_tris (kernel choice)
    uint32_t n_nodes = 0;   // host copy of U-1, the internal nodes (kernel choice)
    const TreeHeader *hdr;
    const uint4 *nodes;
    const float *tris;
    const float *tri_prim;  // 16 f32 per triangle: primary-ray records for origin cam[0..2]
    const uint4 *node_prim; // per node {clip0 - O[axis], clip1 - O[axis], z, w} for the same origin
    const uint4 *node_cull; // node_prim with leaves no primary ray can hit cut off (k_node_prim)
    const uint32_t *dup_cnt;
    const uint32_t *rng_in; // 5 planes of nrows*w: XORWOW v at the start of the frame (read only)
    uint32_t *pixacc;       // per-pixel {hits<<16 | samples} of the refill kernel (kept 0)
    uint32_t *out;          // nrows*w pixels
    uint32_t *ray_stats;    // optional 3 u32 per ray {nodes, leaves, tris}
    uint32_t *work;         // tile counter of the persistent kernel (zeroed per launch)
    uint32_t *spill;        // per-lane stack spill area (spill_words(grid) u32)
    const uint32_t *chunk_order = nullptr;  // packet kernel: chunk permutation (launch_chunk_order)
    uint32_t *chunk_cost = nullptr;         // packet kernel: per-chunk cycle accumulator (zeroed)
    const float *fast = nullptr;            // any-hit shortcut boxes (k_fast_fit); null: exact walk only
    const float *fast2 = nullptr;           // miss-proof boxes (miss_box); null: no miss proof
    // frustum bins (bih_bins.hip) of this camera and image: per TW x TH tile
    // of the full image the triangles whose footprint touches it
    // (bin_list[bin_off[b] .. bin_off[b+1])), and the global list
    // (bin_glist[0 .. *bin_gstat)); null: no bins (rows not tile-aligned)
    const uint32_t *bin_off = nullptr;
    const float *bin_list = nullptr;        // 48-byte entries (bih_bins.hip)
    const float *bin_glist = nullptr;       // global list entries
    const float *bin_rec = nullptr;         // per triangle the 64-byte record (k_bin_fp): plan values at 12..15
    const uint2 *bin_path = nullptr;        // [U][32] root path steps per leaf
    uint32_t bins_x = 0;
    const uint32_t *bin_gstat = nullptr;    // bins status: global list length or kBinsUnusable
    // the launch's tile queue (launch_bin_queue) and this render slot's queue
    // state (kBinSetWords, zero at launch: band heads, fallback count, per-CU
    // slots), plus the other set, which this launch zeroes for the slot's next one
    const uint32_t *bin_queue = nullptr;
    // (a queue ordered by measured cost) each band's first heavy tiles --
    // their count follows the band headers -- are taken as `hsplit` items
    // each, over frame ranges (the other live tiles: nsplit); hsplit ==
    // nsplit: no heavy items
    uint32_t hsplit = 1;
    uint32_t *bin_cost = nullptr;           // non-null: k_render_bins records each live tile's cycles per frame
    const uint32_t *bin_qhdr = nullptr;
    uint32_t *bin_heads = nullptr;
    uint32_t *bin_heads_next = nullptr;
    uint32_t *bin_fb = nullptr;             // fallback records of the slot (k_render_bins), 8 words each
    uint32_t dbg = 0;                       // timing experiments only (BIH_DBG): 1 skip background, 2 skip live
    // k_render_bins / k_render_fallback: frames d_base's frame .. + nframes - 1
    // in one launch (bih_render_device_frames); frame j's pixels at
    // out + j * out_stride, its XORWOW draws 2*spp*j past rng_in's
    uint32_t nframes = 1;
    uint32_t shared_grid = 0;   // 1: another render is in flight: a multi-frame k_render_bins leaves it room
    uint64_t out_stride = 0;
    // k_render_bins: frames per queue item (an item covers its tile in
    // frames [s*fpi, min((s+1)*fpi, nframes)) of the launch, s = 0 ..
    // nsplit-1); few tiles per launch (a rank's bands) take fewer frames per
    // item so that the items still outnumber the waves
    uint32_t fpi = 1;
    uint32_t nsplit = 1;
    // (non-zero) k_render_bins chooses the split itself from the queue's live
    // tile count: about live_items items per launch (fpi / nsplit above
    // only serve without it); bit 31: heavy tiles split further (hsplit)
    uint32_t live_items = 0;
    // k_render_bins: queue rounds each wave takes without atomics (BinQueue)
    uint32_t static_rounds = 1;
    // one-frame k_render_bins (config C4's primary rays): per local tile the
    // 64-bit mask of its samples that hit (lane = pixel * spp + sample), 0 for
    // background tiles; k_render_fallback writes the undecided packets'
    unsigned long long *hit_mask = nullptr;
    // Stamped XORWOW state (bih_capi.cpp, round 5): per local tile of the
    // launch rows a u64 stamp {cur frame:26 | cur buffer:1, prev frame:26 |
    // prev buffer:1, seq:10}; the tile's pixels' state at frame F sits in
    // st_buf[b] (5 planes of nrows*w).  A launch reads each live tile's state
    // from its stamp (`prev` when this launch already rewrote the stamp: its
    // seq), steps it to the item's first frame, and the item that ends at the
    // launch's last frame writes the state after it into the other buffer and
    // the new stamp.  Background tiles (no triangle can be hit) are not
    // touched: their states catch up when they turn live (k_rng_sync bounds
    // the gap).  null: rng_in (the k_rng_advance ring).
    unsigned long long *stamps = nullptr;
    uint32_t *st_buf0 = nullptr, *st_buf1 = nullptr;
    // k_render_bins' hit cache across launches: per local tile 64 lanes'
    // last hit triangles (hcache) and a stamp (hstamp) -- valid while it
    // equals hseq, the camera set's queue sequence number (bih_capi.cpp); null:
    // the cache lives within an item only
    uint32_t *hcache = nullptr;
    uint32_t *hstamp = nullptr;
    uint32_t hseq = 0;
    uint32_t st_f0 = 0;     // the launch's first frame
    uint32_t st_seq = 0;    // this launch's sequence number (1 .. 1023)
};

// stamp word (RenderArgs::stamps)
constexpr uint32_t kStampFrameBits = 26;
constexpr uint32_t kStampFrameMax = (1u << kStampFrameBits) - 1u;

// Camera of the frustum bins (bih_bins.hip), f64: forward normal n (A.n > 0,
// A = lower_left - O), and the (u, v) of a camera-relative point X:
// u = (X.hu) an / (X.n) - ahu, v = (X.vv) an / (X.n) - avv.
struct BinCamera {
    double n[3], hu[3], vv[3];
    double A[3], hh[3], vert[3], delta[3];   // A = lower_left - O, h, vert, |f32 D - D| bound
    double nlen, an, ahu, avv;
    double dn_lb;                             // <= D.n of every f32 primary ray (det_lower_bound)
    float dmax[3];
    float o[3];                               // origin (f32, as the kernels hold it)
    uint32_t w, h, tw, th;
};
// Device buffers of the frustum bins.
struct BinBuffers {
    uint32_t bins_x = 0, bins_y = 0;
    uint2 *brect = nullptr;       // [n] bin rectangle per triangle
    uint32_t *cnt = nullptr;      // [nb] entries per tile (k_bin_count); cntq and cur follow (zeroed together)
    uint32_t *cntq = nullptr;     // [nb][kBinBuckets - 1] entries per tile in the buckets but the last
    uint32_t *cur = nullptr;      // [nb][kBinBuckets] the fill's cursors per tile and bucket
    uint32_t *blkcnt = nullptr;   // [blocks][kBinBlockTiles] u64: k_bin_count's per-block (tile, bucket) counts
    uint32_t *off = nullptr;      // [nb + 1] list offsets, off[nb] = list length
    uint32_t *gcount = nullptr;   // [8] global list length, status (k_bin_status), list total, alive count,
                                  // 64-bit list total, pair-result cursor
    uint32_t *live = nullptr;     // [n] alive triangles (k_live_compact)
    uint32_t *bmask = nullptr;    // [blocks][4] u64 alive masks of k_cam_tris' blocks
    uint32_t *bcnt = nullptr;     // [blocks] their counts
    uint32_t *boff = nullptr;     // [blocks + 1] the counts' exclusive scan
    uint32_t *bpart = nullptr;    // its scan scratch
    uint32_t *glist = nullptr;    // [n] global list (triangles)
    uint32_t *partials = nullptr; // scan scratch
    float *binrec = nullptr;      // [n][16] list entry of each triangle
    uint2 *path = nullptr;        // [U][32] root path steps per leaf
    uint32_t *pres = nullptr;     // [pres_cap] per (triangle, tile) pair: k_bin_count's class / pixel mask / bucket
    uint32_t pres_cap = 0;
    uint32_t *pbase = nullptr;    // [blocks] each count block's base in pres (~0: none)
    uint32_t *cost = nullptr;     // [nb] cycles per frame of each live tile's packet, written by
                                  // k_render_bins launches that measure (RenderArgs::bin_cost)
};

// Device buffers of one tree.
struct DeviceTree {
    int device = 0;
    uint32_t n = 0, u = 0;
    uint64_t content = 0;          // TreeHeader::content of the last build
    uint32_t gen = 0;              // the tree generation this buffer holds (bih_capi.cpp)
    size_t bytes = 0;
    uint64_t allocs = 0;           // hipMalloc calls made for this tree (bih_tree_info.device_allocs)
    float *v = nullptr;            // input soup f32[9N] (device copy)
    bool owns_v = false;
    TreeHeader *hdr = nullptr;
    float *tri_lo = nullptr, *tri_hi = nullptr;     // f32[3N]
    uint32_t *keys = nullptr, *vals = nullptr;      // sorted morton / tri idx
    uint32_t *keys2 = nullptr, *vals2 = nullptr;    // sort ping-pong
    uint32_t *scan_tmp = nullptr;                   // scan scratch; after the build the leaf of
                                                    // each sorted triangle (k_run_compact)
    uint32_t *flags = nullptr;                      // (unused since round 4: k_runs)
    uint32_t *unique_mc = nullptr, *dup_cnt = nullptr;
    int32_t *first_idx = nullptr, *leaf_parent = nullptr;
    float *clip = nullptr;
    int32_t *axis = nullptr, *children = nullptr, *parent = nullptr;
    uint8_t *is_leaf = nullptr;
    int2 *fit_rng = nullptr;                        // [U-1] leaf range of each node (k_karras)
    float *fit_seg = nullptr;                       // [6][seg_capacity] leaf-box segment tree (k_fit)
    uint4 *nodes = nullptr;
    float *tris_s = nullptr;
    uint32_t *hist = nullptr;                       // radix histograms
    uint32_t *partials = nullptr;
    unsigned long long *prep_part = nullptr;        // k_prep per-block AABB keys
    TreeHeader *hdr_host = nullptr;                 // pinned host copy of hdr (k_fit writes it)
    hipEvent_t ev0 = nullptr, ev1 = nullptr;        // build timing (build_ms)
    hipGraphExec_t graph = nullptr;                 // the build's kernels for graph_n triangles of graph_v
    uint32_t graph_n = 0;
    const float *graph_v = nullptr;
    uint32_t fail_alloc = 0;                        // tests (BIH_PARAM_TEST_ALLOC_FAIL): the k-th
                                                    // buffer allocation of the next build fails
};

// builder (bih_build.hip); returns hipError_t as int
// sync = false: returns once the kernels are enqueued (no header read back;
// t.u / t.content keep their values, ms_out is not written)
int build_tree_device(DeviceTree &t, void *stream, float *ms_out, bool sync = true);
void free_tree_device(DeviceTree &t);

// render (bih_render.hip)
int upload_rng_tables(int device);
long bins_timeline_dump(const char *path);         // diagnostic builds (BIH_BINS_TIMELINE)
// stamped XORWOW state (RenderArgs::stamps): every tile's stamp = frame F in
// buffer 0; and k_rng_sync: every pixel's state brought to frame T -- into
// its tile's other buffer with a new stamp (seq), or (full != null) into
// `full` for every pixel (leaving the stamped state)
int launch_stamp_init(unsigned long long *stamps, uint32_t ntiles, uint32_t frame, void *stream);
int launch_rng_sync(unsigned long long *stamps, uint32_t *buf0, uint32_t *buf1, uint32_t *full, uint32_t w,
                    uint32_t nrows, uint32_t spp, uint32_t target, uint32_t seq, int device, void *stream);
const uint32_t *rng_tables_device(int device);      // xorwow_init_tables_host() on the device
// config C4 (bih_whitted.hip): device bytes of the ray queues for `rays`
// samples, and the frame's launches (k_wh_gen, 9 x k_wh_trace, k_wh_shade);
// ev_k0/ev_k1 bracket the trace launches.  d_hits (optional): u32 hit count
// per sample.
size_t whitted_bytes(uint64_t rays);
int launch_whitted(const RenderArgs &a, void *mem, uint64_t rays, uint32_t *d_hits, void *stream, void *ev_k0,
                   void *ev_k1, bool count, const unsigned long long *hit_mask = nullptr, uint32_t tiles_x = 0);
int whitted_work(const void *mem, uint64_t rays, uint32_t ray_counts[9], unsigned long long work[18], void *stream);
int launch_rng_init(uint32_t *rng, uint32_t w, uint32_t row0, uint32_t nrows, uint32_t band_h,
                    uint32_t band_step, uint64_t seed, uint64_t skip, int device, void *stream);
// dst = src's per-pixel state advanced by `steps` draws (planes of `pixels`; dst may be src)
int launch_rng_advance(const uint32_t *src, uint32_t *dst, uint64_t pixels, uint32_t steps, int device,
                       void *stream);
// ev_k0 / ev_k1 (hipEvent_t or null): recorded right before and after the
// main render kernel (bih_last_render_ms)
int launch_render(const RenderArgs &a, uint32_t traverse, void *stream, void *ev_k0 = nullptr,
                  void *ev_k1 = nullptr);
uint32_t wave_grid_blocks(int device);     // persistent grid of the render kernels
size_t spill_words(uint32_t blocks);
// chunks of the packet kernel's tile queue for a w x nrows launch (0: no packet kernel)
uint32_t chunk_count(uint32_t w, uint32_t nrows, uint32_t spp, uint32_t *chunks_x);
// order[] = the chunks of every band by descending cost[] (k_chunk_order)
int launch_chunk_order(const uint32_t *cost, uint32_t chunks_x, uint32_t nchunks, uint32_t *order,
                       void *stream);
// primary-ray records for camera origin `origin`: n triangle records
// (16 f32, k_tri_prim), then m = U-1 node records (u32x4, k_node_prim) + 1
// pad, then the same m + 1 records with unhittable subtrees cut off, then
// per-leaf and per-node alive bytes, then the any-hit walk's two shortcut
// box sets (m + 1 records of 16 x 32 bit each, k_fast_fit / k_fast_refs:
// tight, then miss-proof for |D| <= dmax per component; launch_fast_boxes)
// and m arrival counters
size_t prim_bytes(uint32_t n, uint32_t m);
size_t fast_offset(uint32_t n, uint32_t m);   // byte offset of the shortcut boxes
int launch_prim(const float *tris, uint32_t n, const uint4 *nodes, const int32_t *first_idx,
                const uint32_t *dup_cnt, const int32_t *leaf_parent, const int32_t *parent,
                uint32_t m, const float origin[3], const float dmax[3], float *prim,
                void *stream);
// node_cull (the second set of node records above) and the alive bytes
int launch_prim_cull(uint32_t n, const uint4 *nodes, const int32_t *first_idx, const uint32_t *dup_cnt,
                     uint32_t m, const float origin[3], float *prim, void *stream);
int launch_fast_boxes(const float *tris, uint32_t n, const uint4 *nodes, const int32_t *first_idx,
                      const uint32_t *dup_cnt, const int32_t *leaf_parent, const int32_t *parent,
                      uint32_t m, const float origin[3], const float dmax[3], float *prim, void *stream);
bool render_uses_prim(uint32_t spp);

// frustum bins (bih_bins.hip): camera setup (false: degenerate camera, no
// bins); then the camera's primary-ray records (launch_prim's triangle and
// node records), the alive list, footprints, per-tile counts and offsets
bool bin_camera(const float cam[12], const float dmax[3], uint32_t w, uint32_t h, uint32_t tw,
                uint32_t th, BinCamera *out);
int launch_bin_footprints(const float *tris, uint32_t n, const uint4 *nodes, uint32_t m, const float origin[3],
                          float *prim, const TreeHeader *hdr, const uint32_t *tri_leaf,
                          const int32_t *leaf_parent, const int32_t *parent, const BinCamera &c,
                          const BinBuffers &b, void *stream);
// lists of 48-byte entries (list: per-tile, gent: the global list's)
// the status word gcount[1] (k_bin_status: the global list length, or
// kBinsUnusable when the lists exceed `cap` entries or the global list
// kBinGlobalMax) and gcount[2] = the list total; the fill and the render read it
int launch_bin_status(const BinBuffers &b, size_t cap, void *stream);
int launch_bin_fill(uint32_t n, const BinCamera &c, const BinBuffers &b, float *list, float *gent,
                    void *stream);
// the render kernel's work queue over one launch's tiles (k_queue_*), in 8
// bands of tile rows: per band the live tiles by descending list length,
// then the background tiles; qhdr (device) = per band {start, live,
// background, items}.  mem: bin_queue_bytes(ntiles)
// cost (optional): per bin the measured cycles per frame of its packet
// (RenderArgs::bin_cost); with it the live tiles go in LPT order of their
// measured cost (finer classes than the list length) and each band's tiles
// costing over kHeavyFactor x the launch's mean come first and are counted in
// *qheavy (k_render_bins splits them over frame ranges: RenderArgs::hsplit).
size_t bin_queue_bytes(uint32_t ntiles);
int launch_bin_queue(const uint32_t *off, const uint32_t *gstat, uint32_t bins_x, uint32_t tiles_x, uint32_t ntiles,
                     uint32_t row0, uint32_t band_h, uint32_t band_step, uint32_t th, void *mem,
                     uint32_t **queue, uint32_t **qhdr, void *stream, const uint32_t *cost = nullptr,
                     uint32_t **qheavy = nullptr);
// exclusive scan of n u32 (bih_build.hip); *total_dev = the sum
int scan_exclusive(const uint32_t *in, uint32_t *out, uint32_t n, uint32_t *partials,
                   uint32_t *total_dev, void *stream);
size_t scan_partials_words(uint32_t n);
uint32_t next_scan_tag();   // tag of a dev::lookback_prefix call (bih_device.h)

// host XORWOW helpers (xorwow_host.cpp)
void xorwow_seed(uint64_t seed, uint32_t v[5], uint32_t *d);
const uint32_t *xorwow_tables_host();   // [32 seq][160][5] ++ [64 step][160][5]
// v = M^skip v (skip draws ahead, host)
void xorwow_skip(uint32_t v[5], uint64_t skip);
// k_rng_init's device tables: jump bytes [4][256][160][5] ++ J, J^64 by nibbles [2][40][16][5]
constexpr size_t kRngNibWords = 40 * 16 * 5;      // one nibble table (bih_render.hip jump_lds)
// ++ nibble tables of M^(2^(7+l)), l = 0..6: kStampJumpFrames frames of 2 * 2^l draws
// (k_rng_sync, one per spp = 2^l)
constexpr uint32_t kStampJumpFrames = 64;
constexpr size_t kRngJumpOffset = (size_t)4 * 256 * 800 + 2 * kRngNibWords;
constexpr size_t kRngInitWords = kRngJumpOffset + 7 * kRngNibWords;
const uint32_t *xorwow_init_tables_host();

}  // namespace bih
