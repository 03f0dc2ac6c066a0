// bih_capi.cpp -- the C ABI of include/bih.h over the HIP builder/renderer.
//
// Mirrors the reference's host seam: GPUArrayManager owns the scene/BIH
// buffers (src/GPUArrayManager.h:46-55), Renderer owns the framebuffer and the
// per-pixel curandState (src/Renderer.cpp:762-797).  Here a bih_tree owns
// both, per device, and errors are returned instead of exit(99)
// (src/Renderer.cpp:63-73).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <mutex>
#include <new>
#include <algorithm>
#include <cmath>
#include <vector>

#include "../../include/bih.h"
#include "bih_internal.h"

#ifndef BIH_DEBUG_KNOBS
#define BIH_DEBUG_KNOBS 0   // 1: honour BIH_DBG (timing experiments; changes pixels)
#endif

// Up to kSlots renders through one tree may be in flight together (issued
// on as many streams): each launch takes one of kSlots {tile queue, spill
// area, events} in turn, and reads its frame's XORWOW state from a ring of
// kSlots + 1 buffers that k_rng_advance fills one frame ahead.
#ifndef BIH_RENDER_SLOTS
#define BIH_RENDER_SLOTS 3
#endif
constexpr int kSlots = BIH_RENDER_SLOTS;
constexpr int kRngBufs = kSlots + 1;
#ifndef BIH_SHARE_ONE_FRAME
#define BIH_SHARE_ONE_FRAME 1
#endif
// one-frame renders also take the shared grid while another render is in flight
constexpr bool kShareOneFrame = BIH_SHARE_ONE_FRAME != 0;
constexpr size_t kEntryBytes = 16 * bih::kBinEntryF4;   // frustum-bin list entry

// Per-camera structures (bih_render.hip / bih_bins.hip): primary-ray records,
// frustum bins and the tile queue of one camera.  A tree keeps kCamSets of
// them: a camera change builds into a set the latest render does not read,
// after only the renders that read that set -- so camera k+1's structures
// build while frame k renders (a moving camera, bench `moving_camera`).
#ifndef BIH_CAM_SETS
#define BIH_CAM_SETS 3
#endif
constexpr int kCamSets = BIH_CAM_SETS;
// sets in use (BIH_CAM_SETS=1..kCamSets in the environment: A/B)
static int cam_sets() {
    static const int n = [] {
        const char *e = getenv("BIH_CAM_SETS");
        const int v = e ? atoi(e) : kCamSets;
        return v < 1 ? 1 : (v > kCamSets ? kCamSets : v);
    }();
    return n;
}
struct CamSet {
    float *prim = nullptr;           // primary-ray triangle + node records (bih::prim_bytes)
    size_t prim_cap = 0;             // bytes
    bool prim_valid = false;
    bool fast_valid = false;         // the BIH walk's shortcut boxes match the records
    bool cull_valid = false;         // node_cull matches the records (launch_prim_cull)
    uint32_t prim_origin[12] = {0};        // bit patterns of the camera they were built for
    // frustum bins (bih_bins.hip) of the camera the records were built for,
    // for one image size and tile shape (bins_key = {w, h, spp})
    char *bins_mem = nullptr;        // brect, cnt, off, gcount, glist, partials, binrec, path, gent
    size_t bins_mem_cap = 0;         // bytes
    float *bin_list = nullptr;       // 48-byte entries (bih::kBinEntryF4 float4)
    size_t bin_list_cap = 0;         // entries
    bih::BinBuffers bins;
    bool bins_valid = false;         // built for prim_origin and bins_key
    bool bins_usable = false;        // built and within the limits (else the kernel skips them)
    uint32_t bins_key[3] = {0, 0, 0};
    float *bin_gent = nullptr;       // global list entries (in bins_mem)
    uint32_t bin_gn = 0;             // global list length (host copy once resolved)
    // bins built without a host round trip (build_bins): the device status
    // word decides the render; the host learns the totals from bins_host once
    // ev_bins has passed (resolve_bins) and regrows the list if it overflowed
    bool bins_pending = false;
    bool bins_regrow = false;        // the last lists overflowed: rebuild with a sized list
    bool bins_redo = false;          // the current lists are unusable but still read by renders
    uint32_t *bins_host = nullptr;   // pinned: {gcount, status, total}
    uint64_t bin_entries = 0;        // list entries over all tiles
    uint32_t gen = 0;                // bih_tree::bins_gen of this set's last bins build
    size_t bins_layout = 0;          // tiles of the bins_mem layout whose scan words are zeroed
    // the render kernel's tile queue over one launch's rows (launch_bin_queue),
    // for q_key = {w, h, spp, row0, nrows, band_h, band_step, gen}
    char *q_mem = nullptr;
    size_t q_cap = 0;
    bool q_valid = false;
    uint32_t q_key[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    uint32_t *q_list = nullptr, *q_hdr = nullptr;
    bool q_cost = false;             // the queue is ordered by measured tile costs (launch_bin_queue's cost)
    // k_render_bins' hit cache across launches (RenderArgs::hcache): hc_tiles x
    // 64 lanes' last hit triangles, then hc_tiles stamps (zeroed when
    // allocated); valid for a tile while its stamp equals hseq, which changes
    // whenever the queue's key (image, rows, bins generation) does
    uint32_t *hc = nullptr;
    size_t hc_tiles = 0;
    uint32_t hseq = 0;
    uint32_t uses = 0;               // frustum-bin renders since these bins were built
    // the last launch that measured tile costs (bins.cost) was over q_key ==
    // cost_key: the next queue of those rows is built from them
    bool cost_known = false;
    uint32_t cost_key[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    uint32_t cost_pending[8] = {0, 0, 0, 0, 0, 0, 0, 0};   // q_key of a measuring launch being prepared
    hipEvent_t ev_bins = nullptr;    // after the readback of the last bins build's {gcount, status, total}
};

// Per-tree parameters (bih_tree_set_param).  None changes a pixel.  Their
// defaults come from the environment, read once per process (A/B scripts),
// never on the render path.
struct TreeParams {
    uint32_t item_tiles = 65536u;     // BIH_PARAM_ITEM_TILES
    bool item_tiles_set = false;      // (set: item_split's rule decides, not the live count)
    uint32_t pair_cap = 0xFFFFFFFFu;  // BIH_PARAM_PAIR_CAP (~0: sized from N)
    uint64_t bins_cap = 0;            // BIH_PARAM_BINS_CAP (0: no cap)
    uint32_t force_fallback = 0;      // BIH_PARAM_FORCE_FALLBACK
    uint32_t wh_counters = 0;         // BIH_PARAM_WHITTED_COUNTERS
    uint32_t static_soup = 0;         // BIH_PARAM_STATIC_SOUP
    uint32_t test_alloc_fail = 0;     // BIH_PARAM_TEST_ALLOC_FAIL (one-shot)
};
static const TreeParams &env_params() {
    static const TreeParams p = [] {
        TreeParams q;
        if (const char *v = getenv("BIH_ITEM_TILES")) {
            q.item_tiles = (uint32_t)strtoul(v, nullptr, 10);
            q.item_tiles_set = true;
        }
        if (const char *v = getenv("BIH_PAIR_CAP")) q.pair_cap = (uint32_t)strtoul(v, nullptr, 10);
        if (const char *v = getenv("BIH_BINS_CAP")) q.bins_cap = (uint64_t)strtoull(v, nullptr, 10);
        if (const char *v = getenv("BIH_BINS_FORCE_FALLBACK")) q.force_fallback = v[0] == '1';
        return q;
    }();
    return p;
}
#if BIH_DEBUG_KNOBS
static uint32_t dbg_bits() {
    static const uint32_t d = [] {
        const char *v = getenv("BIH_DBG");
        return v ? (uint32_t)atoi(v) & ~4u : 0u;
    }();
    return d;
}
#endif

struct bih_tree {
    bih::DeviceTree t;
    // Rebuilds write the oldest of three tree buffers and rotate (back[0] =
    // the previous generation, back[1] = the one before): renders of the
    // trees still in flight keep reading theirs while the next one is built,
    // and two asynchronous rebuilds can run at once (pipelined frames: frame
    // k+1's build beside frame k's, on the other build stream).  gen counts
    // rotations; DeviceTree::gen is the generation a buffer holds and
    // slot_gen[k] the one render slot k read, so a rebuild waits only for the
    // renders that read its target buffer.
    bih::DeviceTree back[2];
    uint32_t gen = 0;
    hipStream_t bstream = nullptr;   // the second build stream (asynchronous rebuilds alternate)
    uint32_t bpar = 0;               // asynchronous rebuilds so far (stream parity)
    uint32_t slot_gen[kSlots] = {};
    hipStream_t slot_stream[kSlots] = {};   // the stream render slot k was issued on
    TreeParams prm = env_params();
    uint64_t allocs = 0;             // hipMalloc calls of the render side (+ t.allocs: the builder's)
    hipStream_t stream = nullptr;
    // ev0/ev1: the render kernel's start and end (bih_last_render_ms); evd:
    // everything the render issued is done (ordering of slot reuse, rebuilds)
    hipEvent_t ev0[kSlots] = {}, ev1[kSlots] = {}, evd[kSlots] = {};
    hipEvent_t ev2[kSlots] = {};     // end of the render's device work (timed renders only)
    bool used[kSlots] = {};
    bool timing = false;             // bih_set_timing: record ev0/ev1/ev2 around each render
    bool last_timed = false;
    bool slot_timed[kSlots] = {};    // the slot's last render recorded ev0/ev1/ev2
    bool built = false;              // a build completed (t.content is its soup's hash)
    int slot = 0;                    // slot of the next render
    int last_slot = -1;              // slot of the last render
    // After the last write to state every render reads, whichever stream
    // issued it: the advance that produced rng buffer rng_cur, the per-camera
    // records (prim) and the tree itself (a build or rebuild).  Every render
    // waits on it, so a render on another stream never reads half-written
    // records.
    hipEvent_t ev_rng = nullptr;
    bool rng_pending = false;
    // after the last (re)build of the tree: the per-camera builds order after
    // it (and after the renders that read their set), not after each other
    hipEvent_t ev_tree = nullptr;
    bool tree_pending = false;
    mutable double build_ms = 0.0;
    // an asynchronous rebuild's device time: read from its events on demand
    // (bih_tree_get_info), not by the rebuild
    mutable bool build_ms_pending = false;
    bool owns_soup = false;          // bih_build: the soup is the tree's own copy (never changes)
    const float *host_v = nullptr;   // scene the tree was built from (identity check)
    // render state cache (Renderer::d_rand_state / CreateCUDABuffers)
    mutable std::mutex mu;
    uint32_t *rng = nullptr;         // [kRngBufs][5][cap] XORWOW planes + [kSlots][cap] accumulators
    size_t rng_cap = 0;              // pixels
    int rng_cur = 0;                 // which XORWOW buffer holds the next frame's input
    uint32_t *fb = nullptr;
    size_t fb_cap = 0;               // pixels
    bool rng_valid = false;
    uint32_t key_w = 0, key_spp = 0, key_row0 = 0, key_nrows = 0, key_bh = 0, key_bs = 0;
    uint64_t key_seed = 0;
    uint32_t next_frame = 0;
    // stamped XORWOW state (RenderArgs::stamps): frustum-bin launches on one
    // stream read and write per-tile state in ring buffers st_a and st_a + 1,
    // no k_rng_advance; any other consumer leaves the mode (prepare_rng)
    unsigned long long *stamps = nullptr;
    size_t stamp_cap = 0;            // tiles
    bool stamped = false;
    int st_a = 0;
    uint32_t st_seq = 0;             // the last launch's sequence number (1 .. 1023)
    uint32_t st_sync = 0;            // frame of the last k_rng_sync / k_stamp_init
    uint32_t stream_run = 0;         // renders in a row on the last render's stream
    bool owns_stream = false;
    uint32_t *work = nullptr;        // persistent-kernel tile counters, kWorkWords per slot
    uint32_t *spill = nullptr;       // traversal stack spill area, spill_words per slot
    size_t spill_per_slot = 0;       // u32
    // cost-ordered tile queue: per slot {cost, order} of chunk_cap u32 each;
    // the cost a render accumulates orders the next render of the same slot
    uint32_t *chunk_buf = nullptr;
    size_t chunk_cap = 0;
    uint32_t chunk_key[kSlots][6] = {};
    // per-camera structures: kCamSets sets, so that the structures of a new
    // camera are built while renders of the previous one still read theirs
    CamSet cs[kCamSets];
    int cs_cur = 0;                  // set of the latest render's camera
    int slot_cs[kSlots] = {};        // set the slot's last render read
    uint32_t bins_gen = 0;           // incremented by every bins build (any set)
    uint32_t hseq_ctr = 0;           // the camera sets' hit-cache sequence numbers (CamSet::hseq), never 0
    // per render slot two sets of 8 band heads (32 words apart): a launch
    // draws from set q_par[slot] and zeroes the other for the slot's next launch
    uint32_t *q_count = nullptr;
    uint32_t q_par[kSlots] = {};
    uint32_t *fb_mem = nullptr;      // per slot: fallback records of k_render_bins (8 words per tile)
    size_t fbq_cap = 0;              // tiles per slot
    // config C4 (bih_whitted.hip): two ray queues, counters and per-sample hits
    char *wh_mem = nullptr;
    size_t wh_rays = 0;              // queue capacity (rays)
    uint64_t wh_last_rays = 0;       // rays of the last Whitted render (its buffer layout)
    int wh_last_slot = -1;           // its slot (evd), when it ran with work counters
    int wh_prev_slot = -1;           // the last Whitted launch's slot (its evd orders the next mask render)
    unsigned long long *wh_mask = nullptr;   // primary samples' hit masks per tile (bounce 0 through the bins)
    size_t wh_mask_cap = 0;                  // tiles
};

namespace {

// Every device allocation of a tree goes through here (bih_tree_info.device_allocs).
template <class T>
hipError_t tree_malloc(bih_tree *tr, T **p, size_t bytes) {
    const hipError_t e = hipMalloc((void **)p, bytes);
    if (e == hipSuccess) ++tr->allocs;
    return e;
}

// Makes `dev` current for the call and restores the caller's device after
// it; no hipSetDevice when it already is (the per-call host path).
struct DeviceGuard {
    int prev = -1;
    bool changed = false;
    explicit DeviceGuard(int dev) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        if (prev != dev) changed = hipSetDevice(dev) == hipSuccess;
    }
    ~DeviceGuard() {
        if (changed && prev >= 0) (void)hipSetDevice(prev);
    }
};

int map_hip(int e) {
    if (e == 0) return BIH_OK;
    if (e == -1000) return BIH_ERR_NONFINITE;
    if (e == (int)hipErrorOutOfMemory || e == (int)hipErrorMemoryAllocation) return BIH_ERR_OOM;
    if (e == (int)hipErrorInvalidDevice || e == (int)hipErrorNoDevice) return BIH_ERR_NO_DEVICE;
    return BIH_ERR_HIP;
}

int check_device(int device) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return BIH_ERR_NO_DEVICE;
    if (device < 0 || device >= n) return BIH_ERR_NO_DEVICE;
    return BIH_OK;
}

// Orders `st` after every render in flight through this tree.
int wait_renders(bih_tree *tr, hipStream_t st) {
    for (int k = 0; k < kSlots; ++k)
        if (tr->used[k]) {
            hipError_t e = hipStreamWaitEvent(st, tr->evd[k], 0);
            if (e != hipSuccess) return map_hip((int)e);
        }
    return BIH_OK;
}

// Orders `st` after every render in flight that read camera set `c`.
int wait_set_readers(bih_tree *tr, int c, hipStream_t st) {
    for (int k = 0; k < kSlots; ++k)
        if (tr->used[k] && tr->slot_cs[k] == c) {
            hipError_t e = hipStreamWaitEvent(st, tr->evd[k], 0);
            if (e != hipSuccess) return map_hip((int)e);
        }
    return BIH_OK;
}

// Cost-ordered tile queue of the packet kernel (bih::launch_chunk_order):
// the chunks of this render start in descending order of the cycles their
// longest packet
// took in the last render of the same slot and geometry (frame f - kSlots in
// a frame sequence), so the slow part of the image starts first and the frame
// does not end on one long packet.  The order never changes a pixel.
// Called after `st` waits for the slot's previous render.  BIH_CHUNK_ORDER=0
// turns it off (tuning / A-B).
// The any-hit walk's shortcut passes (k_render_packet_asm, bih_render.hip):
// 2 = hit shortcut + miss proof (default), BIH_FAST=1 the hit shortcut only,
// BIH_FAST=0 neither (A-B).  They never change a pixel.
int fast_enabled() {
    static const int level = [] {
        const char *e = getenv("BIH_FAST");
        if (e && strcmp(e, "0") == 0) return 0;
        if (e && strcmp(e, "1") == 0) return 1;
        return 2;
    }();
    return level;
}

int prepare_chunk_order(bih_tree *tr, uint32_t w, uint32_t spp, const bih_rows &rows, int slot,
                        hipStream_t st, bih::RenderArgs &a) {
    static const bool enabled = [] {
        const char *e = getenv("BIH_CHUNK_ORDER");
        return !(e && strcmp(e, "0") == 0);
    }();
    a.chunk_order = nullptr;
    a.chunk_cost = nullptr;
    uint32_t cx = 0;
    const uint32_t n = bih::chunk_count(w, rows.nrows, spp, &cx);
    if (!enabled || n == 0) return BIH_OK;
    if (tr->chunk_cap < n) {
        // every render that may still use the old buffers has finished
        for (int k = 0; k < kSlots; ++k)
            if (tr->used[k]) (void)hipEventSynchronize(tr->evd[k]);
        if (tr->chunk_buf) (void)hipFree(tr->chunk_buf);
        tr->chunk_buf = nullptr;
        tr->chunk_cap = 0;
        hipError_t e = tree_malloc(tr, &tr->chunk_buf, (size_t)kSlots * 2 * n * sizeof(uint32_t));
        if (e != hipSuccess) return map_hip((int)e);
        tr->chunk_cap = n;
        memset(tr->chunk_key, 0, sizeof tr->chunk_key);
    }
    uint32_t *cost = tr->chunk_buf + (size_t)slot * 2 * tr->chunk_cap;
    uint32_t *order = cost + tr->chunk_cap;
    const uint32_t key[6] = {w, spp, rows.row0, rows.nrows, rows.band_h, rows.band_step};
    hipError_t e = hipSuccess;
    if (memcmp(key, tr->chunk_key[slot], sizeof key) != 0) {
        e = hipMemsetAsync(cost, 0, n * sizeof(uint32_t), st);   // no history: identity order
        if (e != hipSuccess) return map_hip((int)e);
        memcpy(tr->chunk_key[slot], key, sizeof key);
    }
    int le = bih::launch_chunk_order(cost, cx, n, order, st);
    if (le) return map_hip(le);
    e = hipMemsetAsync(cost, 0, n * sizeof(uint32_t), st);
    if (e != hipSuccess) return map_hip((int)e);
    a.chunk_order = order;
    a.chunk_cost = cost;
    return BIH_OK;
}

// Orders `st` after every render in flight that read generation g (the
// buffer a rebuild is about to overwrite), and after that buffer's own last
// build (it may have run on the other build stream).
int wait_tree_buffer(bih_tree *tr, const bih::DeviceTree &b, hipStream_t st) {
    if (!b.hdr) return BIH_OK;   // never built: no reader
    for (int k = 0; k < kSlots; ++k)
        if (tr->used[k] && tr->slot_gen[k] == b.gen && hipEventQuery(tr->evd[k]) != hipSuccess) {
            hipError_t e = hipStreamWaitEvent(st, tr->evd[k], 0);
            if (e != hipSuccess) return map_hip((int)e);
        }
    if (b.ev1 && hipEventQuery(b.ev1) != hipSuccess) {
        hipError_t e = hipStreamWaitEvent(st, b.ev1, 0);
        if (e != hipSuccess) return map_hip((int)e);
    }
    return BIH_OK;
}

int finish_build(bih_tree *tr) {
    float ms = 0.f;
    bool async = false;
    const bool had = tr->built;
    const uint64_t old_content = tr->t.content;
    const uint32_t old_n = tr->t.n, old_u = tr->t.u;
    int e = 0;
    hipStream_t bst = tr->stream;   // the stream the build runs on (ev_tree follows it)
    // tests: the next build that allocates its buffers fails part-way
    auto arm_fail = [&](bih::DeviceTree &d) {
        if (tr->prm.test_alloc_fail && !d.hdr) {
            d.fail_alloc = tr->prm.test_alloc_fail;
            tr->prm.test_alloc_fail = 0;
        }
    };
    if (!had) {
        // first build (or after a failed one): in place, after every render
        // launched through this tree (it may run on another stream)
        int rc = wait_renders(tr, tr->stream);
        if (rc) return rc;
        arm_fail(tr->t);
        e = bih::build_tree_device(tr->t, tr->stream, &ms);
    } else {
        // rebuild into the oldest buffer (allocated by its first build): only
        // the renders that read it are waited for; the renders of the newer
        // trees run on beside the build
        bih::DeviceTree &b = tr->back[1];
        // a soup that cannot have changed since the last build (the tree's own
        // copy, or BIH_PARAM_STATIC_SOUP) gives the same tree, header and
        // content hash bit for bit: nothing to read back, so the host does not
        // wait for the build -- it runs behind the renders in flight, and the
        // next render orders after it (ev_tree).  Consecutive asynchronous
        // rebuilds alternate between the tree's stream and a second build
        // stream, so frame k+1's build runs beside frame k's (each chain of
        // ~15 short kernels leaves most of the GPU idle); each render still
        // waits for its own frame's tree.  BIH_BUILD_PIPE=0: one stream (A/B).
        async = tr->owns_soup || tr->prm.static_soup;
        static const bool pipe = [] {
            const char *v = getenv("BIH_BUILD_PIPE");
            return !(v && v[0] == '0');
        }();
        if (async && pipe && (tr->bpar++ & 1u)) {
            if (!tr->bstream && hipStreamCreateWithFlags(&tr->bstream, hipStreamNonBlocking) != hipSuccess) {
                (void)hipGetLastError();
                tr->bstream = nullptr;
            }
            if (tr->bstream) bst = tr->bstream;
        }
        int rc = wait_tree_buffer(tr, b, bst);
        if (rc) return rc;
        if (!b.owns_v) b.v = tr->t.v;   // the same soup (the owning copy is one buffer's)
        b.n = tr->t.n;
        b.device = tr->t.device;
        if (async) {
            b.u = tr->t.u;
            b.content = tr->t.content;
        }
        arm_fail(b);
        e = bih::build_tree_device(b, bst, &ms, !async);
        if (e == 0 || e == -1000) {
            // rotate: the new tree becomes current, the current the previous
            std::swap(tr->back[1], tr->back[0]);   // back[1] = previous-previous, back[0] = the new one
            std::swap(tr->back[0], tr->t);         // t = the new one, back[0] = previous
            tr->t.gen = ++tr->gen;
        }
    }
    tr->build_ms = ms;
    tr->build_ms_pending = async && e == 0;
    tr->built = e == 0;
    // the per-pixel RNG state does not depend on the geometry: a rebuild (the
    // reference rebuilds every frame) keeps the frame sequence going.  The
    // per-camera structures (triangle and node records, shortcut boxes,
    // frustum bins, tile queues) are functions of the tree, and the tree of
    // the soup: a rebuild of an unchanged soup (same content hash, N and U;
    // the tree is bit-identical) keeps them
    const bool same = had && e == 0 && tr->t.content == old_content && tr->t.n == old_n && tr->t.u == old_u;
    if (!same)
        for (CamSet &c : tr->cs) {
            c.prim_valid = false;  // triangle records follow the (re)sorted triangles
            c.bins_valid = false;
        }
    if (e) return map_hip(e);
    // renders issued on other streams order after the (re)build (every
    // render and camera build waits on ev_tree).  A first build waited for
    // every render, so it also follows the last advance of the XORWOW ring;
    // a rebuild did not, and leaves ev_rng to the renders
    hipError_t he = hipEventRecord(tr->ev_tree, bst);
    if (he == hipSuccess && !had) he = hipEventRecord(tr->ev_rng, tr->stream);
    if (he != hipSuccess) return map_hip((int)he);
    if (!had) tr->rng_pending = true;
    tr->tree_pending = true;
    return BIH_OK;
}

int create_tree(int device, void *stream, bih_tree **out) {
    bih_tree *tr = new (std::nothrow) bih_tree();
    if (!tr) return BIH_ERR_OOM;
    tr->t.device = device;
    hipError_t e = hipSuccess;
    if (stream) {
        tr->stream = (hipStream_t)stream;
    } else {
        e = hipStreamCreateWithFlags(&tr->stream, hipStreamNonBlocking);
        tr->owns_stream = (e == hipSuccess);
    }
    for (int k = 0; k < kSlots && e == hipSuccess; ++k) {
        e = hipEventCreate(&tr->ev0[k]);
        if (e == hipSuccess) e = hipEventCreate(&tr->ev1[k]);
        if (e == hipSuccess) e = hipEventCreateWithFlags(&tr->evd[k], hipEventDisableTiming);
        if (e == hipSuccess) e = hipEventCreate(&tr->ev2[k]);
    }
    if (e == hipSuccess) e = hipEventCreateWithFlags(&tr->ev_rng, hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&tr->ev_tree, hipEventDisableTiming);
    for (CamSet &c : tr->cs) {
        if (e == hipSuccess) e = hipEventCreateWithFlags(&c.ev_bins, hipEventDisableTiming);
        if (e == hipSuccess) e = hipHostMalloc((void **)&c.bins_host, 4 * sizeof(uint32_t), hipHostMallocDefault);
    }
    if (e == hipSuccess && bih::upload_rng_tables(device) != 0) e = hipErrorUnknown;
    if (e != hipSuccess) {
        delete tr;
        return map_hip((int)e);
    }
    *out = tr;
    return BIH_OK;
}

}  // namespace

extern "C" {

int bih_abi_version(void) { return BIH_ABI_VERSION; }

int bih_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

const char *bih_strerror(int code) {
    switch (code) {
    case BIH_OK: return "ok";
    case BIH_ERR_INVALID: return "invalid argument";
    case BIH_ERR_NO_DEVICE: return "no HIP device (or invalid device index)";
    case BIH_ERR_HIP: return "HIP runtime error";
    case BIH_ERR_OOM: return "out of memory";
    case BIH_ERR_NONFINITE: return "scene holds a non-finite coordinate";
    case BIH_ERR_TOO_LARGE: return "too many triangles";
    case BIH_ERR_MISMATCH: return "scene does not match the tree";
    case BIH_ERR_IO: return "file could not be opened or read";
    case BIH_ERR_PARSE: return "malformed scene file";
    default: return "unknown error";
    }
}

// Camera(vec3(2,0,-2), (float)W/H): Renderer.cpp:99; members computed in
// double and rounded to f32 (Camera.cu:5-9).
int bih_camera_reference(uint32_t w, uint32_t h, bih_camera *out) {
    if (!out || w == 0 || h == 0) return BIH_ERR_INVALID;
    const float aspect = (float)w / (float)h;
    const float o[3] = {2.0f, 0.0f, -2.0f};
    for (int a = 0; a < 3; ++a) out->origin[a] = o[a];
    out->lower_left[0] = (float)((double)o[0] - 2.0);
    out->lower_left[1] = (float)((double)o[1] - 1.0);
    out->lower_left[2] = (float)((double)o[2] + 1.0);
    out->horizontal[0] = (float)((double)aspect * 2.0);
    out->horizontal[1] = 0.0f;
    out->horizontal[2] = 0.0f;
    out->vertical[0] = 0.0f;
    out->vertical[1] = 2.0f;
    out->vertical[2] = 0.0f;
    return BIH_OK;
}

int bih_camera_ray_bound(const bih_camera *cam, float dmax[3]) {
    if (!cam || !dmax) return BIH_ERR_INVALID;
    for (int c = 0; c < 3; ++c) {
        float mx = 0.0f;
        for (int k = 0; k < 4; ++k) {
            const float u = (float)(k & 1), v = (float)(k >> 1);
            const float d = ((cam->lower_left[c] + u * cam->horizontal[c]) + v * cam->vertical[c]) -
                            cam->origin[c];
            mx = std::max(mx, std::fabs(d));
        }
        const float mag = ((std::fabs(cam->lower_left[c]) + std::fabs(cam->horizontal[c])) +
                           std::fabs(cam->vertical[c])) + std::fabs(cam->origin[c]);
        dmax[c] = (mx * 1.001f + 1e-6f) + std::ldexp(mag, -21);
    }
    return BIH_OK;
}

int bih_build(const bih_scene *scene, int device, bih_tree **out) {
    if (!scene || !out || (scene->n_tris && !scene->v)) return BIH_ERR_INVALID;
    if (scene->n_tris > BIH_MAX_TRIS) return BIH_ERR_TOO_LARGE;
    int rc = check_device(device);
    if (rc) return rc;
    DeviceGuard g(device);
    bih_tree *tr = nullptr;
    rc = create_tree(device, nullptr, &tr);
    if (rc) return rc;
    tr->t.n = scene->n_tris;
    tr->host_v = scene->v;
    size_t bytes = (size_t)scene->n_tris * 36;
    hipError_t e = tree_malloc(tr, &tr->t.v, bytes ? bytes : 16);
    if (e == hipSuccess) {
        tr->t.owns_v = true;
        tr->owns_soup = true;
        tr->t.bytes += bytes;
        if (bytes) e = hipMemcpy(tr->t.v, scene->v, bytes, hipMemcpyHostToDevice);
    }
    if (e != hipSuccess) {
        bih_free(tr);
        return map_hip((int)e);
    }
    rc = finish_build(tr);
    if (rc) {
        bih_free(tr);
        return rc;
    }
    *out = tr;
    return BIH_OK;
}

int bih_build_device(const float *d_v, uint32_t n_tris, int device, void *stream, bih_tree **out) {
    if (!out || (n_tris && !d_v)) return BIH_ERR_INVALID;
    if (n_tris > BIH_MAX_TRIS) return BIH_ERR_TOO_LARGE;
    int rc = check_device(device);
    if (rc) return rc;
    DeviceGuard g(device);
    bih_tree *tr = nullptr;
    rc = create_tree(device, stream, &tr);
    if (rc) return rc;
    tr->t.n = n_tris;
    tr->t.v = const_cast<float *>(d_v);
    tr->t.owns_v = false;
    rc = finish_build(tr);
    if (rc) {
        bih_free(tr);
        return rc;
    }
    *out = tr;
    return BIH_OK;
}

int bih_rebuild(bih_tree *tr) {
    if (!tr) return BIH_ERR_INVALID;
    DeviceGuard g(tr->t.device);
    std::lock_guard<std::mutex> lk(tr->mu);
    return finish_build(tr);
}

void bih_free(bih_tree *tr) {
    if (!tr) return;
    DeviceGuard g(tr->t.device);
    if (tr->stream) (void)hipStreamSynchronize(tr->stream);
    for (int k = 0; k < kSlots; ++k)
        if (tr->used[k]) (void)hipEventSynchronize(tr->evd[k]);
    // a bins readback into bins_host may still be in flight (a failed render)
    for (CamSet &c : tr->cs)
        if (c.bins_pending) (void)hipEventSynchronize(c.ev_bins);
    if (tr->bstream) (void)hipStreamSynchronize(tr->bstream);
    bih::free_tree_device(tr->t);
    bih::free_tree_device(tr->back[0]);   // (the soup is freed by whichever buffer owns it)
    bih::free_tree_device(tr->back[1]);
    if (tr->bstream) (void)hipStreamDestroy(tr->bstream);
    if (tr->rng) (void)hipFree(tr->rng);
    if (tr->fb) (void)hipFree(tr->fb);
    if (tr->work) (void)hipFree(tr->work);
    if (tr->spill) (void)hipFree(tr->spill);
    if (tr->chunk_buf) (void)hipFree(tr->chunk_buf);
    for (CamSet &c : tr->cs) {
        if (c.prim) (void)hipFree(c.prim);
        if (c.bins_mem) (void)hipFree(c.bins_mem);
        if (c.bin_list) (void)hipFree(c.bin_list);
        if (c.q_mem) (void)hipFree(c.q_mem);
        if (c.hc) (void)hipFree(c.hc);
        if (c.ev_bins) (void)hipEventDestroy(c.ev_bins);
        if (c.bins_host) (void)hipHostFree(c.bins_host);
    }
    if (tr->q_count) (void)hipFree(tr->q_count);
    if (tr->fb_mem) (void)hipFree(tr->fb_mem);
    if (tr->stamps) (void)hipFree(tr->stamps);
    if (tr->wh_mem) (void)hipFree(tr->wh_mem);
    if (tr->wh_mask) (void)hipFree(tr->wh_mask);
    for (int k = 0; k < kSlots; ++k) {
        if (tr->ev0[k]) (void)hipEventDestroy(tr->ev0[k]);
        if (tr->evd[k]) (void)hipEventDestroy(tr->evd[k]);
        if (tr->ev1[k]) (void)hipEventDestroy(tr->ev1[k]);
        if (tr->ev2[k]) (void)hipEventDestroy(tr->ev2[k]);
    }
    if (tr->ev_rng) (void)hipEventDestroy(tr->ev_rng);
    if (tr->ev_tree) (void)hipEventDestroy(tr->ev_tree);
    if (tr->owns_stream) (void)hipStreamDestroy(tr->stream);
    delete tr;
}

// An asynchronous rebuild (BIH_PARAM_STATIC_SOUP) may still be running: the
// host-side readers of the tree (info, export) wait for it first, and take
// its device time from its events.
static int wait_async_build(const bih_tree *tr) {
    if (!tr->build_ms_pending) return BIH_OK;
    float ms = 0.f;
    hipError_t e = hipEventSynchronize(tr->t.ev1);
    if (e == hipSuccess) e = hipEventElapsedTime(&ms, tr->t.ev0, tr->t.ev1);
    if (e != hipSuccess) return map_hip((int)e);
    tr->build_ms = ms;
    tr->build_ms_pending = false;
    return BIH_OK;
}

int bih_tree_get_info(const bih_tree *tr, bih_tree_info *info) {
    if (!tr || !info) return BIH_ERR_INVALID;
    DeviceGuard g(tr->t.device);
    // a rebuild rotates the tree buffers under the same lock: never read a half-rotated tree
    std::lock_guard<std::mutex> lk(tr->mu);
    if (int rc = wait_async_build(tr)) return rc;
    bih::TreeHeader h;
    if (tr->t.hdr) {
        hipError_t e = hipMemcpy(&h, tr->t.hdr, sizeof h, hipMemcpyDeviceToHost);
        if (e != hipSuccess) return map_hip((int)e);
    } else {
        memset(&h, 0, sizeof h);
    }
    info->n_tris = tr->t.n;
    info->n_unique = tr->t.u;
    for (int a = 0; a < 3; ++a) {
        info->scene_lo[a] = h.scene_lo[a];
        info->scene_hi[a] = h.scene_hi[a];
    }
    info->device = tr->t.device;
    // tree + canonical arrays, the XORWOW ring (kRngBufs x 5 planes) and the
    // per-slot accumulators, the host-path framebuffer, the per-camera
    // records, and the per-slot tile queues, spill areas and chunk orders
    size_t cam = 0;
    for (const CamSet &c : tr->cs)
        cam += c.prim_cap + c.bins_mem_cap + c.bin_list_cap * kEntryBytes + c.q_cap + c.hc_tiles * 65 * 4;
    info->device_bytes = tr->t.bytes + tr->back[0].bytes + tr->back[1].bytes + (tr->rng_cap * (5 * kRngBufs + kSlots) + tr->fb_cap) * 4 + cam +
                         ((size_t)kSlots * (bih::kWorkWords + tr->spill_per_slot) +
                          (size_t)kSlots * 2 * tr->chunk_cap +
                          (tr->q_count ? (size_t)kSlots * 2 * bih::kBinSetWords : 0) +
                          (size_t)kSlots * tr->fbq_cap * 8) * 4 +
                         (tr->wh_mem ? bih::whitted_bytes(tr->wh_rays) : 0) + tr->wh_mask_cap * 8 + tr->stamp_cap * 8;
    info->build_ms = tr->build_ms;
    info->device_allocs = tr->allocs + tr->t.allocs + tr->back[0].allocs + tr->back[1].allocs;
    return BIH_OK;
}

int bih_tree_export(const bih_tree *tr, int which, void *dst, size_t *bytes) {
    if (!tr || !bytes) return BIH_ERR_INVALID;
    std::lock_guard<std::mutex> lk(tr->mu);   // (as bih_tree_get_info)
    const uint64_t N = tr->t.n, U = tr->t.u, M = U > 0 ? U - 1 : 0;
    const void *src = nullptr;
    size_t need = 0;
    switch (which) {
    case BIH_ARR_MORTON_SORTED: src = tr->t.keys; need = N * 4; break;
    case BIH_ARR_TRI_INDEX: src = tr->t.vals; need = N * 4; break;
    case BIH_ARR_UNIQUE_MC: src = tr->t.unique_mc; need = U * 4; break;
    case BIH_ARR_DUP_COUNT: src = tr->t.dup_cnt; need = U * 4; break;
    case BIH_ARR_FIRST_IDX: src = tr->t.first_idx; need = U * 4; break;
    case BIH_ARR_LEAF_PARENT: src = tr->t.leaf_parent; need = U * 4; break;
    case BIH_ARR_CLIP: src = tr->t.clip; need = M * 8; break;
    case BIH_ARR_AXIS: src = tr->t.axis; need = M * 4; break;
    case BIH_ARR_CHILDREN: src = tr->t.children; need = M * 8; break;
    case BIH_ARR_IS_LEAF: src = tr->t.is_leaf; need = M * 2; break;
    case BIH_ARR_PARENT: src = tr->t.parent; need = M * 4; break;
    case BIH_ARR_TRI_LO: src = tr->t.tri_lo; need = N * 12; break;
    case BIH_ARR_TRI_HI: src = tr->t.tri_hi; need = N * 12; break;
    default: return BIH_ERR_INVALID;
    }
    if (!dst) {
        *bytes = need;
        return BIH_OK;
    }
    if (*bytes < need) return BIH_ERR_INVALID;
    *bytes = need;
    if (need == 0) return BIH_OK;
    DeviceGuard g(tr->t.device);
    if (int rc = wait_async_build(tr)) return rc;
    hipError_t e = hipMemcpy(dst, src, need, hipMemcpyDeviceToHost);
    return map_hip((int)e);
}

static uint32_t *rng_buf(const bih_tree *tr, int k) {
    return tr->rng + (size_t)k * 5 * tr->rng_cap;
}

// Ensures the per-pixel RNG state for this framebuffer geometry sits at the
// start of `frame` in buffer rng_cur (InitRandGPU once, then cudaRender's
// 2*spp draws per frame; a short gap runs the generators forward, anything
// else re-seeds with a skip-ahead).  Runs on `st` after the renders that
// read rng_cur before (see bih_render_device).
// Waits for every render in flight through the tree (they may read a buffer
// that is about to be replaced).
static int drain_renders(bih_tree *tr) {
    for (int k = 0; k < kSlots; ++k)
        if (tr->used[k]) {
            hipError_t e = hipEventSynchronize(tr->evd[k]);
            if (e != hipSuccess) return map_hip((int)e);
        }
    return BIH_OK;
}

// The next render's stream waits for the state every render reads (ev_rng).
static hipError_t wait_rng(bih_tree *tr, hipStream_t st) {
    return tr->rng_pending ? hipStreamWaitEvent(st, tr->ev_rng, 0) : hipSuccess;
}

// The XORWOW ring (kRngBufs x 5 planes) and the per-slot accumulators for P
// pixels; a new ring holds no state (the next render seeds it).
static int ensure_rng(bih_tree *tr, size_t P, hipStream_t st) {
    if (P <= tr->rng_cap) return BIH_OK;
    int rc = drain_renders(tr);
    if (rc) return rc;
    if (tr->rng) (void)hipFree(tr->rng);
    tr->rng = nullptr;
    tr->rng_cap = 0;
    const size_t words = P * (5 * kRngBufs + kSlots);
    hipError_t e = tree_malloc(tr, &tr->rng, words * sizeof(uint32_t));
    if (e == hipSuccess) e = hipMemsetAsync(tr->rng + 5 * kRngBufs * P, 0, kSlots * P * sizeof(uint32_t), st);
    if (e != hipSuccess) return map_hip((int)e);
    tr->rng_cap = P;
    tr->rng_cur = 0;
    tr->rng_valid = false;
    tr->stamped = false;
    return BIH_OK;
}

// Stamped state (RenderArgs::stamps) unless BIH_STAMPED=0 (A/B); it never
// changes a pixel.
constexpr uint32_t kStampRun = 3;

static bool share_alternating() {
    static const bool on = [] {
        const char *e = getenv("BIH_SHARE_ALTERNATING");
        return !(e && strcmp(e, "0") == 0);
    }();
    return on;
}

// Items per multi-frame k_render_bins launch the kernel aims at from the
// queue's live tile count (RenderArgs::live_items; BIH_LIVE_ITEMS for A/B,
// 0: item_split's count of all tiles decides).  A/B (r06u, 16 frames per
// call): 1M soup at 1080p (24k live tiles) one item per tile either way;
// the 69k torus (7.3k live) 0.0255 -> 0.0221 ms per frame in items of 8
// frames; 30000 (items of 4) 0.0229
static uint32_t live_items_target() {
    static const uint32_t n = [] {
        const char *e = getenv("BIH_LIVE_ITEMS");
        return e ? (uint32_t)strtoul(e, nullptr, 10) : 16384u;
    }();
    return n;
}

// k_render_bins' static queue rounds in one-frame launches (BinQueue;
// BIH_STATIC_ROUNDS for A/B: one-frame calls 1 round 0.0824 ms, 2 0.0822,
// 3 0.086, 5 0.106 -- a wave cannot hand on its later static items, r05n)
static uint32_t static_rounds_one() {
    static const uint32_t n = [] {
        const char *e = getenv("BIH_STATIC_ROUNDS");
        const int v = e ? atoi(e) : -1;
        return v >= 0 && v <= 64 ? (uint32_t)v : 1u;
    }();
    return n;
}

// The render in `slot` was issued on `st` (before last_slot moves to it).
static void note_stream(bih_tree *tr, int slot, hipStream_t st) {
    const bool same = tr->last_slot >= 0 && tr->slot_stream[tr->last_slot] == st;
    tr->stream_run = same ? tr->stream_run + 1 : 1;
    tr->slot_stream[slot] = st;
}

static bool stamps_enabled() {
    static const bool on = [] {
        const char *e = getenv("BIH_STAMPED");
        return !(e && strcmp(e, "0") == 0);
    }();
    return on;
}

static int unstamp(bih_tree *tr, hipStream_t st);

// Grows the stamp array.  A stamped run in progress is first folded back into
// the ring (unstamp: every pixel's state at next_frame, rng_cur), so that the
// next render continues the sequence from the right state instead of the
// buffer stamped mode started from.
static int ensure_stamps(bih_tree *tr, size_t ntiles, hipStream_t st) {
    if (tr->stamp_cap >= ntiles) return BIH_OK;
    if (tr->stamped) {
        int rc = unstamp(tr, st);
        if (rc) return rc;
        const hipError_t e = hipStreamSynchronize(st);   // the sync kernel reads the stamps
        if (e != hipSuccess) return map_hip((int)e);
    }
    int rc = drain_renders(tr);
    if (rc) return rc;
    if (tr->stamps) (void)hipFree(tr->stamps);
    tr->stamps = nullptr;
    tr->stamp_cap = 0;
    tr->stamped = false;
    hipError_t e = tree_malloc(tr, &tr->stamps, ntiles * sizeof(unsigned long long));
    if (e != hipSuccess) return map_hip((int)e);
    tr->stamp_cap = ntiles;
    return BIH_OK;
}

static uint32_t next_stamp_seq(bih_tree *tr) {
    tr->st_seq = tr->st_seq % 1023u + 1u;
    return tr->st_seq;
}

// The persistent render kernels' work words and stack spill areas.
static int ensure_work(bih_tree *tr) {
    if (tr->work) return BIH_OK;
    tr->spill_per_slot = bih::spill_words(bih::wave_grid_blocks(tr->t.device));
    hipError_t e = tree_malloc(tr, &tr->work, kSlots * bih::kWorkWords * sizeof(uint32_t));
    if (e == hipSuccess) e = tree_malloc(tr, &tr->spill, kSlots * tr->spill_per_slot * sizeof(uint32_t));
    return map_hip((int)e);
}

// The frustum-bin kernel's queue state: per slot two sets, zero (each
// launch zeroes the other set for the slot's next launch).
static int ensure_qcount(bih_tree *tr) {
    if (tr->q_count) return BIH_OK;
    const size_t bytes = (size_t)kSlots * 2 * bih::kBinSetWords * sizeof(uint32_t);
    hipError_t e = tree_malloc(tr, &tr->q_count, bytes);
    if (e == hipSuccess) e = hipMemset(tr->q_count, 0, bytes);
    return map_hip((int)e);
}

// kSlots x `need` units of `unit` words (fallback records, split start
// states), grown after every render in flight.
static int ensure_per_slot(bih_tree *tr, uint32_t **buf, size_t *cap, size_t need, size_t unit) {
    if (*cap >= need) return BIH_OK;
    int rc = drain_renders(tr);
    if (rc) return rc;
    if (*buf) (void)hipFree(*buf);
    *buf = nullptr;
    *cap = 0;
    hipError_t e = tree_malloc(tr, buf, (size_t)kSlots * need * unit * sizeof(uint32_t));
    if (e != hipSuccess) return map_hip((int)e);
    *cap = need;
    return BIH_OK;
}

// Armed after prepare_rng: unless disarmed (the render was issued), the
// ring's state is dropped so that the next render re-seeds.
struct RngGuard {
    bih_tree *tr;
    bool armed = true;
    ~RngGuard() {
        if (armed) {
            tr->rng_valid = false;
            tr->stamped = false;
        }
    }
};

static bool rng_same_px(const bih_tree *tr, uint32_t w, uint32_t spp, uint64_t seed, const bih_rows &rows) {
    return tr->rng_valid && tr->key_w == w && tr->key_spp == spp && tr->key_seed == seed &&
           tr->key_row0 == rows.row0 && tr->key_nrows == rows.nrows && tr->key_bh == rows.band_h &&
           tr->key_bs == rows.band_step;
}

// Leaves stamped mode: every pixel's state at next_frame into a ring buffer
// of its own, which becomes rng_cur (after the stamped launches: they order
// ev_rng, which every render waits on first).
static int unstamp(bih_tree *tr, hipStream_t st) {
    if (!tr->stamped) return BIH_OK;
    tr->stamped = false;
    const int c = (tr->st_a + 2) % kRngBufs;
    tr->rng_cur = c;
    const int e = bih::launch_rng_sync(tr->stamps, rng_buf(tr, tr->st_a), rng_buf(tr, (tr->st_a + 1) % kRngBufs),
                                       rng_buf(tr, c), tr->key_w, tr->key_nrows, tr->key_spp, tr->next_frame,
                                       0xFFFFu, tr->t.device, st);
    if (e) tr->rng_valid = false;
    return map_hip(e);
}

static int prepare_rng(bih_tree *tr, uint32_t w, uint32_t spp, uint32_t frame, uint64_t seed,
                       const bih_rows &rows, hipStream_t st) {
    const size_t P = (size_t)rows.nrows * w;
    int rc = ensure_rng(tr, P, st);
    if (rc) return rc;
    bool same_px = rng_same_px(tr, w, spp, seed, rows);
    if (tr->stamped) {
        // the stamped state back into the ring, or dropped (re-seeded below)
        if (same_px && frame >= tr->next_frame) {
            rc = unstamp(tr, st);
            if (rc) return rc;
        } else {
            tr->stamped = false;
            tr->rng_cur = (tr->st_a + 2) % kRngBufs;
            tr->rng_valid = false;
            same_px = false;
        }
    }
    const bool same = same_px && tr->next_frame == frame;
    if (same_px && frame > tr->next_frame && (uint64_t)(frame - tr->next_frame) * 2 * spp <= 4096) {
        // a short gap in the frame sequence: run the generators forward
        // (cheaper than re-seeding with the 2^67-subsequence jump)
        const uint32_t steps = (frame - tr->next_frame) * 2 * spp;
        uint32_t *b = rng_buf(tr, tr->rng_cur);
        int e = bih::launch_rng_advance(b, b, P, steps, tr->t.device, st);
        if (e) return map_hip(e);
    } else if (!same) {
        uint64_t skip = (uint64_t)2 * spp * frame;
        int e = bih::launch_rng_init(rng_buf(tr, tr->rng_cur), w, rows.row0,
                                     rows.nrows, rows.band_h, rows.band_step,
                                     seed, skip, tr->t.device, st);
        if (e) return map_hip(e);
        tr->rng_valid = true;
        tr->key_w = w;
        tr->key_spp = spp;
        tr->key_seed = seed;
        tr->key_row0 = rows.row0;
        tr->key_nrows = rows.nrows;
        tr->key_bh = rows.band_h;
        tr->key_bs = rows.band_step;
    }
    tr->next_frame = frame + 1;
    return BIH_OK;
}

// k_render_bins' queue in LPT order of measured tile costs (prepare_bin_queue)
// unless BIH_COST_QUEUE=0 (A/B); it never changes a pixel.
static bool cost_queue_enabled() {
    static const bool on = [] {
        const char *e = getenv("BIH_COST_QUEUE");
        return !(e && strcmp(e, "0") == 0);
    }();
    return on;
}

// k_render_bins' hit cache across launches unless BIH_HIT_CACHE_XL=0 (A/B);
// it never changes a pixel.
static bool hit_cache_enabled() {
    static const bool on = [] {
        const char *e = getenv("BIH_HIT_CACHE_XL");
        return !(e && strcmp(e, "0") == 0);
    }();
    return on;
}

// Frustum bins are on unless BIH_BINS=0 (A-B); they never change a pixel.
static bool bins_enabled() {
    static const bool on = [] {
        const char *e = getenv("BIH_BINS");
        return !(e && strcmp(e, "0") == 0);
    }();
    return on;
}

// Packet tile of spp samples per pixel (TileShape in bih_render.hip).
static void tile_shape(uint32_t spp, uint32_t *tw, uint32_t *th) {
    const int L = __builtin_ctz(spp);
    const uint32_t lp = 6 - L;
    *tw = 1u << ((lp + 1) / 2);
    *th = 1u << (lp / 2);
}

// (Re)builds the frustum bins for `cam` and a w x h image on `st`, after the
// primary-ray records; every render that read the old ones has finished
// (the caller waited for them).  Synchronises `st` once to size the lists.
// Runs the camera's primary-ray records (launch_prim) when `need_prim` and
// the bins take no part.
static int prim_only(bih_tree *tr, CamSet &c, const bih_camera *cam, const float dmax[3], bool need_prim, hipStream_t st) {
    if (!need_prim) return BIH_OK;
    const uint32_t n_int = tr->t.u > 0 ? tr->t.u - 1 : 0;
    return map_hip(bih::launch_prim(tr->t.tris_s, tr->t.n, tr->t.nodes, tr->t.first_idx, tr->t.dup_cnt,
                                    tr->t.leaf_parent, tr->t.parent, n_int, cam->origin, dmax, c.prim, st));
}

// (Re)builds the frustum bins for `cam` and a w x h image on `st`; with
// `need_prim` also the camera's primary-ray records (k_cam_tris, or
// launch_prim when no bins are built).  Every render that read the old ones
// has finished (the caller waited for them).  Synchronises `st` once to size
// the lists the first time.
static int build_bins(bih_tree *tr, CamSet &c, const bih_camera *cam, const float dmax[3], uint32_t w,
                      uint32_t h, uint32_t spp, bool need_prim, hipStream_t st) {
    c.bins_valid = true;
    c.bins_usable = false;
    c.uses = 0;
    c.gen = ++tr->bins_gen;
    c.bins_key[0] = w;
    c.bins_key[1] = h;
    c.bins_key[2] = spp;
    const uint32_t n = tr->t.n, U = tr->t.u;
    uint32_t tw = 0, th = 0;
    tile_shape(spp, &tw, &th);
    bih::BinCamera bc;
    if (n == 0 || U < 2 || w > 0xffffu || h > 0xffffu ||
        !bih::bin_camera(reinterpret_cast<const float *>(cam), dmax, w, h, tw, th, &bc))
        return prim_only(tr, c, cam, dmax, need_prim, st);   // no bins: the kernel runs the shortcut passes instead
    bih::BinBuffers b;
    b.bins_x = (w + tw - 1) / tw;
    b.bins_y = (h + th - 1) / th;
    const size_t nb = (size_t)b.bins_x * b.bins_y;
    auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
    const uint32_t nblk = (n + 255) / 256;   // k_cam_tris blocks (bih::kThreads)
    // cnt, cntq and cur follow each other with no gap (k_cam_tris zeroes them as one range)
    const size_t s_brect = al((size_t)n * 8), s_cnt = nb * 4, s_cntq = nb * 4 * (bih::kBinBuckets - 1),
                 s_cur = al(nb * 4 * bih::kBinBuckets),
                 s_off = al((nb + 1) * 4),
                 s_g = al(8 * 4), s_glist = al((size_t)n * 4 + 4),
                 s_part = al(bih::scan_partials_words((uint32_t)nb) * 4),
                 // (the path table sized for U = N, its largest: a rebuilt tree of another soup
                 // of the same size fits the same layout, no allocation per changed soup)
                 s_rec = al((size_t)n * 64), s_path = al((size_t)n * 256),
                 s_gent = al((size_t)4097 * kEntryBytes), s_live = al((size_t)n * 4 + 4), s_bmask = al((size_t)nblk * 32),
                 s_bcnt = al((size_t)nblk * 4 + 4), s_boff = al((size_t)nblk * 4 + 8),
                 s_bpart = al(bih::scan_partials_words(nblk) * 4),
                 s_blkcnt = al((size_t)nblk * bih::kBinBlockTiles * 8),
                 s_pbase = al((size_t)nblk * 4), s_cost = al(nb * 4);
    // pair results (k_bin_count -> k_bin_fill): 4 B per (triangle, tile)
    // pair; blocks past the buffer recompute in the fill
    uint32_t pres_cap = (uint32_t)std::min<uint64_t>(4ull * n + (1u << 20), 0x3FFFFFFFull);
    pres_cap = std::min<uint32_t>(pres_cap, tr->prm.pair_cap);   // tests: blocks past a small buffer recompute
    const size_t s_pres = al((size_t)pres_cap * 4);
    const size_t need = s_brect + s_cnt + s_cntq + s_cur + s_off + s_g + s_glist + s_part + s_rec + s_path + s_gent +
                        s_live + s_bmask + s_bcnt + s_boff + s_bpart + s_blkcnt + s_pbase + s_pres + s_cost;
    if (c.bins_mem_cap < need) {
        hipError_t e = hipStreamSynchronize(st);   // renders that read the old bins
        if (e != hipSuccess) return map_hip((int)e);
        if (c.bins_mem) (void)hipFree(c.bins_mem);
        c.bins_mem = nullptr;
        c.bins_mem_cap = 0;
        e = tree_malloc(tr, &c.bins_mem, need);
        if (e != hipSuccess) return map_hip((int)e);
        c.bins_mem_cap = need;
        c.bins_layout = 0;
    }
    char *p = c.bins_mem;
    b.brect = reinterpret_cast<uint2 *>(p); p += s_brect;
    b.cnt = reinterpret_cast<uint32_t *>(p); p += s_cnt;
    b.cntq = reinterpret_cast<uint32_t *>(p); p += s_cntq;
    b.cur = reinterpret_cast<uint32_t *>(p); p += s_cur;
    b.off = reinterpret_cast<uint32_t *>(p); p += s_off;
    b.gcount = reinterpret_cast<uint32_t *>(p); p += s_g;
    b.glist = reinterpret_cast<uint32_t *>(p); p += s_glist;
    b.partials = reinterpret_cast<uint32_t *>(p); p += s_part;
    b.binrec = reinterpret_cast<float *>(p); p += s_rec;
    b.path = reinterpret_cast<uint2 *>(p); p += s_path;
    float *gent = reinterpret_cast<float *>(p); p += s_gent;
    b.live = reinterpret_cast<uint32_t *>(p); p += s_live;
    b.bmask = reinterpret_cast<uint32_t *>(p); p += s_bmask;
    b.bcnt = reinterpret_cast<uint32_t *>(p); p += s_bcnt;
    b.boff = reinterpret_cast<uint32_t *>(p); p += s_boff;
    b.bpart = reinterpret_cast<uint32_t *>(p); p += s_bpart;
    b.blkcnt = reinterpret_cast<uint32_t *>(p); p += s_blkcnt;
    b.pbase = reinterpret_cast<uint32_t *>(p); p += s_pbase;
    b.pres = reinterpret_cast<uint32_t *>(p); p += s_pres;
    b.pres_cap = pres_cap;
    b.cost = reinterpret_cast<uint32_t *>(p);
    c.cost_known = false;   // the tiles' measured costs belong to the previous bins
    // the scans' look-back words (partials, bpart) must start at tag 0 (never
    // a call's tag) wherever this layout puts them: stale data there must not
    // pass for a published prefix.  Later calls leave older, unique tags.
    if (c.bins_layout != nb) {
        hipError_t e = hipMemsetAsync(b.partials, 0, s_part, st);
        if (e == hipSuccess) e = hipMemsetAsync(b.bpart, 0, s_bpart, st);
        if (e != hipSuccess) return map_hip((int)e);
        c.bins_layout = nb;
    }
    // the triangle records are rewritten in any case (k_cam_tris computes the
    // alive list from them); the node records too
    int le = bih::launch_bin_footprints(tr->t.tris_s, n, tr->t.nodes, U - 1, cam->origin, c.prim, tr->t.hdr,
                                        tr->t.scan_tmp, tr->t.leaf_parent, tr->t.parent, bc, b, st);
    if (le) return map_hip(le);
    hipError_t e = hipSuccess;
    // A list buffer from an earlier camera: build into it without a host
    // round trip (k_bin_status tells the fill and the render whether the
    // lists fit; resolve_bins reads the totals later).  Otherwise size the
    // list from the counts (one synchronisation).  BIH_BINS_SYNC=1 always
    // synchronises (A/B); BIH_BINS_CAP caps the list (tests: overflow).
    static const bool always_sync = [] {
        const char *v = getenv("BIH_BINS_SYNC");
        return v && v[0] == '1';
    }();
    const size_t cap_test = (size_t)tr->prm.bins_cap;
    const bool speculative = c.bin_list_cap > 0 && !always_sync && !c.bins_regrow;
    if (speculative) {
        const size_t cap = cap_test ? std::min(cap_test, c.bin_list_cap) : c.bin_list_cap;
        le = bih::launch_bin_status(b, cap, st);
        if (le) return map_hip(le);
        e = hipMemcpyAsync(c.bins_host, b.gcount, 3 * sizeof(uint32_t), hipMemcpyDeviceToHost, st);
        if (e == hipSuccess) e = hipEventRecord(c.ev_bins, st);
        if (e != hipSuccess) return map_hip((int)e);
        c.bins_pending = true;
    } else {
        c.bins_pending = false;
        uint32_t g[6] = {0, 0, 0, 0, 0, 0};   // gcount words; [4..5] = 64-bit list total
        e = hipMemcpyAsync(g, b.gcount, sizeof g, hipMemcpyDeviceToHost, st);
        if (e == hipSuccess) e = hipStreamSynchronize(st);
        if (e != hipSuccess) return map_hip((int)e);
        c.bins_regrow = false;
        const uint64_t total = (uint64_t)g[4] | ((uint64_t)g[5] << 32);
        // every packet tests the whole global list: beyond a few thousand
        // triangles the shortcut passes are the better proof
        if (g[0] > bih::kBinGlobalMax) return BIH_OK;
        // lists past the u32 offsets or half the free device memory: no bins
        // for this camera (the BIH walk with its shortcut passes renders it)
        size_t mem_free = 0, mem_total = 0;
        if (hipMemGetInfo(&mem_free, &mem_total) != hipSuccess) mem_free = 0;
        const uint64_t cap = total + total / 8 + 1024;
        if (cap > 0xFFFFFFFFull || cap * kEntryBytes > (uint64_t)mem_free / 2 + (uint64_t)c.bin_list_cap * kEntryBytes)
            return BIH_OK;
        if (c.bin_list_cap < total + 1) {
            if (c.bin_list) (void)hipFree(c.bin_list);   // st waited for every render
            c.bin_list = nullptr;
            c.bin_list_cap = 0;
            e = tree_malloc(tr, &c.bin_list, cap * kEntryBytes);
            if (e != hipSuccess) {
                (void)hipGetLastError();   // not sticky: this camera renders without bins
                c.bin_list = nullptr;
                return BIH_OK;
            }
            c.bin_list_cap = cap;
        }
        le = bih::launch_bin_status(b, c.bin_list_cap, st);
        if (le) return map_hip(le);
        c.bin_gn = g[0];
        c.bin_entries = total;
    }
    le = bih::launch_bin_fill(n, bc, b, c.bin_list, gent, st);
    if (le) return map_hip(le);
    c.bins = b;
    c.bin_gent = gent;
    c.bins_usable = true;
    return BIH_OK;
}

// The totals of a bins build made without a host round trip, once its
// readback has landed (`block`: wait for it).  A global list past
// kBinGlobalMax turns the bins off for this camera (the shortcut walk); lists
// past the buffer make the next render rebuild them with a sized buffer.
// Until then the device status word already kept every render exact (the
// lists were not written; every live packet took the exact walk).
static void resolve_bins(CamSet &c, bool block) {
    if (!c.bins_pending) return;
    const hipError_t e = block ? hipEventSynchronize(c.ev_bins) : hipEventQuery(c.ev_bins);
    if (e != hipSuccess) return;   // hipErrorNotReady: later
    c.bins_pending = false;
    const uint32_t gc = c.bins_host[0], st = c.bins_host[1], tot = c.bins_host[2];
    c.bin_gn = gc;
    c.bin_entries = tot;
    if (st != bih::kBinsUnusable) return;
    if (gc > bih::kBinGlobalMax) {
        c.bins_usable = false;
    } else {
        c.bins_regrow = true;
        c.bins_valid = false;   // rebuilt by the next render (after its readers)
        c.bins_redo = true;
    }
}

// A camera set's tile-queue memory for `ntiles` tiles (its renders in
// flight may read the old one).
static int ensure_queue_mem(bih_tree *tr, CamSet &c, uint32_t ntiles, hipStream_t st) {
    if (c.hc_tiles < ntiles) {
        // the hit cache: its stamps start at 0, which no queue's hseq is
        int rc = drain_renders(tr);
        if (rc) return rc;
        if (c.hc) (void)hipFree(c.hc);
        c.hc = nullptr;
        c.hc_tiles = 0;
        hipError_t e = tree_malloc(tr, &c.hc, (size_t)ntiles * 65 * sizeof(uint32_t));
        if (e == hipSuccess) e = hipMemsetAsync(c.hc + (size_t)ntiles * 64, 0, (size_t)ntiles * sizeof(uint32_t), st);
        if (e != hipSuccess) return map_hip((int)e);
        c.hc_tiles = ntiles;
    }
    const size_t need = bih::bin_queue_bytes(ntiles);
    if (c.q_cap >= need) return BIH_OK;
    int rc = drain_renders(tr);
    if (rc) return rc;
    if (c.q_mem) (void)hipFree(c.q_mem);
    c.q_mem = nullptr;
    c.q_cap = 0;
    c.q_valid = false;
    hipError_t e = tree_malloc(tr, &c.q_mem, need);
    if (e != hipSuccess) return map_hip((int)e);
    c.q_cap = need;
    return BIH_OK;
}

// The render kernel's tile queue for this launch's rows (launch_bin_queue):
// rebuilt when the bins or the rows change, after every render that may
// still read the old one.
static int prepare_bin_queue(bih_tree *tr, CamSet &c, int ci, uint32_t w, uint32_t h, uint32_t spp, const bih_rows &rows,
                             int slot, hipStream_t st, bih::RenderArgs &a, uint32_t nframes) {
    uint32_t tw = 0, th = 0;
    tile_shape(spp, &tw, &th);
    const uint32_t tiles_x = (w + tw - 1) / tw;
    const uint32_t ntiles = tiles_x * ((rows.nrows + th - 1) / th);
    const size_t nrec = (size_t)ntiles * nframes;   // fallback records: one per packet at most
    const uint32_t key[8] = {w, h, spp, rows.row0, rows.nrows, rows.band_h, rows.band_step, c.gen};
    int rc = ensure_qcount(tr);
    if (rc) return rc;
    // Queue order: the first launch over these rows (and bins) orders the
    // tiles by list length and measures each live tile's cycles per frame
    // (bins.cost); the next one rebuilds the queue in LPT order of those costs,
    // with the heaviest tiles split over frame ranges (RenderArgs::hsplit) --
    // once per camera and row set (BIH_COST_QUEUE=0: list length only, A/B).
    // Only the order of the work changes, never a pixel.
    const bool measured = cost_queue_enabled() && c.cost_known && memcmp(key, c.cost_key, sizeof key) == 0;
    if (!c.q_valid || memcmp(key, c.q_key, sizeof key) != 0 || (measured && !c.q_cost)) {
        // (after every render that reads the old queue -- and the one that
        // measured the costs)
        rc = wait_set_readers(tr, ci, st);
        if (rc) return rc;
        rc = ensure_queue_mem(tr, c, ntiles, st);
        if (rc) return rc;
        if (!c.q_valid || memcmp(key, c.q_key, sizeof key) != 0) {
            // other tiles, rows or bins: the cached hits of the old queue are void
            c.hseq = ++tr->hseq_ctr;
            if (c.hseq == 0) c.hseq = ++tr->hseq_ctr;
        }
        int le = bih::launch_bin_queue(c.bins.off, c.bins.gcount + 1, c.bins.bins_x, tiles_x, ntiles, rows.row0,
                                       rows.band_h, rows.band_step, th, c.q_mem, &c.q_list, &c.q_hdr,
                                       st, measured ? c.bins.cost : nullptr);
        if (le) return map_hip(le);
        memcpy(c.q_key, key, sizeof key);
        c.q_valid = true;
        c.q_cost = measured;
    }
    // (measured from the camera's second render on: a camera that moves every
    // frame never renders twice, and the measuring instance costs ~1.4x)
    // (cost_known is set once the measuring launch is issued: render_device_impl)
    if (!c.q_cost && !measured && cost_queue_enabled() && c.uses >= 1) {
        a.bin_cost = c.bins.cost;
        memcpy(c.cost_pending, key, sizeof key);
    }
    // heavy tiles: as many items as the others (RenderArgs::nsplit), or --
    // with measured costs -- 2 or 4 times as many, up to one frame each
    a.hsplit = a.nsplit;
    if (c.q_cost && nframes >= 4)
        a.hsplit = std::max(a.nsplit, std::min(nframes, a.nsplit * (nframes >= 8 ? 4u : 2u)));
    if (a.live_items && c.q_cost && nframes >= 4) a.live_items |= 0x80000000u;   // (the kernel's split: heavy tiles too)
    rc = ensure_per_slot(tr, &tr->fb_mem, &tr->fbq_cap, nrec, 8);
    if (rc) return rc;
    a.bin_fb = tr->fb_mem + (size_t)slot * tr->fbq_cap * 8;
    a.bin_queue = c.q_list;
    a.bin_qhdr = c.q_hdr;
    if (hit_cache_enabled() && c.hc && c.hc_tiles >= ntiles) {
        a.hcache = c.hc;
        a.hstamp = c.hc + c.hc_tiles * 64;
        a.hseq = c.hseq;
    }
    // timing experiments (BIH_DBG bits: skip phases or checks; they change
    // pixels, so only a BIH_DEBUG_KNOBS=1 build reads them) and the fallback
    // test mode (routes packets to the exact walk: same pixels)
#if BIH_DEBUG_KNOBS
    a.dbg = dbg_bits();
#endif
    if (tr->prm.force_fallback) a.dbg |= 4u;
    // (q_par[slot] flips once the launch that zeroes the other set is issued)
    const uint32_t par = tr->q_par[slot];
    a.bin_heads = tr->q_count + (size_t)(2 * slot + par) * bih::kBinSetWords;
    a.bin_heads_next = tr->q_count + (size_t)(2 * slot + (par ^ 1u)) * bih::kBinSetWords;
    return BIH_OK;
}

// Frames per k_render_bins item (*fpi) and item splits (*nsplit) of an
// nframes launch over a w x nrows image: every frame of the launch in one
// item when the launch has many tiles (the list is walked nframes times while
// it is cached), fewer when it has few (a rank's bands of the frame), so the
// items keep outnumbering the resident waves.  BIH_PARAM_ITEM_TILES is the
// tile count below which an item's frames are split; it changes the order of
// the work, never a pixel.
static void item_split(const bih_tree *tr, uint32_t w, uint32_t nrows, uint32_t spp, uint32_t nframes,
                       uint32_t *fpi, uint32_t *nsplit) {
    uint32_t tw = 0, th = 0;
    tile_shape(spp, &tw, &th);
    const uint64_t ntiles = (uint64_t)((w + tw - 1) / tw) * ((nrows + th - 1) / th);
    uint64_t ns = ntiles ? (tr->prm.item_tiles + ntiles / 2) / ntiles : nframes;
    ns = std::max<uint64_t>(1, std::min<uint64_t>(ns, nframes));
    *fpi = (uint32_t)((nframes + ns - 1) / ns);
    *nsplit = (nframes + *fpi - 1) / *fpi;
}

// nframes > 1 (bih_render_device_frames): frames frame .. frame+nframes-1 in
// one frustum-bin launch, frame j at d_out + j * out_stride.  Returns
// kRenderPerFrame, before any RNG work, when this render does not go
// through the bins (the caller then renders the frames one by one).
constexpr int kRenderPerFrame = 1;
// hit_mask (config C4's primary rays, one frame): also write each tile's
// 64-bit mask of the samples that hit (RenderArgs::hit_mask), and leave the
// XORWOW ring at this frame's state for the Whitted render that follows
// (kRenderPerFrame, before any work, when the bins do not cover the render).
static int render_device_impl(bih_tree *tr, const bih_camera *cam, uint32_t w, uint32_t h, uint32_t spp,
                              uint32_t frame, uint64_t seed, const bih_rows *rows_in, uint32_t traverse,
                              uint32_t *d_out, uint32_t *d_ray_stats, void *stream, uint32_t nframes,
                              uint64_t out_stride, unsigned long long *hit_mask = nullptr,
                              bool have_lock = false) {
    if (!tr || !cam || !d_out || w == 0 || h == 0 || spp == 0 || traverse > 1) return BIH_ERR_INVALID;
    bih_rows rows = rows_in ? *rows_in : bih_rows{0, h, h, 1};
    if (rows.nrows == 0) return BIH_OK;
    if (rows.band_h == 0 || rows.band_step == 0) return BIH_ERR_INVALID;
    // the last local row must map inside the frame
    uint64_t lr = rows.nrows - 1;
    uint64_t ylast = rows.row0 + (lr / rows.band_h) * (uint64_t)rows.band_h * rows.band_step +
                     (lr % rows.band_h);
    if (ylast >= h) return BIH_ERR_INVALID;
    if ((uint64_t)h * w > 0xFFFFFFFFull) return BIH_ERR_TOO_LARGE;
    DeviceGuard g(tr->t.device);
    // (a Whitted call holds the lock across its mask render and its launch)
    std::unique_lock<std::mutex> lk(tr->mu, std::defer_lock);
    if (!have_lock) lk.lock();
    hipStream_t st = stream ? (hipStream_t)stream : tr->stream;
    // the camera's set of per-camera structures: the one built for this
    // camera, else the next one after the latest render's (with two sets:
    // not the one the renders in flight read)
    uint32_t ob[12];
    static_assert(sizeof(bih_camera) == sizeof ob, "bih_camera is 12 f32");
    memcpy(ob, cam, sizeof ob);
    const int nsets = cam_sets();
    int ci = (tr->cs_cur + 1) % nsets;
    for (int k = 0; k < nsets; ++k) {
        const int j = (tr->cs_cur + k) % nsets;
        if (tr->cs[j].prim_valid && memcmp(ob, tr->cs[j].prim_origin, sizeof ob) == 0) {
            ci = j;
            break;
        }
    }
    CamSet &c = tr->cs[ci];
    resolve_bins(c, false);
    {
        const int rw = ensure_work(tr);
        if (rw) return rw;
    }
    // Dependencies (f = this render, S = kSlots):
    //  - slot: render f-S used this tile queue and spill area, and read rng
    //    buffer (cur+1)%(S+1), which the advance below rewrites;
    //  - rng: the advance issued with render f-1 produced buffer cur (and
    //    ran after render f-1-S, the last reader of buffer cur before).
    // Renders f-S+1 .. f-1 are not waited for: consecutive frames on
    // separate streams overlap, each filling the one before's tail.
    // The camera's structures come first: a new camera's build waits only
    // for the tree and for the renders that read its set (not for the
    // renders or camera builds in flight on other streams), then the slot and
    // the RNG ring as below.
    const int slot = tr->slot;
    int rc = BIH_OK;
    hipError_t e = hipSuccess;
    // the last (re)build: waited for right before the first work of this
    // call that reads the tree, so that the XORWOW advance (which does not)
    // runs beside a rebuild still in flight
    // a build that has completed needs no wait (no barrier packet on `st`)
    if (tr->tree_pending && hipEventQuery(tr->ev_tree) == hipSuccess) tr->tree_pending = false;
    bool tree_waited = !tr->tree_pending;
    auto wait_tree = [&]() -> hipError_t {
        if (tree_waited) return hipSuccess;
        tree_waited = true;
        return hipStreamWaitEvent(st, tr->ev_tree, 0);
    };
    // primary-ray records follow the camera (the origin; the miss-proof boxes
    // also the direction bounds)
    const uint32_t n_int = tr->t.u > 0 ? tr->t.u - 1 : 0;
    if (bih::render_uses_prim(spp) && tr->t.n > 0) {
        const size_t need = bih::prim_bytes(tr->t.n, n_int);
        const bool grow = c.prim_cap < need;
        // (grown to the size of U = N, the most a soup of N triangles can have:
        // trees of other soups of that size reuse it)
        const size_t alloc = bih::prim_bytes(tr->t.n, tr->t.n > 0 ? tr->t.n - 1 : 0);
        if (grow || !c.prim_valid || memcmp(ob, c.prim_origin, sizeof ob) != 0) {
            // rewritten in place: after every render still reading the records
            rc = wait_set_readers(tr, ci, st);
            if (rc) return rc;
        }
        if (grow) {
            rc = drain_renders(tr);
            if (rc) return rc;
            if (c.prim) (void)hipFree(c.prim);
            c.prim = nullptr;
            c.prim_cap = 0;
            e = tree_malloc(tr, &c.prim, std::max(need, alloc));
            if (e != hipSuccess) return map_hip((int)e);
            c.prim_cap = std::max(need, alloc);
            c.prim_valid = false;
        }
        // the frustum bins' build computes the records itself (k_cam_tris)
        const bool want_bins = bins_enabled() && traverse == BIH_TRAVERSE_ANYHIT && !d_ray_stats && n_int > 0;
        bool need_prim = false;
        if (!c.prim_valid || memcmp(ob, c.prim_origin, sizeof ob) != 0) {
            // |D| per component over the primary rays: D = (llc + u h + v vert) - O
            // (Camera.cu:18-20) is affine in (u, v) in [0, 1]^2, so its largest
            // magnitude is at a corner.  The kernel evaluates it in f32: four
            // rounded ops whose results are bounded by |llc|+|h|+|vert|+|O|,
            // so each adds at most 2^-24 of that; the slack takes 2^-21
            // (twice the sum) plus a relative 1e-3 (tests/test_miss_box.py
            // checks it against the kernel's evaluation with offset origins)
            float dmax[3];
            (void)bih_camera_ray_bound(cam, dmax);
            if (want_bins) {
                need_prim = true;
            } else {
                e = wait_tree();
                if (e != hipSuccess) return map_hip((int)e);
                int le = bih::launch_prim(tr->t.tris_s, tr->t.n, tr->t.nodes, tr->t.first_idx,
                                          tr->t.dup_cnt, tr->t.leaf_parent, tr->t.parent, n_int,
                                          cam->origin, dmax, c.prim, st);
                if (le) return map_hip(le);
            }
            memcpy(c.prim_origin, ob, sizeof ob);
            c.prim_valid = true;
            c.bins_valid = false;
            c.fast_valid = false;
            c.cull_valid = false;
        }
        const bool bins_key_ok = c.bins_key[0] == w && c.bins_key[1] == h && c.bins_key[2] == spp;
        if (want_bins && (!c.bins_valid || !bins_key_ok)) {
            // rewritten in place (the triangle and node records too): after
            // every render still reading them (a no-op wait when need_prim
            // already waited above)
            rc = wait_set_readers(tr, ci, st);
            if (rc) return rc;
            float dmax[3];
            (void)bih_camera_ray_bound(cam, dmax);
            e = wait_tree();
            if (e != hipSuccess) return map_hip((int)e);
            rc = build_bins(tr, c, cam, dmax, w, h, spp, need_prim, st);
            if (rc) {
                if (need_prim) c.prim_valid = false;
                return rc;
            }
            c.bins_redo = false;
        }
    }
    if (tr->used[slot]) {
        e = hipStreamWaitEvent(st, tr->evd[slot], 0);
        if (e != hipSuccess) return map_hip((int)e);
    }
    // (also after the structures of a camera an earlier render on another
    // stream built, when this render reuses them)
    e = wait_rng(tr, st);
    if (e != hipSuccess) return map_hip((int)e);
    bih::RenderArgs a;
    bool use_bins = false;
    if (c.bins_usable && c.bins_valid && c.bins_key[0] == w && c.bins_key[1] == h &&
        c.bins_key[2] == spp && traverse == BIH_TRAVERSE_ANYHIT && !d_ray_stats && c.prim) {
        uint32_t tw = 0, th = 0;
        tile_shape(spp, &tw, &th);
        // a packet's rows are one bin row when tiles and bands align
        use_bins = rows.row0 % th == 0 && rows.band_h % th == 0;
    }
    if ((nframes > 1 || hit_mask) && !use_bins) return kRenderPerFrame;
    const size_t P = (size_t)rows.nrows * w;
    // stamped state (RenderArgs::stamps): a frustum-bin launch that follows
    // kStampRun renders on its own stream reads and writes per-tile state and
    // runs no k_rng_advance.  Stamped launches order after each other (ev_rng
    // after the render), which would take away the overlap of frames issued
    // on several streams: a render on another stream leaves the mode
    // (prepare_rng), and renders alternating streams never enter it.
    const bool same_stream = tr->last_slot >= 0 && tr->slot_stream[tr->last_slot] == st;
    const bool stamp_ok = use_bins && !hit_mask && stamps_enabled() &&
                          (uint64_t)frame + nframes <= bih::kStampFrameMax && same_stream &&
                          (tr->stamped || tr->stream_run >= kStampRun);
    const bool stamped = stamp_ok && tr->stamped && rng_same_px(tr, w, spp, seed, rows) && frame >= tr->next_frame &&
                         (uint64_t)(frame - tr->next_frame) * 2 * spp <= 4096;
    if (stamped) {
        // bound the steps a tile's state lags behind (background tiles are
        // not stepped): every kStampJumpFrames frames all tiles to the frame
        // a whole number of those after the last sync (background tiles
        // then jump by one table, k_rng_sync); a tile lags at most two runs
        if (frame - tr->st_sync >= bih::kStampJumpFrames) {
            const uint32_t T = frame - (frame - tr->st_sync) % bih::kStampJumpFrames;
            rc = map_hip(bih::launch_rng_sync(tr->stamps, rng_buf(tr, tr->st_a), rng_buf(tr, (tr->st_a + 1) % kRngBufs),
                                              nullptr, w, rows.nrows, spp, T, next_stamp_seq(tr), tr->t.device, st));
            if (rc) {
                tr->stamped = false;
                tr->rng_valid = false;
                return rc;
            }
            tr->st_sync = T;
        }
    } else {
        // the frame's per-pixel XORWOW state (InitRandGPU / the state earlier
        // frames left), and the state cudaRender leaves behind for the frame
        // after this launch's last (CUDAKernels.cu:419)
        rc = prepare_rng(tr, w, spp, frame, seed, rows, st);
        if (rc) return rc;
    }
    // next_frame now points past this launch while rng_cur still holds its
    // first frame's state: a failure before the launch is issued makes the
    // next call re-seed instead of rendering from stale state
    RngGuard rng_guard{tr};
    if (!stamped && stamp_ok) {
        // into stamped mode: every tile at this frame in rng_cur; after every
        // render in flight (they may read the ring buffers)
        uint32_t tw = 0, th = 0;
        tile_shape(spp, &tw, &th);
        const size_t ntiles = (size_t)((w + tw - 1) / tw) * ((rows.nrows + th - 1) / th);
        rc = ensure_stamps(tr, ntiles, st);
        if (rc) return rc;
        for (int k = 0; k < kSlots; ++k)
            if (tr->used[k]) {
                e = hipStreamWaitEvent(st, tr->evd[k], 0);
                if (e != hipSuccess) return map_hip((int)e);
            }
        rc = map_hip(bih::launch_stamp_init(tr->stamps, (uint32_t)ntiles, frame, st));
        if (rc) return rc;
        tr->stamped = true;
        tr->st_a = tr->rng_cur;
        tr->st_sync = frame;
    }
    const bool use_stamps = stamp_ok;   // (stamped mode from here on)
    const int cur = tr->rng_cur, nxt = (cur + 1) % kRngBufs;
    a.nframes = nframes;
    a.out_stride = out_stride;
    if (use_bins && nframes > 1) {
        // frames per k_render_bins item (item_split; A/B, 1M soup at 1080p, 16 frames per call: one item of 16 frames
        // per tile 0.047 ms per frame, two of 8 0.051; a rank's eighth of the
        // bands, 8 frames per call: items of 8 frames 0.0107 ms per frame, of
        // 2 0.0078; 16 per call, items of 4: 0.0069)
        item_split(tr, w, rows.nrows, spp, nframes, &a.fpi, &a.nsplit);
        // (a caller's BIH_PARAM_ITEM_TILES keeps item_split's rule)
        a.live_items = tr->prm.item_tiles_set ? 0u : live_items_target();
    } else {
        a.fpi = nframes;
        a.nsplit = 1;
    }
    // queue rounds dealt without atomics: one-frame items are short (~10 us),
    // so a refill's round trip is a large part of each
    a.static_rounds = nframes == 1 ? static_rounds_one() : 1u;
    if (use_stamps) {
        // (each item steps its tile's state to its first frame itself)
        a.stamps = tr->stamps;
        a.st_buf0 = rng_buf(tr, tr->st_a);
        a.st_buf1 = rng_buf(tr, (tr->st_a + 1) % kRngBufs);
        a.st_f0 = frame;
        a.st_seq = next_stamp_seq(tr);
    }
    if (hit_mask) {
        // the ring stays at this frame: the Whitted render of the same frame
        // draws the same jitter and advances it
        a.hit_mask = hit_mask;
        tr->next_frame = frame;
    } else if (!use_stamps) {
        // the state after this launch's frames (the next launch's input;
        // the render reads rng_cur only).  (On a stream of its own beside the
        // render, the next render's wait across queues cost more than the
        // advance: one-frame calls 0.107 against 0.087 ms, r05m.)
        rc = map_hip(bih::launch_rng_advance(rng_buf(tr, cur), rng_buf(tr, nxt), P, 2 * spp * nframes, tr->t.device, st));
        if (rc) return rc;
    }
    if (!hit_mask) tr->next_frame = frame + nframes;
    e = wait_tree();
    if (e != hipSuccess) return map_hip((int)e);
    if (use_bins) {
        a.bin_off = c.bins.off;
        a.bin_list = c.bin_list;
        a.bin_glist = c.bin_gent;
        a.bin_rec = c.bins.binrec;
        a.bin_path = c.bins.path;
        a.bins_x = c.bins.bins_x;
        a.bin_gstat = c.bins.gcount + 1;
        rc = prepare_bin_queue(tr, c, ci, w, h, spp, rows, slot, st, a, nframes);
        if (rc) return rc;
        if (hit_mask) a.bin_cost = nullptr;   // (the mask pass's kernel does not measure)
    } else {
        // the cost order pays off for the long BIH walks; with the bins the
        // packets are short and the order's own launch costs more (A/B)
        rc = prepare_chunk_order(tr, w, spp, rows, slot, st, a);
        if (rc) return rc;
    }
    // the BIH walk kernels read the culled node records: built on first use
    // for this camera (renders through the bins never need them)
    if (!use_bins && bih::render_uses_prim(spp) && c.prim && n_int > 0 && !c.cull_valid) {
        rc = wait_set_readers(tr, ci, st);
        if (rc) return rc;
        const int le = bih::launch_prim_cull(tr->t.n, tr->t.nodes, tr->t.first_idx, tr->t.dup_cnt, n_int,
                                             cam->origin, c.prim, st);
        if (le) return map_hip(le);
        c.cull_valid = true;
    }
    // the BIH walk's shortcut boxes (any-hit without bins), built on first
    // use for this camera
    const bool use_fast = c.prim && n_int > 0 && fast_enabled() > 0 && !use_bins &&
                          traverse == BIH_TRAVERSE_ANYHIT && !d_ray_stats;
    if (use_fast && !c.fast_valid) {
        rc = wait_set_readers(tr, ci, st);
        if (rc) return rc;
        float dmax[3];
        (void)bih_camera_ray_bound(cam, dmax);
        const int le = bih::launch_fast_boxes(tr->t.tris_s, tr->t.n, tr->t.nodes, tr->t.first_idx,
                                              tr->t.dup_cnt, tr->t.leaf_parent, tr->t.parent, n_int,
                                              cam->origin, dmax, c.prim, st);
        if (le) return map_hip(le);
        c.fast_valid = true;
    }
    // the next render (on any stream) orders after the advance above, the
    // per-camera records, the shortcut boxes and the tile queue, which it
    // reads as they stand now
    // (stamped: after the render instead -- the next launch reads its stamps)
    if (!use_stamps) {
        e = hipEventRecord(tr->ev_rng, st);
        if (e != hipSuccess) return map_hip((int)e);
        tr->rng_pending = true;
    }
    memcpy(a.cam, cam, sizeof a.cam);
    a.w = w;
    a.h = h;
    a.spp = spp;
    a.row0 = rows.row0;
    a.nrows = rows.nrows;
    a.band_h = rows.band_h;
    a.band_step = rows.band_step;
    uint32_t v[5], d0;
    bih::xorwow_seed(seed, v, &d0);
    a.d_base = d0 + (uint32_t)((uint64_t)2 * spp * frame) * 362437u;
    a.hdr = tr->t.hdr;
    a.hdr_n_tris = tr->t.n;
    a.n_nodes = n_int;
    a.nodes = tr->t.nodes;
    a.tris = tr->t.tris_s;
    a.tri_prim = c.prim;
    a.node_prim = c.prim ? reinterpret_cast<const uint4 *>(c.prim + 16ull * tr->t.n) : nullptr;
    a.node_cull = a.node_prim ? a.node_prim + (n_int + 1) : nullptr;
    a.dup_cnt = tr->t.dup_cnt;
    if (use_fast) {
        a.fast = reinterpret_cast<const float *>(reinterpret_cast<const char *>(c.prim) +
                                                 bih::fast_offset(tr->t.n, n_int));
        if (fast_enabled() > 1) a.fast2 = a.fast + 16ull * (n_int + 1);
    }
    a.rng_in = rng_buf(tr, cur);
    a.pixacc = tr->rng + (size_t)5 * kRngBufs * tr->rng_cap + (size_t)slot * tr->rng_cap;
    a.out = d_out;
    a.ray_stats = d_ray_stats;
    a.work = tr->work + (size_t)slot * bih::kWorkWords;
    a.spill = tr->spill + (size_t)slot * tr->spill_per_slot;
    // another render still running: a multi-frame launch takes fewer
    // resident blocks so that the two overlap (bih_render.hip,
    // bins_grid_blocks); alone, it takes every slot
    // (a render queued on this same stream cannot overlap this one)
    for (int k = 0; k < kSlots && (nframes > 1 || kShareOneFrame) && !a.shared_grid && !use_stamps; ++k)
        if (k != slot && tr->used[k] && tr->slot_stream[k] != st && hipEventQuery(tr->evd[k]) == hipErrorNotReady)
            a.shared_grid = 1;
    // ... and when the caller alternates streams (the last render went to
    // another one), even if that render has finished: the next call is
    // likely to follow on another stream, and its advance and first waves
    // then find free slots instead of waiting for this launch's drain
    // (BIH_SHARE_ALTERNATING=0: A/B)
    if (!a.shared_grid && !use_stamps && (nframes > 1 || kShareOneFrame) && share_alternating() &&
        tr->last_slot >= 0 && tr->slot_stream[tr->last_slot] != st)
        a.shared_grid = 1;
    rc = bih::launch_render(a, traverse, st, tr->timing ? tr->ev0[slot] : nullptr,
                            tr->timing ? tr->ev1[slot] : nullptr);
    if (rc) return map_hip(rc);
    if (use_bins) tr->q_par[slot] ^= 1u;   // this launch zeroes the other set for the next
    if (a.bin_cost) {
        // the next queue of these rows is ordered by the costs this launch writes
        memcpy(c.cost_key, c.cost_pending, sizeof c.cost_key);
        c.cost_known = true;
    }
    if (use_stamps) {
        e = hipEventRecord(tr->ev_rng, st);
        if (e != hipSuccess) return map_hip((int)e);
        tr->rng_pending = true;
    }
    if (tr->timing) {
        e = hipEventRecord(tr->ev2[slot], st);
        if (e != hipSuccess) return map_hip((int)e);
    }
    tr->last_timed = tr->timing;
    tr->slot_timed[slot] = tr->timing;
    e = hipEventRecord(tr->evd[slot], st);
    if (e != hipSuccess) return map_hip((int)e);
    tr->used[slot] = true;
    tr->slot_gen[slot] = tr->gen;
    note_stream(tr, slot, st);
    tr->slot_cs[slot] = ci;
    if (use_bins) ++c.uses;
    tr->cs_cur = ci;
    tr->last_slot = slot;
    tr->slot = (slot + 1) % kSlots;
    if (!hit_mask && !use_stamps) tr->rng_cur = nxt;  // frame+1's state
    rng_guard.armed = false;
    return BIH_OK;
}

int bih_render_device(const bih_tree *ctr, const bih_camera *cam, uint32_t w, uint32_t h, uint32_t spp,
                      uint32_t frame, uint64_t seed, const bih_rows *rows_in, uint32_t traverse,
                      uint32_t *d_out, uint32_t *d_ray_stats, void *stream) {
    return render_device_impl(const_cast<bih_tree *>(ctr), cam, w, h, spp, frame, seed, rows_in, traverse,
                              d_out, d_ray_stats, stream, 1, 0);
}

int bih_render_device_frames(const bih_tree *ctr, const bih_camera *cam, uint32_t w, uint32_t h, uint32_t spp,
                             uint32_t frame0, uint32_t nframes, uint64_t seed, const bih_rows *rows_in,
                             uint32_t *d_out, uint64_t out_stride, void *stream) {
    bih_tree *tr = const_cast<bih_tree *>(ctr);
    if (!tr || !cam || !d_out || w == 0 || h == 0 || spp == 0 || nframes == 0 || nframes > 64)
        return BIH_ERR_INVALID;
    const uint64_t nrows = rows_in ? rows_in->nrows : h;
    if (nframes > 1 && out_stride < nrows * w) return BIH_ERR_INVALID;
    // one launch: items (<= tiles per band x nframes) and records stay far below 2^31
    const bool one_launch = nframes > 1 && (uint64_t)((w + 7) / 4) * ((nrows + 3) / 4 + 1) * nframes < (1ull << 28);
    if (one_launch) {
        const int rc = render_device_impl(tr, cam, w, h, spp, frame0, seed, rows_in, BIH_TRAVERSE_ANYHIT, d_out,
                                          nullptr, stream, nframes, out_stride);
        if (rc != kRenderPerFrame) return rc;
    }
    for (uint32_t j = 0; j < nframes; ++j) {
        const int rc = render_device_impl(tr, cam, w, h, spp, frame0 + j, seed, rows_in, BIH_TRAVERSE_ANYHIT,
                                          d_out + (uint64_t)j * out_stride, nullptr, stream, 1, 0);
        if (rc) return rc;
    }
    return BIH_OK;
}

int bih_reserve(bih_tree *tr, uint32_t w, uint32_t h, uint32_t spp, const bih_rows *rows_in, uint32_t max_frames) {
    if (!tr || w == 0 || h == 0 || spp == 0 || max_frames == 0 || max_frames > 64) return BIH_ERR_INVALID;
    const bih_rows rows = rows_in ? *rows_in : bih_rows{0, h, h, 1};
    if (rows.nrows == 0) return BIH_OK;
    if (rows.band_h == 0 || rows.band_step == 0 || (uint64_t)h * w > 0xFFFFFFFFull) return BIH_ERR_INVALID;
    DeviceGuard g(tr->t.device);
    std::lock_guard<std::mutex> lk(tr->mu);
    const size_t P = (size_t)rows.nrows * w;
    int rc = ensure_rng(tr, P, tr->stream);
    if (!rc) rc = ensure_work(tr);
    if (!rc) rc = ensure_qcount(tr);
    if (rc) return rc;
    // the frustum-bin path: tile queues of every camera set, fallback records
    // (one per packet and frame at most), the stamps
    uint32_t tw = 0, th = 0;
    tile_shape(spp, &tw, &th);
    const uint32_t ntiles = ((w + tw - 1) / tw) * ((rows.nrows + th - 1) / th);
    for (int k = 0; k < cam_sets() && !rc; ++k) rc = ensure_queue_mem(tr, tr->cs[k], ntiles, tr->stream);
    if (!rc) rc = ensure_per_slot(tr, &tr->fb_mem, &tr->fbq_cap, (size_t)ntiles * max_frames, 8);
    if (!rc && stamps_enabled()) rc = ensure_stamps(tr, ntiles, tr->stream);
    if (rc) return rc;
    return map_hip((int)hipStreamSynchronize(tr->stream));
}

int bih_tree_set_param(bih_tree *tr, int param, uint64_t value) {
    if (!tr) return BIH_ERR_INVALID;
    std::lock_guard<std::mutex> lk(tr->mu);
    switch (param) {
    case BIH_PARAM_ITEM_TILES:
        if (value == 0 || value > 0xFFFFFFFFull) return BIH_ERR_INVALID;
        tr->prm.item_tiles = (uint32_t)value;
        tr->prm.item_tiles_set = true;
        return BIH_OK;
    case BIH_PARAM_PAIR_CAP: {
        const uint32_t v = (uint32_t)std::min<uint64_t>(value, 0xFFFFFFFFull);
        if (v == tr->prm.pair_cap) return BIH_OK;
        tr->prm.pair_cap = v;
        break;
    }
    case BIH_PARAM_BINS_CAP:
        if (value == tr->prm.bins_cap) return BIH_OK;
        tr->prm.bins_cap = value;
        break;
    case BIH_PARAM_FORCE_FALLBACK:
        if (value > 1) return BIH_ERR_INVALID;
        tr->prm.force_fallback = (uint32_t)value;
        return BIH_OK;
    case BIH_PARAM_WHITTED_COUNTERS:
        if (value > 1) return BIH_ERR_INVALID;
        tr->prm.wh_counters = (uint32_t)value;
        return BIH_OK;
    case BIH_PARAM_STATIC_SOUP:
        if (value > 1) return BIH_ERR_INVALID;
        // the caller may write the soup from now on: no asynchronous rebuild
        // (which reads it) may still be running on the second build stream
        if (!value && tr->bstream) {
            DeviceGuard g(tr->t.device);
            const hipError_t e = hipStreamSynchronize(tr->bstream);
            if (e != hipSuccess) return map_hip((int)e);
        }
        tr->prm.static_soup = (uint32_t)value;
        return BIH_OK;
    case BIH_PARAM_TEST_ALLOC_FAIL:
        if (value > 64) return BIH_ERR_INVALID;
        tr->prm.test_alloc_fail = (uint32_t)value;
        return BIH_OK;
    default:
        return BIH_ERR_INVALID;
    }
    // the bins of every camera set were built under the old cap: rebuilt by
    // their next render
    for (CamSet &c : tr->cs) c.bins_valid = false;
    return BIH_OK;
}

int bih_render_whitted_device(const bih_tree *ctr, const bih_camera *cam, uint32_t w, uint32_t h,
                              uint32_t spp, uint32_t frame, uint64_t seed, const bih_rows *rows_in,
                              uint32_t *d_out, uint32_t *d_hits, void *stream) {
    bih_tree *tr = const_cast<bih_tree *>(ctr);
    if (!tr || !cam || !d_out || w == 0 || h == 0 || spp == 0) return BIH_ERR_INVALID;
    bih_rows rows = rows_in ? *rows_in : bih_rows{0, h, h, 1};
    if (rows.nrows == 0) return BIH_OK;
    if (rows.band_h == 0 || rows.band_step == 0) return BIH_ERR_INVALID;
    uint64_t lr = rows.nrows - 1;
    uint64_t ylast = rows.row0 + (lr / rows.band_h) * (uint64_t)rows.band_h * rows.band_step +
                     (lr % rows.band_h);
    if (ylast >= h) return BIH_ERR_INVALID;
    // u32 ray ids, and k_wh_trace_dyn's u32 fetch counter overshoots the ray
    // count by at most one 64-ray fetch per wave of its grid (<= 2^20 lanes)
    if ((uint64_t)h * w * spp > 0xFFFFFFFFull - (1ull << 20)) return BIH_ERR_TOO_LARGE;
    DeviceGuard g(tr->t.device);
    // one lock over the mask render and the Whitted launch: no other call
    // through this tree slips in between
    std::lock_guard<std::mutex> lk(tr->mu);
    hipStream_t st = stream ? (hipStream_t)stream : tr->stream;
    // Bounce 0 through the frustum bins: the any-hit render of the same
    // frame (the primary render's kernels) leaves per tile the mask of its
    // samples that hit; only those enter the closest-hit walk of bounce 0 (a
    // proven miss has no closest hit: same visit set, same test).  Its pixels
    // go to d_out, which the Whitted shade overwrites.  BIH_WH_BINS=0: every
    // primary sample is walked (A/B).
    unsigned long long *mask = nullptr;
    uint32_t mask_tiles_x = 0;
    static const bool wh_bins = [] {
        const char *e = getenv("BIH_WH_BINS");
        return !(e && e[0] == '0');
    }();
    // With work counters on, every primary sample is walked, so that the
    // counts equal the oracle's on every frame.
    if (wh_bins && bins_enabled() && !tr->prm.wh_counters && spp <= 64 && (spp & (spp - 1)) == 0 &&
        tr->t.u > 1) {
        uint32_t tw = 0, th = 0;
        tile_shape(spp, &tw, &th);
        mask_tiles_x = (w + tw - 1) / tw;
        const size_t ntiles = (size_t)mask_tiles_x * ((rows.nrows + th - 1) / th);
        if (tr->wh_mask_cap < ntiles) {
            int rc = drain_renders(tr);
            if (rc) return rc;
            if (tr->wh_mask) (void)hipFree(tr->wh_mask);
            tr->wh_mask = nullptr;
            tr->wh_mask_cap = 0;
            hipError_t e = tree_malloc(tr, &tr->wh_mask, ntiles * 8);
            if (e != hipSuccess) return map_hip((int)e);
            tr->wh_mask_cap = ntiles;
        } else if (tr->wh_prev_slot >= 0 && tr->used[tr->wh_prev_slot]) {
            // the mask is rewritten in place: after the last Whitted launch
            // (its k_wh_gen reads the previous mask), whatever stream it ran on
            hipError_t e = hipStreamWaitEvent(st, tr->evd[tr->wh_prev_slot], 0);
            if (e != hipSuccess) return map_hip((int)e);
        }
        const int mrc = render_device_impl(tr, cam, w, h, spp, frame, seed, &rows, BIH_TRAVERSE_ANYHIT, d_out,
                                           nullptr, stream, 1, 0, tr->wh_mask, true);
        if (mrc == BIH_OK) mask = tr->wh_mask;
        else if (mrc != kRenderPerFrame) return mrc;
    }
    // the queues are shared by every Whitted render of this tree: order after
    // every render in flight (and after the last writer of the RNG ring)
    int rc = wait_renders(tr, st);
    if (rc) return rc;
    {
        hipError_t e = wait_rng(tr, st);
        if (e != hipSuccess) return map_hip((int)e);
    }
    if (tr->tree_pending && hipEventQuery(tr->ev_tree) == hipSuccess) tr->tree_pending = false;
    if (tr->tree_pending) {   // the last (re)build (a rebuild does not order ev_rng)
        hipError_t e = hipStreamWaitEvent(st, tr->ev_tree, 0);
        if (e != hipSuccess) return map_hip((int)e);
    }
    // bih_whitted_work describes the last Whitted launch issued: none until
    // this one is (a failure below, or a reallocated wh_mem, leaves nothing
    // to read)
    tr->wh_last_slot = -1;
    rc = prepare_rng(tr, w, spp, frame, seed, rows, st);
    if (rc) return rc;
    RngGuard rng_guard{tr};
    const size_t P = (size_t)rows.nrows * w;
    const uint64_t rays = (uint64_t)P * spp;
    const int cur = tr->rng_cur, nxt = (cur + 1) % kRngBufs;
    rc = map_hip(bih::launch_rng_advance(rng_buf(tr, cur), rng_buf(tr, nxt), P, 2 * spp, tr->t.device, st));
    if (rc) return rc;
    if (tr->wh_rays < rays) {
        hipError_t e = hipStreamSynchronize(st);   // the previous Whitted render's readers
        if (e != hipSuccess) return map_hip((int)e);
        if (tr->wh_mem) (void)hipFree(tr->wh_mem);
        tr->wh_mem = nullptr;
        tr->wh_rays = 0;
        e = tree_malloc(tr, &tr->wh_mem, bih::whitted_bytes(rays));
        if (e != hipSuccess) return map_hip((int)e);
        tr->wh_rays = rays;
    }
    hipError_t e = hipEventRecord(tr->ev_rng, st);
    if (e != hipSuccess) return map_hip((int)e);
    tr->rng_pending = true;
    bih::RenderArgs a;
    memcpy(a.cam, cam, sizeof a.cam);
    a.w = w;
    a.h = h;
    a.spp = spp;
    a.row0 = rows.row0;
    a.nrows = rows.nrows;
    a.band_h = rows.band_h;
    a.band_step = rows.band_step;
    uint32_t v[5], d0;
    bih::xorwow_seed(seed, v, &d0);
    a.d_base = d0 + (uint32_t)((uint64_t)2 * spp * frame) * 362437u;
    a.hdr = tr->t.hdr;
    a.hdr_n_tris = tr->t.n;
    a.n_nodes = tr->t.u > 0 ? tr->t.u - 1 : 0;
    a.nodes = tr->t.nodes;
    a.tris = tr->t.tris_s;
    a.dup_cnt = tr->t.dup_cnt;
    a.rng_in = rng_buf(tr, cur);
    a.out = d_out;
    const int slot = tr->slot;
    const bool count = tr->prm.wh_counters != 0;
    rc = bih::launch_whitted(a, tr->wh_mem, rays, d_hits, st, tr->timing ? tr->ev0[slot] : nullptr,
                             tr->timing ? tr->ev1[slot] : nullptr, count, mask, mask_tiles_x);
    if (rc) return map_hip(rc);
    tr->wh_last_rays = rays;
    tr->wh_last_slot = count ? slot : -1;
    tr->wh_prev_slot = slot;
    if (tr->timing) {
        e = hipEventRecord(tr->ev2[slot], st);
        if (e != hipSuccess) return map_hip((int)e);
    }
    tr->last_timed = tr->timing;
    tr->slot_timed[slot] = tr->timing;
    e = hipEventRecord(tr->evd[slot], st);
    if (e != hipSuccess) return map_hip((int)e);
    tr->used[slot] = true;
    tr->slot_gen[slot] = tr->gen;
    note_stream(tr, slot, st);
    tr->slot_cs[slot] = -1;            // reads no camera set
    tr->last_slot = slot;
    tr->slot = (slot + 1) % kSlots;
    tr->rng_cur = nxt;
    rng_guard.armed = false;
    return BIH_OK;
}

int bih_whitted_work(const bih_tree *ctr, uint32_t rays[BIH_WHITTED_BOUNCES + 1],
                     uint64_t nodes[BIH_WHITTED_BOUNCES + 1], uint64_t tris[BIH_WHITTED_BOUNCES + 1]) {
    bih_tree *tr = const_cast<bih_tree *>(ctr);
    if (!tr || !rays || !nodes || !tris) return BIH_ERR_INVALID;
    DeviceGuard g(tr->t.device);
    std::lock_guard<std::mutex> lk(tr->mu);
    // the last Whitted render, with counters on, and no Whitted render since
    if (tr->wh_last_slot < 0 || !tr->wh_mem) return BIH_ERR_INVALID;
    hipError_t e = hipEventSynchronize(tr->evd[tr->wh_last_slot]);
    if (e != hipSuccess) return map_hip((int)e);
    unsigned long long w[2 * (BIH_WHITTED_BOUNCES + 1)];
    const int rc = bih::whitted_work(tr->wh_mem, tr->wh_last_rays, rays, w, tr->stream);
    if (rc) return map_hip(rc);
    for (int d = 0; d <= BIH_WHITTED_BOUNCES; ++d) {
        nodes[d] = w[2 * d];
        tris[d] = w[2 * d + 1];
    }
    return BIH_OK;
}

int bih_render_whitted(const bih_scene *scene, const bih_tree *ctr, const bih_camera *cam,
                       bih_framebuffer *fb) {
    bih_tree *tr = const_cast<bih_tree *>(ctr);
    if (!tr || !cam || !fb || !fb->rgba) return BIH_ERR_INVALID;
    if (scene && (scene->n_tris != tr->t.n || (tr->host_v && scene->v != tr->host_v)))
        return BIH_ERR_MISMATCH;
    if (fb->w == 0 || fb->h == 0 || fb->spp == 0) return BIH_ERR_INVALID;
    DeviceGuard g(tr->t.device);
    const size_t P = (size_t)fb->h * fb->w;
    {
        std::lock_guard<std::mutex> lk(tr->mu);
        if (P > tr->fb_cap) {
            if (tr->fb) (void)hipFree(tr->fb);
            tr->fb = nullptr;
            tr->fb_cap = 0;
            hipError_t e = tree_malloc(tr, &tr->fb, P * 4);
            if (e != hipSuccess) return map_hip((int)e);
            tr->fb_cap = P;
        }
    }
    int rc = bih_render_whitted_device(tr, cam, fb->w, fb->h, fb->spp, fb->frame, fb->seed, nullptr, tr->fb,
                                       nullptr, nullptr);
    if (rc) return rc;
    hipError_t e = hipMemcpyAsync(fb->rgba, tr->fb, P * 4, hipMemcpyDeviceToHost, tr->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(tr->stream);
    return map_hip((int)e);
}

int bih_sync(const bih_tree *tr, void *stream) {
    if (!tr) return BIH_ERR_INVALID;
    DeviceGuard g(tr->t.device);
    hipStream_t st = stream ? (hipStream_t)stream : tr->stream;
#if BIH_BINS_TIMELINE
    if (const char *path = getenv("BIH_TIMELINE_OUT")) {
        if (hipStreamSynchronize(st) == hipSuccess) (void)bih::bins_timeline_dump(path);
    }
#endif
#if BIH_WAVE_TIMELINE
    if (tr->spill && tr->last_slot >= 0 && hipStreamSynchronize(st) == hipSuccess) {
        // per-wave records of k_render_packet_asm at each wave's spill base
        const size_t per = (size_t)(bih::kStackDepth - 16) * 3 * 64;   // kPacketRegs = 16
        const size_t waves = tr->spill_per_slot / per;
        std::vector<uint32_t> h(tr->spill_per_slot);
        if (hipMemcpy(h.data(), tr->spill + (size_t)tr->last_slot * tr->spill_per_slot,
                      h.size() * 4, hipMemcpyDeviceToHost) == hipSuccess) {
            // times: s_memrealtime (100 MHz), relative to the XCD's first
            // wave start and its last wave end
            uint64_t x0[16], x1[16];
            for (int x = 0; x < 16; ++x) { x0[x] = ~0ull; x1[x] = 0; }
            for (size_t w = 0; w < waves; ++w) {
                const uint32_t *r = h.data() + w * per;
                const uint64_t b = r[0] | ((uint64_t)r[1] << 32), e = r[2] | ((uint64_t)r[3] << 32);
                const uint32_t x = r[9] & 15;
                if (!b || e < b) continue;
                x0[x] = b < x0[x] ? b : x0[x];
                x1[x] = e > x1[x] ? e : x1[x];
            }
            double life = 0, spans = 0;
            uint64_t npk = 0, nlive = 0, maxpk = 0;
            double maxpk_at = 0, maxpk_frac = 0;
            std::vector<double> ends, lasts;
            for (size_t w = 0; w < waves; ++w) {
                const uint32_t *r = h.data() + w * per;
                const uint64_t b = r[0] | ((uint64_t)r[1] << 32), e = r[2] | ((uint64_t)r[3] << 32);
                const uint64_t l = r[4] | ((uint64_t)r[5] << 32);
                const uint64_t m = r[10] | ((uint64_t)r[11] << 32);
                const uint32_t x = r[9] & 15;
                if (!b || e < b) continue;
                const double span = (double)(x1[x] - x0[x]);
                life += (double)(e - b) / span;
                ends.push_back((double)(e - x0[x]) / span);
                lasts.push_back((double)(l - x0[x]) / span);
                npk += r[6];
                nlive += r[7];
                if (r[8] > maxpk) {
                    maxpk = r[8];
                    maxpk_at = (double)(m - x0[x]) / span;
                    maxpk_frac = (double)r[8] / span;
                }
            }
            for (int x = 0; x < 16; ++x)
                if (x1[x]) spans = spans > (double)(x1[x] - x0[x]) ? spans : (double)(x1[x] - x0[x]);
            if (!ends.empty()) {
                std::sort(ends.begin(), ends.end());
                std::sort(lasts.begin(), lasts.end());
                auto q = [](const std::vector<double> &v, double f) { return v[(size_t)(f * (v.size() - 1))]; };
                fprintf(stderr,
                        "wave-timeline waves %zu xcd-span max %.0f x10ns mean-life %.3f packets %llu live %llu "
                        "max-packet %llu x10ns = %.3f span, starts at %.3f | wave end q10 %.3f q50 %.3f q90 %.3f | "
                        "last packet start q50 %.3f q90 %.3f q99 %.3f max %.3f\n",
                        ends.size(), spans, life / ends.size(), (unsigned long long)npk,
                        (unsigned long long)nlive, (unsigned long long)maxpk, maxpk_frac, maxpk_at,
                        q(ends, 0.1), q(ends, 0.5), q(ends, 0.9), q(lasts, 0.5), q(lasts, 0.9),
                        q(lasts, 0.99), q(lasts, 1.0));
            }
        }
    }
#endif
#ifndef BIH_PHASES
#define BIH_PHASES BIH_FAST_COUNTERS
#endif
#if BIH_PHASES && !BIH_FAST_COUNTERS
    if (tr->work && tr->last_slot >= 0) {
        uint32_t c[80];
        if (hipMemcpyAsync(c, tr->work + (size_t)tr->last_slot * bih::kWorkWords, sizeof c,
                           hipMemcpyDeviceToHost, st) == hipSuccess &&
            hipStreamSynchronize(st) == hipSuccess) {
            const unsigned long long *ph = reinterpret_cast<const unsigned long long *>(c + 64);
            fprintf(stderr,
                    "bin-phases (wave cycles) queue %llu background %llu setup %llu walk %llu verify %llu"
                    " write %llu\n", ph[0], ph[1], ph[2], ph[3], ph[4], ph[5]);
        }
    }
#endif
#if BIH_FAST_COUNTERS
    if (tr->work && tr->last_slot >= 0) {
        uint32_t c[80];
        if (hipMemcpyAsync(c, tr->work + (size_t)tr->last_slot * bih::kWorkWords, sizeof c,
                           hipMemcpyDeviceToHost, st) == hipSuccess &&
            hipStreamSynchronize(st) == hipSuccess) {
            const unsigned long long *cy = reinterpret_cast<const unsigned long long *>(c + 32);
            fprintf(stderr,
                    "fast-counters packets %u lanes %u | pass1 steps %u tests %u cand %u verified %u"
                    " | pass2 packets %u steps %u tests %u verified %u proven-miss %u"
                    " | exact packets %u lanes %u | cycles pass1 %llu (walk %llu) pass2 %llu"
                    " exact %llu\n",
                    c[16], c[17], c[18], c[19], c[20], c[21], c[22], c[23], c[24], c[25], c[26],
                    c[28], c[29], cy[0], cy[3], cy[1], cy[2]);
            const unsigned long long *cb = reinterpret_cast<const unsigned long long *>(c + 48);
            fprintf(stderr,
                    "bin-counters packets %u lanes %u entries %u mt %u found %u verified %u"
                    " unverified %u packets-with-miss %u planned %u plan-disagrees %u cache-hits %u"
                    " | cycles walk %llu verify %llu\n",
                    c[40], c[41], c[42], c[43], c[44], c[45], c[46], c[47], c[39], c[38], c[52], cb[0], cb[1]);
            const unsigned long long *ph = reinterpret_cast<const unsigned long long *>(c + 64);
            fprintf(stderr,
                    "bin-phases (wave cycles) queue %llu background %llu setup %llu walk %llu verify %llu"
                    " write %llu\n", ph[0], ph[1], ph[2], ph[3], ph[4], ph[5]);
        }
    }
#endif
#if BIH_PACKET_COUNTERS
    if (tr->work && tr->last_slot >= 0) {
        uint32_t c[bih::kWorkWords];
        if (hipMemcpyAsync(c, tr->work + (size_t)tr->last_slot * bih::kWorkWords, sizeof c, hipMemcpyDeviceToHost, st) == hipSuccess &&
            hipStreamSynchronize(st) == hipSuccess) {
            fprintf(stderr, "packet-counters packets %u nodes %u leaves %u tris %u pushes %u pops %u maxsp %u depth",
                    c[16], c[17], c[18], c[19], c[20], c[21], c[22]);
            for (int k = 0; k < 32; ++k) fprintf(stderr, " %u", c[24 + k]);
            fprintf(stderr, " mt");
            for (int k = 0; k < 8; ++k) fprintf(stderr, " %u", c[56 + k]);
            fprintf(stderr, " lanes-node(log2)");
            for (int k = 0; k < 8; ++k) fprintf(stderr, " %u", c[bih::kHistWord + k]);
            fprintf(stderr, " lanes-tri(log2)");
            for (int k = 0; k < 8; ++k) fprintf(stderr, " %u", c[bih::kHistWord + 8 + k]);
            fprintf(stderr, "\npackets by log2(node steps): bin count nodes tris\n");
            for (int k = 0; k < 16; ++k)
                if (c[bih::kHistWord + 16 + k])
                    fprintf(stderr, "  %2d %8u %10u %10u\n", k, c[bih::kHistWord + 16 + k],
                            c[bih::kHistWord + 32 + k], c[bih::kHistWord + 48 + k]);
        }
    }
#endif
    return map_hip((int)hipStreamSynchronize(st));
}

int bih_set_timing(bih_tree *tr, int on) {
    if (!tr) return BIH_ERR_INVALID;
    std::lock_guard<std::mutex> lk(tr->mu);
    tr->timing = on != 0;
    return BIH_OK;
}

int bih_last_render_ms(const bih_tree *tr, double *ms) {
    if (!tr || !ms || tr->last_slot < 0 || !tr->last_timed) return BIH_ERR_INVALID;
    DeviceGuard g(tr->t.device);
    const int k = tr->last_slot;
    hipError_t e = hipEventSynchronize(tr->evd[k]);
    if (e != hipSuccess) return map_hip((int)e);
    float f = 0.f;
    e = hipEventElapsedTime(&f, tr->ev0[k], tr->ev1[k]);
    if (e != hipSuccess) return map_hip((int)e);
    *ms = f;
    return BIH_OK;
}

int bih_last_render_times(const bih_tree *tr, double *kernel_ms, double *tail_ms) {
    if (!tr || !kernel_ms || !tail_ms || tr->last_slot < 0 || !tr->last_timed) return BIH_ERR_INVALID;
    DeviceGuard g(tr->t.device);
    const int k = tr->last_slot;
    hipError_t e = hipEventSynchronize(tr->evd[k]);
    if (e != hipSuccess) return map_hip((int)e);
    float f0 = 0.f, f1 = 0.f;
    e = hipEventElapsedTime(&f0, tr->ev0[k], tr->ev1[k]);
    if (e == hipSuccess) e = hipEventElapsedTime(&f1, tr->ev1[k], tr->ev2[k]);
    if (e != hipSuccess) return map_hip((int)e);
    *kernel_ms = f0;
    *tail_ms = f1;
    return BIH_OK;
}

int bih_render_history(const bih_tree *tr, uint32_t n, double *t) {
    if (!tr || !t || n == 0 || n > (uint32_t)kSlots || tr->last_slot < 0 || !tr->last_timed) return BIH_ERR_INVALID;
    DeviceGuard g(tr->t.device);
    std::lock_guard<std::mutex> lk(tr->mu);
    // slot of the i-th of the last n renders (slots are taken in turn)
    auto slot_of = [&](uint32_t i) { return (tr->last_slot - (int)(n - 1 - i) + 2 * kSlots) % kSlots; };
    for (uint32_t i = 0; i < n; ++i)
        if (!tr->used[slot_of(i)] || !tr->slot_timed[slot_of(i)]) return BIH_ERR_INVALID;
    const hipEvent_t base = tr->ev0[slot_of(0)];
    for (uint32_t i = 0; i < n; ++i) {
        const int k = slot_of(i);
        hipError_t e = hipEventSynchronize(tr->evd[k]);
        float a = 0.f, b = 0.f, c = 0.f;
        if (e == hipSuccess) e = hipEventElapsedTime(&a, base, tr->ev0[k]);
        if (e == hipSuccess) e = hipEventElapsedTime(&b, base, tr->ev1[k]);
        if (e == hipSuccess) e = hipEventElapsedTime(&c, base, tr->ev2[k]);
        if (e != hipSuccess) return map_hip((int)e);
        t[3 * i] = a;
        t[3 * i + 1] = b;
        t[3 * i + 2] = c;
    }
    return BIH_OK;
}

int bih_host_register(void *ptr, size_t bytes) {
    if (!ptr || bytes == 0) return BIH_ERR_INVALID;
    if (bih_device_count() <= 0) return BIH_ERR_NO_DEVICE;
    return map_hip((int)hipHostRegister(ptr, bytes, hipHostRegisterPortable));
}

int bih_host_unregister(void *ptr) {
    if (!ptr) return BIH_ERR_INVALID;
    if (bih_device_count() <= 0) return BIH_ERR_NO_DEVICE;
    return map_hip((int)hipHostUnregister(ptr));
}

int bih_bins_get_stats(const bih_tree *ctr, bih_bins_stats *out) {
    if (!ctr || !out) return BIH_ERR_INVALID;
    bih_tree *tr = const_cast<bih_tree *>(ctr);
    DeviceGuard g(tr->t.device);
    std::lock_guard<std::mutex> lk(tr->mu);
    CamSet &c = tr->cs[tr->cs_cur];   // the latest render's camera
    resolve_bins(c, true);
    memset(out, 0, sizeof *out);
    out->usable = c.bins_usable && c.bins_valid ? 1u : 0u;
    out->tiles_x = c.bins.bins_x;
    out->tiles_y = c.bins.bins_y;
    out->list_entries = c.bin_entries;
    out->global_entries = c.bin_gn;
    return BIH_OK;
}

static int render_host(const bih_scene *scene, const bih_tree *ctr, const bih_camera *cam,
                       bih_framebuffer *fb, uint32_t row0, uint32_t nrows) {
    bih_tree *tr = const_cast<bih_tree *>(ctr);
    if (!tr || !cam || !fb || !fb->rgba) return BIH_ERR_INVALID;
    if (scene && (scene->n_tris != tr->t.n || (tr->host_v && scene->v != tr->host_v)))
        return BIH_ERR_MISMATCH;
    if (fb->w == 0 || fb->h == 0 || fb->spp == 0) return BIH_ERR_INVALID;
    if ((uint64_t)row0 + nrows > fb->h) return BIH_ERR_INVALID;
    if (nrows == 0) return BIH_OK;
    DeviceGuard g(tr->t.device);
    const size_t P = (size_t)nrows * fb->w;
    {
        std::lock_guard<std::mutex> lk(tr->mu);
        if (P > tr->fb_cap) {
            if (tr->fb) (void)hipFree(tr->fb);
            tr->fb = nullptr;
            tr->fb_cap = 0;
            hipError_t e = tree_malloc(tr, &tr->fb, P * 4);
            if (e != hipSuccess) return map_hip((int)e);
            tr->fb_cap = P;
        }
    }
    bih_rows rows{row0, nrows, nrows, 1};
    int rc = bih_render_device(tr, cam, fb->w, fb->h, fb->spp, fb->frame, fb->seed, &rows,
                               BIH_TRAVERSE_ANYHIT, tr->fb, nullptr, nullptr);
    if (rc) return rc;
    hipError_t e = hipMemcpyAsync(fb->rgba, tr->fb, P * 4, hipMemcpyDeviceToHost, tr->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(tr->stream);
    return map_hip((int)e);
}

int bih_render(const bih_scene *scene, const bih_tree *tr, const bih_camera *cam, bih_framebuffer *fb) {
    if (!fb) return BIH_ERR_INVALID;
    return render_host(scene, tr, cam, fb, 0, fb->h);
}

int bih_render_rows(const bih_scene *scene, const bih_tree *tr, const bih_camera *cam,
                    bih_framebuffer *fb, uint32_t row0, uint32_t nrows) {
    return render_host(scene, tr, cam, fb, row0, nrows);
}

}  // extern "C"
