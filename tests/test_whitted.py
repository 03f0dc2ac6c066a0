"""Config C4 (BASELINE.json configs[3]): 8-bounce Whitted mirror rays.

The reference has primary rays only (Color, src/CUDAKernels.cu:370-389), so
C4's semantics are this build's own (oracle
ob_render_whitted); parity is the HIP path against that oracle, bit-exact.
CPU tests pin the oracle's rules on hand-built scenes; -m gpu tests compare
bih_render_whitted_device with it."""
import numpy as np
import pytest

from conftest import edge_scenes

F32 = np.float32
BG, Y = (20.0, 20.0, 40.0), (255.0, 255.0, 0.0)


def shade(h):
    """f32 shade of a sample with h hits (the oracle's whitted_shade)."""
    c = [F32(x) for x in (Y if h > 8 else BG)]
    for _ in range(min(h, 8)):
        c = [F32(0.5) * F32(y) + F32(0.5) * x for x, y in zip(c, Y)]
    return c


def pixel_of(hs):
    """rgbToInt of the spp samples' mean shade (cudaRender :420-422)."""
    col = [F32(0), F32(0), F32(0)]
    for h in hs:
        col = [a + b for a, b in zip(col, shade(h))]
    fs = F32(len(hs))
    r, g, b = [int(max(F32(0), min(F32(255), c / fs))) for c in col]
    return (b << 16) | (g << 8) | r


def _mirror_pair(gap=1.0, size=50.0):
    """Two large facing squares (4 triangles) at z = 0 (facing +z) and z = gap
    (facing -z): a ray between them bounces until the path limit."""
    s = size
    lo = [[-s, -s, 0, s, -s, 0, s, s, 0], [-s, -s, 0, s, s, 0, -s, s, 0]]           # normal +z
    hi = [[-s, -s, gap, s, s, gap, s, -s, gap], [-s, -s, gap, -s, s, gap, s, s, gap]]  # normal -z
    return np.array(lo + hi, F32)


def test_shades_are_dyadic_and_distinct():
    vals = [pixel_of([h] * 4) for h in range(10)]
    assert len(set(vals)) == 10
    assert vals[0] == 0x281414                    # every sample missed: (20, 20, 40)
    assert vals[9] == 0x00FFFF or vals[9] == pixel_of([9] * 4)


def test_oracle_mirror_pair_known_answers(oracle_mod):
    ot = oracle_mod.OracleTree(_mirror_pair())
    # a ray from between the mirrors, slanted: hits the bottom mirror first
    t, i = ot.closest((0.0, 0.0, 0.5), (0.1, 0.05, -1.0))
    assert i >= 0 and abs(t - 0.5) < 1e-6
    # the ray leaving the top mirror downwards from outside: back face culled
    t, i = ot.closest((0.0, 0.0, 2.0), (0.0, 0.0, -1.0))
    assert i >= 0 and abs(t - 2.0) < 1e-6          # passes through the top (back face), hits the bottom
    # a camera between the mirrors looking down: every sample hits all 9 times
    cam = np.array([0, 0, 0.5, -0.2, -0.2, 0.0, 0.4, 0, 0, 0, 0.4, 0], F32)
    img, st, dep = ot.render_whitted(8, 8, cam=cam, depths=True)
    assert (dep == 9).all()
    assert st.slab_miss == 8 * 8 * 4 * 9        # rays traced: primary + 8 bounces each
    assert (img == pixel_of([9] * 4)).all()


def test_oracle_single_mirror_one_bounce(oracle_mod):
    """One mirror facing the camera: every primary ray hits once, its reflection
    leaves the scene: h = 1."""
    tri = np.array([[-10, -10, 0, 10, -10, 0, 0, 10, 0]], F32)     # normal +z
    tri = np.concatenate([tri, tri + F32(100)])                   # two leaves, far apart
    ot = oracle_mod.OracleTree(tri)
    cam = np.array([0, 0, 5, -0.5, -0.5, 0, 1, 0, 0, 0, 1, 0], F32)
    img, _, dep = ot.render_whitted(16, 16, cam=cam, depths=True)
    assert (dep == 1).all()
    assert (img == pixel_of([1] * 4)).all()


def test_oracle_closest_equals_brute_force(oracle_mod, bihrt_mod):
    """The C4 closest hit (reference walk's visit set, min (t, i)) against a
    brute-force minimum over every triangle (restating RayTriangleIntersection
    per triangle through ob_mt): equal except where f32 plane rounding makes
    the reference walk skip a leaf (the reference's own behaviour)."""
    tris = bihrt_mod.scenes.soup(1500, seed=8, lo=(0.0, -1.0, 0.0), size=(2.667, 2.0, 2.0))
    ot = oracle_mod.OracleTree(tris)
    rng = np.random.default_rng(3)
    sorted_tris = tris[ot.tri_idx]
    agree = 0
    n = 120
    for _ in range(n):
        o = rng.uniform([-0.5, -1.5, -1.0], [3.0, 1.5, 3.0]).astype(F32)
        d = (rng.uniform([0.5, -0.8, 0.2], [2.0, 0.8, 1.8]) - o).astype(F32)
        t, i = ot.closest(o, d, 0.0)
        best = (np.float32(np.finfo(F32).max), -1)
        for k in range(sorted_tris.shape[0]):
            hit, tk = oracle_mod.mt(sorted_tris[k], o, d)
            if hit and 0.0 < tk < float(np.finfo(F32).max) and (tk, k) < best:
                best = (np.float32(tk), k)
        agree += (i == best[1]) and (i < 0 or t == float(best[0]))
    assert agree >= n - 1


def test_oracle_whitted_primary_hits_match_primary_render(oracle_mod):
    """h > 0 exactly for the samples the primary render (reference walk)
    counts as hits: the C4 path starts from cudaRender's rays."""
    tris = edge_scenes()["cornell"]
    ot = oracle_mod.OracleTree(tris)
    img_w, _, dep = ot.render_whitted(64, 64, depths=True)
    img_p, _ = ot.render(64, 64)
    hits_per_px = (dep.reshape(64, 64, 4) > 0).sum(-1)
    k_from_primary = {0x281414: 0, 0x1e4e4e: 1, 0x148989: 2, 0x0ac4c4: 3, 0x00ffff: 4}
    assert np.array_equal(hits_per_px, np.vectorize(k_from_primary.get)(img_p))
    # and the pixel is the formula of the per-sample hit counts
    d = dep.reshape(64, 64, 4)
    for y in range(0, 64, 7):
        for x in range(0, 64, 5):
            assert img_w[y, x] == pixel_of(d[y, x].tolist())


# --- GPU parity (bih_render_whitted_device vs the oracle) ----------------------

def _whitted_device(bihrt, g, w, h, frame, rows=None, spp=4):
    import torch
    nrows = rows.nrows if rows is not None else h
    out = torch.zeros(nrows * w, dtype=torch.int32, device="cuda")
    hits = torch.zeros(nrows * w * spp, dtype=torch.int32, device="cuda")
    r = bihrt.Renderer(g, w, h, spp=spp)
    r.render_whitted_device(out.data_ptr(), frame, rows=rows, hits_ptr=hits.data_ptr())
    r.sync()
    return (out.cpu().numpy().view(np.uint32).reshape(nrows, w),
            hits.cpu().numpy().astype(np.uint8))


@pytest.mark.gpu
@pytest.mark.parametrize("scene", ["cornell", "bih1_dodeca", "clustered", "signed_zero", "one_tri",
                                   "dup_all", "torus", "soup100k"])
def test_whitted_matches_oracle(scene, gpu, bihrt_mod, oracle_mod):
    S = bihrt_mod.scenes
    tris = {"torus": S.torus, "soup100k": lambda: S.soup(100_000, seed=2)}.get(
        scene, lambda: edge_scenes()[scene])()
    g = bihrt_mod.GPUArrayManager(tris)
    ot = oracle_mod.OracleTree(tris)
    w, h = (160, 90) if scene in ("torus", "soup100k") else (64, 48)
    for frame in (0, 2):
        img, hits = _whitted_device(bihrt_mod, g, w, h, frame)
        ref, _, dep = ot.render_whitted(w, h, frame=frame, depths=True)
        assert np.array_equal(hits, dep), (scene, frame, int((hits != dep).sum()))
        assert np.array_equal(img, ref), (scene, frame)


@pytest.mark.gpu
@pytest.mark.parametrize("scene", ["torus", "soup100k"])
def test_whitted_work_counters_match_oracle(scene, gpu, bihrt_mod, oracle_mod):
    """BIH_PARAM_WHITTED_COUNTERS: the rays traced, nodes entered and
    triangles tested over all bounces equal the oracle's counters (the same
    walk step for step), with the bounce-queue ray order on; the image is the
    same as without counters."""
    S = bihrt_mod.scenes
    tris = S.torus() if scene == "torus" else S.soup(100_000, seed=2)
    g = bihrt_mod.GPUArrayManager(tris)
    ot = oracle_mod.OracleTree(tris)
    w, h = 160, 90
    g.set_param(bihrt_mod.PARAM_WHITTED_COUNTERS, 1)
    img, hits = _whitted_device(bihrt_mod, g, w, h, 1)
    r = bihrt_mod.Renderer(g, w, h)
    wk = r.whitted_work()
    ref, st, dep = ot.render_whitted(w, h, frame=1, depths=True)
    assert np.array_equal(img, ref) and np.array_equal(hits, dep)
    assert sum(wk["rays"]) == st.slab_miss          # rays traced (oracle: slab_miss field)
    assert sum(wk["nodes"]) == st.node_visits
    assert sum(wk["tris"]) == st.tri_tests
    # rays of bounce d = samples with at least d hits
    for d in range(9):
        assert wk["rays"][d] == int((dep >= d).sum()), d
    # a second frame of the same camera: the frustum bins are usable from now
    # on, and with counters on every primary sample is still walked, so the
    # counts stay the oracle's
    img2, hits2 = _whitted_device(bihrt_mod, g, w, h, 2)
    wk2 = r.whitted_work()
    ref2, st2, dep2 = ot.render_whitted(w, h, frame=2, depths=True)
    assert np.array_equal(img2, ref2) and np.array_equal(hits2, dep2)
    assert (sum(wk2["rays"]), sum(wk2["nodes"]), sum(wk2["tris"])) == (st2.slab_miss, st2.node_visits,
                                                                        st2.tri_tests)
    g.set_param(bihrt_mod.PARAM_WHITTED_COUNTERS, 0)
    img0, _ = _whitted_device(bihrt_mod, g, w, h, 1)
    assert np.array_equal(img0, ref)
    with pytest.raises(bihrt_mod.BihError):
        r.whitted_work()                               # the last render had no counters


@pytest.mark.gpu
def test_whitted_1m_512x288_matches_oracle(gpu, bihrt_mod, oracle_mod):
    """C4's scene (1M-triangle soup) at 512x288, every pixel and every
    sample's hit count against the oracle."""
    tris = bihrt_mod.scenes.soup(1_000_000, seed=1)
    g = bihrt_mod.GPUArrayManager(tris)
    ot = oracle_mod.OracleTree(tris)
    img, hits = _whitted_device(bihrt_mod, g, 512, 288, 0)
    ref, _, dep = ot.render_whitted(512, 288, depths=True)
    assert np.array_equal(hits, dep), int((hits != dep).sum())
    assert np.array_equal(img, ref)
    assert (dep >= 2).sum() > 1000 and (dep == 9).sum() > 0   # secondary rays do real work


@pytest.mark.gpu
def test_whitted_rows_and_host_entry(gpu, bihrt_mod, oracle_mod):
    """Row bands (global pixel RNG) reassemble the frame; bih_render_whitted
    (host framebuffer) equals the device render."""
    from bihrt.tiling import band_rows, rows_of_rank
    tris = bihrt_mod.scenes.torus()
    g = bihrt_mod.GPUArrayManager(tris)
    w, h = 96, 64
    full, _ = _whitted_device(bihrt_mod, g, w, h, 1)
    for rank in range(3):
        img, _ = _whitted_device(bihrt_mod, g, w, h, 1, rows=band_rows(h, 8, rank, 3))
        assert np.array_equal(img, full[rows_of_rank(h, 8, rank, 3)])
    r = bihrt_mod.Renderer(g, w, h)
    host = r.render_whitted(1)
    assert np.array_equal(host, full)


@pytest.mark.gpu
def test_whitted_4k_properties(gpu, bihrt_mod, oracle_mod):
    """Full C4 size (1M soup, 3840x2160, 4 spp): every pixel is the shade of
    its samples' hit counts, sampled rows equal the oracle, and a re-render of
    the frame is identical."""
    import torch
    tris = bihrt_mod.scenes.soup(1_000_000, seed=1)
    d = torch.from_numpy(tris).cuda()
    g = bihrt_mod.GPUArrayManager.from_device(d.data_ptr(), tris.shape[0])
    w, h = 3840, 2160
    img, hits = _whitted_device(bihrt_mod, g, w, h, 0)
    img2, _ = _whitted_device(bihrt_mod, g, w, h, 0)
    assert np.array_equal(img, img2)
    hs = hits.reshape(h, w, 4)
    assert hs.max() <= 9 and (hs == 9).any() and (hs == 0).any()
    lut = {}
    for y in range(0, h, 97):
        for x in range(0, w, 89):
            key = tuple(hs[y, x].tolist())
            if key not in lut:
                lut[key] = pixel_of(list(key))
            assert img[y, x] == lut[key]
    ot = oracle_mod.OracleTree(tris)
    # every 64th row (34 rows, 0.52 M primary samples and their bounces)
    # against the oracle, pixels and per-sample hit counts
    ref, _, dep = ot.render_whitted(w, h, rows=(0, 34, 64), depths=True)
    assert np.array_equal(img[0::64], ref), int((img[0::64] != ref).sum())
    assert np.array_equal(hs[0::64].reshape(-1), dep)


@pytest.mark.gpu
def test_whitted_frames_on_alternating_streams(gpu, bihrt_mod, oracle_mod):
    """Whitted frames issued back to back on two streams, no host wait in
    between: each call's bounce-0 mask render rewrites the tree's shared hit
    mask only after the previous call's Whitted launch has read it (ADVICE
    r5: the mask render waits on the last Whitted launch's event, and one
    lock covers both phases).  Every frame, pixels and per-sample hit counts,
    equals the oracle's."""
    import torch
    tris = bihrt_mod.scenes.soup(60_000, seed=6)
    g = bihrt_mod.GPUArrayManager(tris)
    ot = oracle_mod.OracleTree(tris)
    w, h, spp = 128, 72, 4
    r = bihrt_mod.Renderer(g, w, h, spp=spp)
    streams = [torch.cuda.Stream() for _ in range(2)]
    frames = list(range(6))
    outs = [torch.zeros(h * w, dtype=torch.int32, device="cuda") for _ in frames]
    hits = [torch.zeros(h * w * spp, dtype=torch.int32, device="cuda") for _ in frames]
    torch.cuda.synchronize()
    for k, f in enumerate(frames):
        r.render_whitted_device(outs[k].data_ptr(), f, hits_ptr=hits[k].data_ptr(),
                                stream=streams[k % 2].cuda_stream)
    torch.cuda.synchronize()
    for k, f in enumerate(frames):
        ref, _, dep = ot.render_whitted(w, h, frame=f, depths=True)
        img = outs[k].cpu().numpy().view(np.uint32).reshape(h, w)
        hs = hits[k].cpu().numpy().astype(np.uint8)
        assert np.array_equal(hs, dep), (f, int((hs != dep).sum()))
        assert np.array_equal(img, ref), (f, int((img != ref).sum()))
    g.close()
