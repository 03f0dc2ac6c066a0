"""GPU parity: the HIP builder and renderer (through the C ABI) against the
strict-IEEE oracle, bit-exact (integer/index/RGBA work and exact f32)."""
import os

import numpy as np
import pytest

from conftest import edge_scenes

pytestmark = pytest.mark.gpu

TREE_KEYS = ["morton", "tri_idx", "unique_mc", "dup_cnt", "first_idx", "leaf_parent", "clip",
             "axis", "children", "is_leaf", "parent", "lo", "hi", "scene_lo", "scene_hi"]


def _tree_equal(gpu_arrays, ot):
    for k in TREE_KEYS:
        a = gpu_arrays[k]
        b = getattr(ot, k)
        assert a.shape == b.shape, (k, a.shape, b.shape)
        # bitwise for floats (distinguishes -0/+0)
        if a.dtype == np.float32:
            assert np.array_equal(a.view(np.uint32), b.view(np.uint32)), k
        else:
            assert np.array_equal(a, b), k


SCENES = edge_scenes()


@pytest.mark.parametrize("name", sorted(SCENES))
def test_build_matches_oracle_edge(name, gpu, bihrt_mod, oracle_mod):
    tris = SCENES[name]
    g = bihrt_mod.GPUArrayManager(tris)
    ot = oracle_mod.OracleTree(tris)
    assert g.info().n_unique == ot.U
    _tree_equal(g.arrays(), ot)


@pytest.mark.parametrize("n,seed", [(1000, 11), (4097, 3), (70_000, 1), (123_457, 5), (300_000, 2),
                                    (1_000_000, 1), (10_000_000, 1)])
def test_build_matches_oracle_soup(n, seed, gpu, bihrt_mod, oracle_mod):
    """Every canonical array bit-equal, up to SURVEY 8f-1's 10M triangles
    (where the segment tree of k_seg_up takes 3 launches)."""
    tris = bihrt_mod.scenes.soup(n, seed=seed)
    g = bihrt_mod.GPUArrayManager(tris)
    ot = oracle_mod.OracleTree(tris)
    _tree_equal(g.arrays(), ot)


def test_build_skewed_codes(gpu, bihrt_mod, oracle_mod):
    """300k triangles packed into a tiny cluster plus two far corners: almost
    every code shares its top digits (one radix bucket holds nearly all keys,
    whole waves rank as one peer group) and many codes repeat (long runs)."""
    rng = np.random.default_rng(7)
    n = 300_000
    c = rng.uniform(0.0, 1e-3, size=(n, 1, 3)).astype(np.float32)
    tris = (c + rng.uniform(-1e-4, 1e-4, size=(n, 3, 3))).astype(np.float32)
    tris[0] = np.array([[-5, -5, -5], [-4.9, -5, -5], [-5, -4.9, -5]], np.float32)
    tris[n // 2] = np.array([[5, 5, 5], [4.9, 5, 5], [5, 4.9, 5]], np.float32)
    g = bihrt_mod.GPUArrayManager(tris)
    ot = oracle_mod.OracleTree(tris)
    assert g.info().n_unique == ot.U < n // 4
    _tree_equal(g.arrays(), ot)


def test_build_equals_reference_dump(gpu, bihrt_mod):
    """The HIP builder's tree of the recovered mesh is the reference's own
    dump, BIH1.txt (all 35 nodes x 8 fields)."""
    from conftest import GOLDEN, bih1_mismatches
    tris = np.load(os.path.join(GOLDEN, "bih1_dodecahedron.npy"))
    g = bihrt_mod.GPUArrayManager(tris)
    a = g.arrays()
    assert g.info().n_unique == 36
    assert bih1_mismatches(a["parent"], a["children"], a["axis"], a["is_leaf"], a["clip"]) == []


def test_build_torus(gpu, bihrt_mod, oracle_mod):
    tris = bihrt_mod.scenes.torus()
    _tree_equal(bihrt_mod.GPUArrayManager(tris).arrays(), oracle_mod.OracleTree(tris))


def test_rebuild_deterministic(gpu, bihrt_mod):
    """Rebuilds rotate through three tree buffers (asynchronous rebuilds of
    consecutive frames alternate between two build streams): each one, into
    any buffer, exports the first build's arrays byte for byte, and the two
    spare buffers are allocated once (by the first two rebuilds)."""
    tris = bihrt_mod.scenes.soup(50_000, seed=9)
    g = bihrt_mod.GPUArrayManager(tris)
    a = g.arrays()
    allocs = []
    for _ in range(5):
        g.rebuild()
        b = g.arrays()
        for k in TREE_KEYS:
            assert np.array_equal(a[k].view(np.uint8), b[k].view(np.uint8)), k
        allocs.append(g.info().device_allocs)
    assert allocs[0] < allocs[1] == allocs[2] == allocs[3] == allocs[4]


@pytest.mark.parametrize("name", ["cornell", "dodeca", "bih1_dodeca", "clustered", "signed_zero", "one_tri",
                                  "dup_all", "flat_z"])
@pytest.mark.parametrize("w,h,spp", [(64, 48, 4), (37, 29, 3)])
def test_render_matches_oracle_small(name, w, h, spp, gpu, bihrt_mod, oracle_mod):
    tris = SCENES[name]
    g = bihrt_mod.GPUArrayManager(tris)
    ot = oracle_mod.OracleTree(tris)
    r = bihrt_mod.Renderer(g, w, h, spp=spp, seed=1984)
    for frame in range(3):
        img = r.render(frame)
        ref, _ = ot.render(w, h, spp=spp, frame=frame, seed=1984)
        assert np.array_equal(img, ref), (name, frame)


def test_cornell_256_frames(gpu, bihrt_mod, oracle_mod):
    tris = bihrt_mod.scenes.cornell()
    g = bihrt_mod.GPUArrayManager(tris)
    ot = oracle_mod.OracleTree(tris)
    r = bihrt_mod.Renderer(g, 256, 256)
    # sequential frames reuse the advanced RNG state; frame 7 re-seeds with a skip-ahead
    for frame in (0, 1, 2, 7, 8):
        img = r.render(frame)
        ref, _ = ot.render(256, 256, frame=frame)
        assert np.array_equal(img, ref), frame


def test_render_rows_tile_reassembles(gpu, bihrt_mod, oracle_mod):
    tris = bihrt_mod.scenes.torus()
    g = bihrt_mod.GPUArrayManager(tris)
    r = bihrt_mod.Renderer(g, 192, 108)
    full = r.render(0)
    parts = [bihrt_mod.Renderer(g, 192, 108).render(0, rows=(y, 27)) for y in range(0, 108, 27)]
    assert np.array_equal(np.concatenate(parts, 0), full)
    ref, _ = oracle_mod.OracleTree(tris).render(192, 108)
    assert np.array_equal(full, ref)


def _device_render(bihrt, g, w, h, spp, frame, traverse, rows=None, stats=False):
    import torch
    nrows = rows.nrows if rows is not None else h
    out = torch.zeros(nrows * w, dtype=torch.int32, device="cuda")
    st = torch.zeros(3 * nrows * w * spp, dtype=torch.int32, device="cuda") if stats else None
    r = bihrt.Renderer(g, w, h, spp=spp)
    r.render_device(out.data_ptr(), frame, rows=rows, traverse=traverse,
                    stats_ptr=st.data_ptr() if stats else None)
    r.sync()
    img = out.cpu().numpy().view(np.uint32).reshape(nrows, w)
    if stats:
        s = st.cpu().numpy().view(np.uint32).reshape(-1, 3)
        return img, s
    return img


@pytest.mark.parametrize("scene", ["torus", "soup"])
def test_per_ray_counters_match_oracle(scene, gpu, bihrt_mod, oracle_mod):
    """The HIP walk visits exactly the reference's nodes and triangles
    (TRAVERSE_REFERENCE) / the oracle's any-hit prefix of them (ANYHIT)."""
    tris = bihrt_mod.scenes.torus() if scene == "torus" else bihrt_mod.scenes.soup(60_000, seed=4)
    g = bihrt_mod.GPUArrayManager(tris)
    ot = oracle_mod.OracleTree(tris)
    w, h, spp = 96, 54, 4
    # reference walk: exactly TraverseTree's node visits, leaf visits and tests
    img, s = _device_render(bihrt_mod, g, w, h, spp, 0, bihrt_mod.TRAVERSE_REFERENCE, stats=True)
    ref, _, rs = ot.render(w, h, spp=spp, mode=oracle_mod.MODE_GPU_REF, ray_stats=True)
    assert np.array_equal(img, ref)
    assert np.array_equal(s[:, 0], rs[:, 0]), "node visits differ"
    assert np.array_equal(s[:, 1], rs[:, 1]), "leaf visits differ"
    assert np.array_equal(s[:, 2], rs[:, 2]), "triangle tests differ"
    # any-hit walk: same RGBA; per ray a subset of the reference walk's work.
    # The per-lane kernels walk in TraverseTree's order, so there the counts
    # equal the oracle's any-hit prefix exactly; the packet kernel walks the
    # union of its lanes' sets in another order.
    img2, s2 = _device_render(bihrt_mod, g, w, h, spp, 0, bihrt_mod.TRAVERSE_ANYHIT, stats=True)
    ref2, _, rs2 = ot.render(w, h, spp=spp, mode=oracle_mod.MODE_GPU_ANYHIT, ray_stats=True)
    assert np.array_equal(img2, ref)
    assert np.array_equal(ref2, ref)
    assert (s2 <= s).all()
    # spp = 3 runs k_render_pixel (one lane per pixel, TraverseTree's order):
    # both walks' counters equal the oracle's exactly
    for trav, mode in ((bihrt_mod.TRAVERSE_REFERENCE, oracle_mod.MODE_GPU_REF),
                       (bihrt_mod.TRAVERSE_ANYHIT, oracle_mod.MODE_GPU_ANYHIT)):
        img3, s3 = _device_render(bihrt_mod, g, 64, 36, 3, 1, trav, stats=True)
        ref3, _, rs3 = ot.render(64, 36, spp=3, frame=1, mode=mode, ray_stats=True)
        assert np.array_equal(img3, ref3)
        assert np.array_equal(s3, rs3), ("spp 3 counters differ from the oracle's", trav)


def test_interleaved_bands(gpu, bihrt_mod, oracle_mod):
    """Row bands as bench.py's multi-GPU tiling uses them."""
    tris = bihrt_mod.scenes.soup(40_000, seed=6)
    g = bihrt_mod.GPUArrayManager(tris)
    w, h, world, B = 160, 90, 3, 8
    full = _device_render(bihrt_mod, g, w, h, 4, 0, bihrt_mod.TRAVERSE_ANYHIT)
    ref, _ = oracle_mod.OracleTree(tris).render(w, h)
    assert np.array_equal(full, ref)
    from bihrt.tiling import band_rows, rows_of_rank
    for rank in range(world):
        rows = band_rows(h, B, rank, world)
        img = _device_render(bihrt_mod, g, w, h, 4, 0, bihrt_mod.TRAVERSE_ANYHIT, rows=rows)
        ys = rows_of_rank(h, B, rank, world)
        assert np.array_equal(img, full[ys])


def test_1m_1080p_properties(gpu, bihrt_mod, oracle_mod):
    """Full BASELINE size: both traversals agree on every pixel; sampled rows
    equal the oracle; re-render of the same frame is identical."""
    tris = bihrt_mod.scenes.soup(1_000_000, seed=1)
    g = bihrt_mod.GPUArrayManager(tris)
    w, h = 1920, 1080
    a = _device_render(bihrt_mod, g, w, h, 4, 0, bihrt_mod.TRAVERSE_ANYHIT)
    b = _device_render(bihrt_mod, g, w, h, 4, 0, bihrt_mod.TRAVERSE_REFERENCE)
    assert np.array_equal(a, b)
    ot = oracle_mod.OracleTree(tris)
    # every 16th row (68 rows, 522k rays) against the oracle
    ref, _ = ot.render(w, h, rows=(0, 68, 16), mode=oracle_mod.MODE_GPU_ANYHIT)
    ys = list(range(0, h, 16))
    assert np.array_equal(a[ys], ref)
    vals = np.unique(a)
    # k of 4 samples hit -> floor((255k + 20(4-k))/4), B = 10(4-k) (CUDAKernels.cu:384-388, :420)
    assert set(vals.tolist()) <= {0x281414, 0x1e4e4e, 0x148989, 0x0ac4c4, 0x00ffff}, \
        [hex(x) for x in vals]


@pytest.mark.parametrize("fname,scene,w,h,frame", [
    ("cornell_256x256_f0.npy", "cornell", 256, 256, 0),
    ("cornell_256x256_f7.npy", "cornell", 256, 256, 7),
    ("dodeca_64x64_f0.npy", "dodeca", 64, 64, 0),
         ("bih1_dodeca_640x480_f0.npy", "bih1_dodeca", 640, 480, 0)])
def test_render_matches_golden_fixture(fname, scene, w, h, frame, gpu, bihrt_mod):
    """The committed golden framebuffers (tests/golden/make_golden.py)."""
    from conftest import GOLDEN
    ref = np.load(os.path.join(GOLDEN, fname))
    g = bihrt_mod.GPUArrayManager(SCENES[scene])
    for trav in (bihrt_mod.TRAVERSE_ANYHIT, bihrt_mod.TRAVERSE_REFERENCE):
        img = _device_render(bihrt_mod, g, w, h, 4, frame, trav)
        assert np.array_equal(img, ref), (fname, trav)


VARIANT_SCRIPT = r'''
import os, sys
import numpy as np
sys.path.insert(0, os.path.join(sys.argv[1], "bih-gpu-raytracer_amd"))
sys.path.insert(0, os.path.join(sys.argv[1], "tests"))
import torch, bihrt
from conftest import edge_scenes
out = {}
for name in ("cornell", "clustered"):
    tris = edge_scenes()[name]
    g = bihrt.GPUArrayManager(tris)
    for tname, trav in (("any", bihrt.TRAVERSE_ANYHIT), ("ref", bihrt.TRAVERSE_REFERENCE)):
        w, h, spp = 64, 48, 4
        img = torch.zeros(w * h, dtype=torch.int32, device="cuda")
        st = torch.zeros(3 * w * h * spp, dtype=torch.int32, device="cuda")
        r = bihrt.Renderer(g, w, h, spp=spp)
        r.render_device(img.data_ptr(), 0, traverse=trav, stats_ptr=st.data_ptr())
        r.sync()
        out[f"{name}_{tname}_img"] = img.cpu().numpy()
        out[f"{name}_{tname}_st"] = st.cpu().numpy()
np.savez(sys.argv[2], **out)
'''


@pytest.mark.parametrize("variant", ["packet2", "packet1"])
def test_kernel_variants_agree(variant, gpu, tmp_path):
    """Every render kernel (BIH_RENDER_KERNEL; the default is the inline-asm
    packet walk) gives the same RGBA, and the same per-ray counters for the
    reference walk, as the default kernel."""
    import subprocess
    import sys
    from conftest import ROOT
    res = {}
    for v in ("default", variant):
        env = dict(os.environ)
        if v != "default":
            env["BIH_RENDER_KERNEL"] = v
        f = tmp_path / f"{v}.npz"
        subprocess.run([sys.executable, "-c", VARIANT_SCRIPT, ROOT, str(f)], env=env, check=True,
                       timeout=300)
        res[v] = np.load(f)
    a, b = res["default"], res[variant]
    for k in a.files:
        if k.endswith("_img") or "_ref_" in k:
            assert np.array_equal(a[k], b[k]), (variant, k)


def test_rebuild_keeps_frame_sequence(gpu, bihrt_mod, oracle_mod):
    """Per-frame rebuild (as Renderer::Render does) between renders: the tree
    is rebuilt bit-identically and the RNG frame sequence continues."""
    tris = SCENES["cornell"]
    g = bihrt_mod.GPUArrayManager(tris)
    ot = oracle_mod.OracleTree(tris)
    r = bihrt_mod.Renderer(g, 96, 64)
    for frame in range(4):
        if frame:
            g.rebuild()
        img = r.render(frame)
        ref, _ = ot.render(96, 64, frame=frame)
        assert np.array_equal(img, ref), frame
    _tree_equal(g.arrays(), ot)


def test_static_soup_rebuilds_do_not_wait(gpu, bihrt_mod, oracle_mod):
    """BIH_PARAM_STATIC_SOUP: bih_rebuild returns without waiting for the
    build, so rebuilds and renders on three streams overlap (the bench's
    with_rebuild leg).  Every frame still equals the oracle's, the tree
    exports the first build's arrays, and build_ms is the last build's device
    time (read from its events)."""
    import torch
    tris = bihrt_mod.scenes.soup(50_000, seed=21)
    d = torch.from_numpy(tris.copy()).cuda()
    g = bihrt_mod.GPUArrayManager.from_device(d.data_ptr(), tris.shape[0])
    with pytest.raises(bihrt_mod.BihError):
        g.set_param(bihrt_mod.PARAM_STATIC_SOUP, 2)
    g.set_param(bihrt_mod.PARAM_STATIC_SOUP, 1)
    a = g.arrays()
    w, h = 160, 90
    r = bihrt_mod.Renderer(g, w, h)
    streams = [torch.cuda.Stream() for _ in range(3)]
    outs = [torch.zeros(h * w, dtype=torch.int32, device="cuda") for _ in range(6)]
    for f in range(6):
        g.rebuild()
        r.render_device(outs[f].data_ptr(), f, stream=streams[f % 3].cuda_stream)
    torch.cuda.synchronize()
    assert g.info().build_ms > 0.0
    ot = oracle_mod.OracleTree(tris)
    for f in range(6):
        ref, _ = ot.render(w, h, frame=f)
        assert np.array_equal(outs[f].cpu().numpy().view(np.uint32).reshape(h, w), ref), f
    b = g.arrays()
    for k in TREE_KEYS:
        assert np.array_equal(a[k].view(np.uint8), b[k].view(np.uint8)), k


def test_rebuild_of_changed_soup_rebuilds_camera_state(gpu, bihrt_mod, oracle_mod):
    """A rebuild keeps the per-camera structures (records, frustum bins, tile
    queues) only when the soup's content hash is unchanged: moving the
    device-resident soup in place between rebuilds (an animated scene, as the
    reference's per-frame rebuild allows) renders the moved geometry, and an
    unchanged rebuild renders the same frame as before (any-hit through the
    bins and the reference walk)."""
    import torch
    tris = bihrt_mod.scenes.soup(50_000, seed=13)
    d = torch.from_numpy(tris.copy()).cuda()
    g = bihrt_mod.GPUArrayManager.from_device(d.data_ptr(), tris.shape[0])
    w, h = 160, 90
    for step in range(4):
        if step:
            if step % 2:
                d[:, 1::3] += 0.05          # move every vertex in y, in place
                tris[:, 1::3] += np.float32(0.05)
                torch.cuda.synchronize()
            g.rebuild()
        ot = oracle_mod.OracleTree(tris)
        for trav in (bihrt_mod.TRAVERSE_ANYHIT, bihrt_mod.TRAVERSE_REFERENCE):
            img = _device_render(bihrt_mod, g, w, h, 4, step, trav)
            ref, _ = ot.render(w, h, frame=step)
            assert np.array_equal(img, ref), (step, trav)


@pytest.mark.gpu
def test_frame_gaps_match_oracle(gpu, bihrt_mod, oracle_mod):
    """Frames rendered out of sequence (the weak-scaling schedule: rank r
    renders r, r+N, ...): short forward gaps advance the stored generators,
    long or backward gaps re-seed; every frame equals the oracle's."""
    tris = SCENES["cornell"]
    g = bihrt_mod.GPUArrayManager(tris)
    ot = oracle_mod.OracleTree(tris)
    r = bihrt_mod.Renderer(g, 80, 48)
    for frame in (0, 3, 11, 12, 600, 2, 9):
        img = r.render(frame)
        ref, _ = ot.render(80, 48, frame=frame)
        assert np.array_equal(img, ref), frame


@pytest.mark.gpu
@pytest.mark.parametrize("nstreams", [2, 3, 4])
def test_frames_in_flight_on_streams(nstreams, gpu, bihrt_mod, oracle_mod):
    """Consecutive frames issued on 2-4 streams overlap on the GPU (the
    library orders only what they share: tile queues, spill areas, the RNG
    ring); a gap, a rebuild and a 1M-scale frame mid-sequence keep every frame
    equal to the oracle's."""
    import torch
    tris = bihrt_mod.scenes.soup(20_000, seed=9)
    g = bihrt_mod.GPUArrayManager(tris)
    ot = oracle_mod.OracleTree(tris)
    w, h = 160, 96
    r = bihrt_mod.Renderer(g, w, h)
    streams = [torch.cuda.Stream() for _ in range(nstreams)]
    frames = [0, 1, 2, 3, 7, 8, 9, 30, 31, 2, 3]
    outs = [torch.zeros(h * w, dtype=torch.int32, device="cuda") for _ in frames]
    for k, f in enumerate(frames):
        if k == 6:
            g.rebuild()
        r.render_device(outs[k].data_ptr(), f, stream=streams[k % nstreams].cuda_stream)
    torch.cuda.synchronize()
    for k, f in enumerate(frames):
        ref, _ = ot.render(w, h, frame=f)
        assert np.array_equal(outs[k].cpu().numpy().view(np.uint32).reshape(h, w), ref), (k, f)


@pytest.mark.gpu
def test_rng_ring_long_sequence_in_flight(gpu, bihrt_mod, oracle_mod):
    """Twenty consecutive frames on three streams cycle the XORWOW ring
    (kSlots + 1 buffers, one advance per frame) five times; a jump back and
    one far ahead re-seed.  Every frame equals the oracle's."""
    import torch
    tris = bihrt_mod.scenes.soup(20_000, seed=5)
    g = bihrt_mod.GPUArrayManager(tris)
    ot = oracle_mod.OracleTree(tris)
    w, h = 96, 64
    r = bihrt_mod.Renderer(g, w, h)
    streams = [torch.cuda.Stream() for _ in range(3)]
    frames = list(range(20)) + [12, 13, 700, 701]
    outs = [torch.zeros(h * w, dtype=torch.int32, device="cuda") for _ in frames]
    for k, f in enumerate(frames):
        r.render_device(outs[k].data_ptr(), f, stream=streams[k % 3].cuda_stream)
    torch.cuda.synchronize()
    refs = {}
    for k, f in enumerate(frames):
        if f not in refs:
            refs[f] = ot.render(w, h, frame=f)[0]
        assert np.array_equal(outs[k].cpu().numpy().view(np.uint32).reshape(h, w), refs[f]), (k, f)


def _grazing_scene(n, seed):
    """Triangles seen almost edge-on: the view ray through each triangle's
    centre meets its plane at an angle of 1e-4 .. 0.3 rad, so det of the
    rays that cross it sits near the 1e-6 threshold, where the intersector's
    rounding is at its worst (the miss-proof boxes' error bound)."""
    rng = np.random.default_rng(seed)
    O = np.array([2.0, 0.0, -2.0])
    P = np.stack([rng.uniform(0.0, 2.6667, n), rng.uniform(-1, 1, n), rng.uniform(0, 2, n)], 1)
    d = P - O
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    side = np.cross(d, rng.normal(size=(n, 3)))
    side /= np.linalg.norm(side, axis=1, keepdims=True)
    normal = np.cross(d, side)
    th = 10.0 ** rng.uniform(-4, -0.5, n)[:, None]
    wdir = np.cos(th) * d + np.sin(th) * normal
    size = rng.uniform(0.01, 0.06, (n, 1))
    v0 = P - 0.5 * size * (wdir + side)
    v1 = v0 + size * wdir
    v2 = v0 + size * side
    flip = rng.random(n) < 0.5
    v1[flip], v2[flip] = v2[flip].copy(), v1[flip].copy()
    return np.concatenate([v0, v1, v2], 1).astype(np.float32)


@pytest.mark.parametrize("scene", ["soup200k", "grazing", "grazing_dense", "torus", "clustered",
                                   "cornell", "signed_zero", "flat_z"])
def test_anyhit_shortcut_matches_exact_walk(scene, gpu, bihrt_mod):
    """The any-hit shortcut passes (tight-box hit + root-path check, and the
    miss-proof boxes) against the exact BIH walk of the same kernel family,
    every pixel of several frames: the reference traversal
    (TRAVERSE_REFERENCE) never takes a shortcut."""
    S = bihrt_mod.scenes
    tris = {"soup200k": lambda: S.soup(200_000, seed=11),
            "grazing": lambda: _grazing_scene(20_000, 1),
            "grazing_dense": lambda: np.concatenate([_grazing_scene(60_000, 2),
                                                     S.soup(60_000, seed=12)]),
            "torus": S.torus}.get(scene, lambda: SCENES[scene])()
    g = bihrt_mod.GPUArrayManager(tris)
    w, h = 480, 270
    for frame in (0, 3):
        a = _device_render(bihrt_mod, g, w, h, 4, frame, bihrt_mod.TRAVERSE_ANYHIT)
        b = _device_render(bihrt_mod, g, w, h, 4, frame, bihrt_mod.TRAVERSE_REFERENCE)
        assert np.array_equal(a, b), (scene, frame, int((a != b).sum()))


@pytest.mark.parametrize("scene", ["soup200k", "grazing_dense", "cornell"])
def test_bins_fallback_matches_exact_walk(scene, gpu, bihrt_mod, monkeypatch):
    """k_render_fallback (the exact walk for packets the frustum-bin kernel
    leaves undecided) on every live packet: PARAM_FORCE_FALLBACK sends
    each one there; every pixel equals the exact walk's, on one stream and
    with frames in flight on three."""
    import torch
    S = bihrt_mod.scenes
    tris = {"soup200k": lambda: S.soup(200_000, seed=11),
            "grazing_dense": lambda: np.concatenate([_grazing_scene(60_000, 2),
                                                     S.soup(60_000, seed=12)])}.get(
        scene, lambda: SCENES[scene])()
    g = bihrt_mod.GPUArrayManager(tris)
    w, h = 480, 270
    ref = [_device_render(bihrt_mod, g, w, h, 4, f, bihrt_mod.TRAVERSE_REFERENCE) for f in range(4)]
    g.set_param(bihrt_mod.PARAM_FORCE_FALLBACK, 1)
    for f in (0, 3):
        a = _device_render(bihrt_mod, g, w, h, 4, f, bihrt_mod.TRAVERSE_ANYHIT)
        assert np.array_equal(a, ref[f]), (scene, f, int((a != ref[f]).sum()))
    r = bihrt_mod.Renderer(g, w, h)
    streams = [torch.cuda.Stream() for _ in range(3)]
    outs = [torch.full((h * w,), -1, dtype=torch.int32, device="cuda") for _ in range(4)]
    for f in range(4):
        r.render_device(outs[f].data_ptr(), f, stream=streams[f % 3].cuda_stream)
    torch.cuda.synchronize()
    for f in range(4):
        a = outs[f].cpu().numpy().view(np.uint32).reshape(h, w)
        assert np.array_equal(a, ref[f]), (scene, "in flight", f, int((a != ref[f]).sum()))


@pytest.mark.parametrize("cap", ["0", "5000"])
def test_pair_results_past_buffer_recompute(cap, gpu, bihrt_mod, monkeypatch):
    """k_bin_fill takes each (triangle, tile) pair's class, pixel mask and
    bucket from k_bin_count's pair buffer; count blocks past the buffer
    (PARAM_PAIR_CAP caps it: 0 = every block, 5000 = most) leave them to be
    computed again by the fill.  Every frame equals the reference walk's."""
    tris = bihrt_mod.scenes.soup(200_000, seed=11)
    g = bihrt_mod.GPUArrayManager(tris)
    g.set_param(bihrt_mod.PARAM_PAIR_CAP, int(cap))
    w, h = 480, 270
    for f in (0, 2):
        a = _device_render(bihrt_mod, g, w, h, 4, f, bihrt_mod.TRAVERSE_ANYHIT)
        b = _device_render(bihrt_mod, g, w, h, 4, f, bihrt_mod.TRAVERSE_REFERENCE)
        assert np.array_equal(a, b), (cap, f, int((a != b).sum()))
    assert g.bins_stats().usable


def test_c2_torus_1080p(gpu, bihrt_mod, oracle_mod):
    """Config C2's size with its stand-in mesh (the 69,432-triangle torus;
    the Stanford bunny is not available offline): 1920x1080 x 4 spp, the
    any-hit render (frustum bins) equals the reference walk on two frames and
    the oracle on every 16th row of frame 0."""
    tris = bihrt_mod.scenes.torus()
    g = bihrt_mod.GPUArrayManager(tris)
    w, h = 1920, 1080
    imgs = []
    for f in (0, 1):
        a = _device_render(bihrt_mod, g, w, h, 4, f, bihrt_mod.TRAVERSE_ANYHIT)
        b = _device_render(bihrt_mod, g, w, h, 4, f, bihrt_mod.TRAVERSE_REFERENCE)
        assert np.array_equal(a, b), (f, int((a != b).sum()))
        imgs.append(a)
    assert g.bins_stats().usable
    ref, _ = oracle_mod.OracleTree(tris).render(w, h, rows=(0, (h + 15) // 16, 16))
    assert np.array_equal(imgs[0][::16], ref)
    assert (imgs[0] != imgs[0][0, 0]).any()   # the torus is in view


def test_c2_torus_calls_of_16_frames(gpu, bihrt_mod, oracle_mod):
    """Config C2's call shape: the torus's ~7.3k live tiles make
    k_render_bins split each tile's 16 frames into items of 8 itself
    (RenderArgs::live_items, from the queue's live count), and from the
    second call on (measured tile costs) split its heavy tiles further.
    Three calls of 16 frames: frames 0, 15, 16, 31 and 47 equal the reference
    walk's one-frame renders of the same indices, frame 47 the oracle on every
    16th row."""
    import torch
    tris = bihrt_mod.scenes.torus()
    g = bihrt_mod.GPUArrayManager(tris)
    w, h = 1920, 1080
    P = w * h
    r = bihrt_mod.Renderer(g, w, h)
    out = torch.full((16 * P,), -1, dtype=torch.int32, device="cuda")
    got = {}
    for c in range(3):
        r.render_device_frames(out.data_ptr(), 16 * c, 16, P)
        r.sync()
        o = out.cpu().numpy().view(np.uint32).reshape(16, h, w)
        for j in (0, 15):
            got[16 * c + j] = o[j].copy()
    for f in (0, 15, 16, 31, 47):
        ref = _device_render(bihrt_mod, g, w, h, 4, f, bihrt_mod.TRAVERSE_REFERENCE)
        assert np.array_equal(got[f], ref), (f, int((got[f] != ref).sum()))
    oref, _ = oracle_mod.OracleTree(tris).render(w, h, frame=47, rows=(0, (h + 15) // 16, 16))
    assert np.array_equal(got[47][::16], oref)


def test_bins_list_total_past_u32_renders_without_bins(gpu, bihrt_mod):
    """33,500 front-facing triangles that each cover the whole 1080p image:
    the frustum-bin lists would hold 33,500 x 129,600 > 2^32 entries.  The
    64-bit list total (k_bin_count) makes the camera render without bins (the
    BIH walk with its proven shortcuts) instead of wrapping the u32 offsets;
    rows rendered that way equal the reference walk's."""
    from bihrt.tiling import band_rows
    w, h = 1920, 1080
    cam = np.array(bihrt_mod.camera_reference(w, h).as_list(), np.float32)
    O, llc, hh, vv = cam[0:3], cam[3:6], cam[6:9], cam[9:12]
    n = 33_500
    d = (1.2 + 1e-5 * np.arange(n, dtype=np.float64))[:, None]

    def P(u, v):
        return O[None, :] + d * ((llc + u * hh + v * vv) - O)[None, :]

    tris = np.concatenate([P(-20, -20), P(-20, 40), P(40, -20)], 1).astype(np.float32)   # front-facing
    g = bihrt_mod.GPUArrayManager(tris)
    rows = band_rows(h, 4, 67, 270)          # rows 268..271
    a = _device_render(bihrt_mod, g, w, h, 4, 0, bihrt_mod.TRAVERSE_ANYHIT, rows=rows)
    st = g.bins_stats()
    assert not st.usable, (st.usable, st.list_entries)
    b = _device_render(bihrt_mod, g, w, h, 4, 0, bihrt_mod.TRAVERSE_REFERENCE, rows=rows)
    assert np.array_equal(a, b)
    assert (a == 0x00FFFF).all()             # every sample hits


def test_10m_4k_shortcut_equals_exact_walk(gpu, bihrt_mod, oracle_mod):
    """Config C5's scene and size on one GPU (10M-triangle soup, 3840x2160,
    4 spp): the any-hit shortcut and the exact walk agree on every pixel of
    two frames; every pixel is one of the five shades."""
    import torch
    tris = bihrt_mod.scenes.soup(10_000_000, seed=1)
    d = torch.from_numpy(tris).cuda()
    g = bihrt_mod.GPUArrayManager.from_device(d.data_ptr(), tris.shape[0])
    w, h = 3840, 2160
    ot = oracle_mod.OracleTree(tris)
    for frame in (0, 5):
        a = _device_render(bihrt_mod, g, w, h, 4, frame, bihrt_mod.TRAVERSE_ANYHIT)
        b = _device_render(bihrt_mod, g, w, h, 4, frame, bihrt_mod.TRAVERSE_REFERENCE)
        assert np.array_equal(a, b), (frame, int((a != b).sum()))
        # against the oracle: frame 0 every 16th row (135 rows, 2.1 M rays),
        # frame 5 six rows spread over the frame
        if frame == 0:
            ref, _ = ot.render(w, h, frame=frame, rows=(0, 135, 16), mode=oracle_mod.MODE_GPU_ANYHIT)
            assert np.array_equal(a[0::16], ref), (frame, int((a[0::16] != ref).sum()))
        else:
            ref, _ = ot.render(w, h, frame=frame, rows=(137, 6, 353), mode=oracle_mod.MODE_GPU_ANYHIT)
            assert np.array_equal(a[[137 + 353 * k for k in range(6)]], ref), frame
    assert set(np.unique(a).tolist()) <= {0x281414, 0x1e4e4e, 0x148989, 0x0ac4c4, 0x00ffff}


def _moved_camera(bihrt, w, h, dx, dy, dz):
    c = bihrt.camera_reference(w, h).as_list()
    for k, d in enumerate((dx, dy, dz)):
        c[k] += d
        c[3 + k] += d
    return bihrt.Camera.from_list(c)


@pytest.mark.parametrize("nstreams,order", [(3, "cycle3"), (3, "alternate2"), (2, "every_frame")])
def test_camera_change_mid_sequence_on_streams(nstreams, order, gpu, bihrt_mod):
    """Frames in flight on several streams while the camera changes (and the
    tree is rebuilt) mid-sequence on a 1M-triangle soup, where rebuilding the
    per-camera records takes long enough to race a render issued on another
    stream: every frame equals the same frame rendered alone on one stream.
    The library keeps two sets of per-camera structures (bih_capi.cpp
    CamSet): a new camera builds into the set the latest render does not
    read; "alternate2" returns to a camera whose set is still valid, and
    "every_frame" moves the camera on every frame."""
    import torch
    tris = bihrt_mod.scenes.soup(1_000_000, seed=1)
    w, h = 320, 180
    cams = [bihrt_mod.camera_reference(w, h), _moved_camera(bihrt_mod, w, h, 0.05, -0.03, 0.2),
            _moved_camera(bihrt_mod, w, h, -0.3, 0.1, -0.1)]
    if order == "cycle3":
        seq = [(0, 0), (1, 0), (2, 1), (3, 1), (4, 2), (5, 0), (6, 2), (7, 2), (8, 1), (9, 1),
               (10, 0), (11, 0)]
    elif order == "alternate2":
        seq = [(f, f % 2) for f in range(12)]
    else:
        seq = [(f, (f * 2) % 3) for f in range(12)]
    rebuild_at = 7

    def run(multi):
        g = bihrt_mod.GPUArrayManager(tris)
        r = bihrt_mod.Renderer(g, w, h)
        streams = [torch.cuda.Stream() for _ in range(nstreams)]
        outs = [torch.full((h * w,), -1, dtype=torch.int32, device="cuda") for _ in seq]
        for k, (f, c) in enumerate(seq):
            if k == rebuild_at:
                g.rebuild()
            r.camera = cams[c]
            if multi:
                r.render_device(outs[k].data_ptr(), f, stream=streams[k % nstreams].cuda_stream)
            else:
                r.render_device(outs[k].data_ptr(), f)
                r.sync()
        torch.cuda.synchronize()
        res = [o.cpu().numpy().view(np.uint32).reshape(h, w) for o in outs]
        g.close()
        return res

    alone = run(False)
    overlapped = run(True)
    for k in range(len(seq)):
        assert np.array_equal(alone[k], overlapped[k]), (k, seq[k], int((alone[k] != overlapped[k]).sum()))
    # the cameras see different images (the check has teeth)
    assert not np.array_equal(alone[0], alone[2])


def test_bins_without_sync_overflow_falls_back(gpu, bihrt_mod, monkeypatch):
    """Camera changes build the frustum bins without a host round trip into
    the list buffer of an earlier camera (bih_capi.cpp build_bins): when the
    lists do not fit (PARAM_BINS_CAP forces it) the device status word sends
    every live packet to the exact walk, the host notices afterwards
    (resolve_bins) and the next render rebuilds a sized list.  Every frame
    equals the reference walk's."""
    import torch
    tris = bihrt_mod.scenes.soup(1_000_000, seed=1)
    w, h = 640, 360
    g = bihrt_mod.GPUArrayManager(tris)
    r = bihrt_mod.Renderer(g, w, h)
    cams = [bihrt_mod.camera_reference(w, h), _moved_camera(bihrt_mod, w, h, 0.05, -0.03, 0.2),
            _moved_camera(bihrt_mod, w, h, -0.3, 0.1, -0.1), _moved_camera(bihrt_mod, w, h, 0.1, 0.05, 0.1)]
    # (frame, camera, forced list capacity or None, bins usable after the frame);
    # the library keeps up to three sets of per-camera structures (CamSet),
    # and a set's first build sizes its list with a round trip: three
    # cameras warm every set first, then the forced capacity acts
    plan = [(0, 0, None, True), (1, 1, None, True), (2, 2, None, True), (3, 3, "1000", False),
            (4, 3, None, True), (5, 0, "1000", False), (6, 0, None, True), (7, 1, None, True)]
    out = torch.zeros(h * w, dtype=torch.int32, device="cuda")
    for f, c, cap, usable in plan:
        g.set_param(bihrt_mod.PARAM_BINS_CAP, 0 if cap is None else int(cap))
        r.camera = cams[c]
        out.fill_(-1)
        r.render_device(out.data_ptr(), f)
        r.sync()
        a = out.cpu().numpy().view(np.uint32).reshape(h, w).copy()
        st = g.bins_stats()
        assert bool(st.usable) == usable, (f, c, cap, st.usable, st.list_entries)
        assert st.list_entries > 1000, (f, st.list_entries)
        out.fill_(-1)
        r.render_device(out.data_ptr(), f, traverse=bihrt_mod.TRAVERSE_REFERENCE)
        r.sync()
        b = out.cpu().numpy().view(np.uint32).reshape(h, w)
        assert np.array_equal(a, b), (f, c, cap, int((a != b).sum()))
    g.close()


@pytest.mark.parametrize("case", ["bins", "bins_items_all_frames", "bins_items_3_frames", "bands",
                                  "bands_items_all_frames", "force_fallback", "spp3_per_frame"])
def test_render_device_frames_equals_single_frames(case, gpu, bihrt_mod, oracle_mod, monkeypatch):
    """bih_render_device_frames: nframes consecutive frames in one call
    (one launch of each kernel through the frustum bins; frame j's jitter
    2*spp*j draws past the launch's RNG state) equal the frames rendered one
    by one, then the frame sequence continues; through the exact-walk
    fallback (every packet undecided) and the per-frame path (spp 3: no bins)
    as well."""
    import torch
    from bihrt.tiling import band_rows
    S = bihrt_mod.scenes
    tris = S.soup(200_000, seed=11)
    g = bihrt_mod.GPUArrayManager(tris)
    w, h = 480, 270
    spp = 3 if case == "spp3_per_frame" else 4
    rows = band_rows(h, 8, 1, 3) if case.startswith("bands") else None
    nrows = rows.nrows if rows is not None else h
    if case == "force_fallback":
        g.set_param(bihrt_mod.PARAM_FORCE_FALLBACK, 1)
    # frames per k_render_bins item (PARAM_ITEM_TILES, bih_capi.cpp
    # item_split): the default splits this small image's 5 frames into 5 items
    # per tile; 1 puts all 5 in one item, 16320 (about 2x the tiles) 3 + 2
    if case.endswith("items_all_frames"):
        g.set_param(bihrt_mod.PARAM_ITEM_TILES, 1)
    elif case.endswith("items_3_frames"):
        g.set_param(bihrt_mod.PARAM_ITEM_TILES, 16320)
    r = bihrt_mod.Renderer(g, w, h, spp=spp)
    ref = []
    for f in range(7):
        o = torch.zeros(nrows * w, dtype=torch.int32, device="cuda")
        r.render_device(o.data_ptr(), f, rows=rows)
        r.sync()
        ref.append(o.cpu().numpy().view(np.uint32))
    stride = nrows * w + 64
    buf = torch.full((6 * stride,), -1, dtype=torch.int32, device="cuda")
    r.render_device_frames(buf.data_ptr(), 0, 5, stride, rows=rows)
    o6 = torch.zeros(nrows * w, dtype=torch.int32, device="cuda")
    r.render_device(o6.data_ptr(), 5, rows=rows)          # the sequence continues
    r.render_device_frames(buf.data_ptr() + 4 * 5 * stride, 6, 1, stride, rows=rows)
    r.sync()
    b = buf.cpu().numpy().view(np.uint32)
    for f in range(5):
        assert np.array_equal(b[f * stride: f * stride + nrows * w], ref[f]), (case, f)
        assert (b[f * stride + nrows * w: (f + 1) * stride] == 0xFFFFFFFF).all()   # stride gap untouched
    assert np.array_equal(o6.cpu().numpy().view(np.uint32), ref[5])
    assert np.array_equal(b[5 * stride: 5 * stride + nrows * w], ref[6])
    if rows is None and spp == 4:
        img, _ = oracle_mod.OracleTree(tris).render(w, h, frame=3)
        assert np.array_equal(b[3 * stride: 3 * stride + h * w].reshape(h, w), img)


@pytest.fixture(scope="module")
def soup1m(bihrt_mod, oracle_mod):
    tris = bihrt_mod.scenes.soup(1_000_000, seed=1)
    return tris, oracle_mod.OracleTree(tris)


@pytest.mark.parametrize("layout", ["frame", "bands_rank3_of8"])
def test_headline_call_shape_equals_oracle(layout, gpu, bihrt_mod, oracle_mod, soup1m):
    """The bench's own call: bih_render_device_frames with 16 frames on the 1M
    soup at 1920x1080 (one k_render_bins launch; per-lane XORWOW state kept in
    LDS across the frames of an item).  Frames 0 and 15 equal the oracle on
    every row, frame 7 on every 16th row; the state then
    carries into the next call (frames 16 and 31, every 16th row) (cudaRender's
    persistent curandState, CUDAKernels.cu:411-419; the frame loop of
    App.cpp:174-186).  `bands_rank3_of8`: rank 3's interleaved 8-row bands of
    an 8-GPU split (few tiles: the item's frames are split, start states from
    k_rng_advance)."""
    import torch
    from bihrt.tiling import band_rows, rows_of_rank
    tris, ot = soup1m
    w, h, G = 1920, 1080, 16
    d = torch.from_numpy(tris).cuda()
    g = bihrt_mod.GPUArrayManager.from_device(d.data_ptr(), tris.shape[0])
    rows = band_rows(h, 8, 3, 8) if layout.startswith("bands") else band_rows(h, 8, 0, 1)
    ys = rows_of_rank(h, 8, 3, 8) if layout.startswith("bands") else np.arange(h)
    r = bihrt_mod.Renderer(g, w, h)
    g.reserve(w, h, 4, rows, G)
    stride = rows.nrows * w
    buf = torch.full((2 * G * stride,), -1, dtype=torch.int32, device="cuda")
    r.render_device_frames(buf.data_ptr(), 0, G, stride, rows=rows)
    r.render_device_frames(buf.data_ptr() + 4 * G * stride, G, G, stride, rows=rows)   # frames 16..31
    r.sync()
    fr = buf.cpu().numpy().view(np.uint32).reshape(2 * G, rows.nrows, w)
    assert g.bins_stats().usable
    # frames 0 and 15 (the first and last of the call): every row against the
    # oracle (full frame: 8.3 M rays each, ~2 s of the oracle on the box's
    # 16 host threads); frames 7, 16 and 31: every 16th local row
    for f in (0, 7, 15, 16, 31):
        pick = np.arange(ys.size) if f in (0, 15) else np.arange(0, ys.size, 16)
        if layout.startswith("bands"):
            ref = np.concatenate([ot.render(w, h, frame=f, rows=(int(y0), 8, 1), mode=oracle_mod.MODE_GPU_ANYHIT,
                                            threads=0)[0] for y0 in ys[pick][::8]]) if f in (0, 15) else \
                np.stack([ot.render(w, h, frame=f, rows=(int(y), 1, 1), mode=oracle_mod.MODE_GPU_ANYHIT,
                                    threads=0)[0][0] for y in ys[pick]])
        elif f in (0, 15):
            ref, _ = ot.render(w, h, frame=f, mode=oracle_mod.MODE_GPU_ANYHIT, threads=0)
        else:
            ref, _ = ot.render(w, h, frame=f, rows=(0, len(pick), 16), mode=oracle_mod.MODE_GPU_ANYHIT, threads=0)
        assert ref.shape == fr[f][pick].shape, (ref.shape, fr[f][pick].shape)
        assert np.array_equal(fr[f][pick], ref), (layout, f, int((fr[f][pick] != ref).sum()))
    assert not np.array_equal(fr[0], fr[15])           # the jitter moves between frames


def test_steady_frame_loop_allocates_nothing(gpu, bihrt_mod):
    """After bih_reserve and one call per camera, a frame loop of 16- and
    4-frame calls on three streams (the bench's headline shape), then calls
    of 1 to 16 frames on one stream (the stamped XORWOW state), make no
    device allocation (bih_tree_info.device_allocs stays put)."""
    import torch
    tris = bihrt_mod.scenes.soup(200_000, seed=3)
    w, h, G = 960, 540, 16
    g = bihrt_mod.GPUArrayManager(tris)
    g.reserve(w, h, 4, None, G)
    r = bihrt_mod.Renderer(g, w, h)
    streams = [torch.cuda.Stream() for _ in range(3)]
    outs = [torch.zeros(G * h * w, dtype=torch.int32, device="cuda") for _ in range(3)]
    r.render_device_frames(outs[0].data_ptr(), 0, 5, h * w, stream=streams[0].cuda_stream)   # camera structures
    torch.cuda.synchronize()
    a0 = g.info().device_allocs
    f = 5
    for k, m in enumerate([16, 4, 16, 16, 4, 1, 16]):
        r.render_device_frames(outs[k % 3].data_ptr(), f, m, h * w, stream=streams[k % 3].cuda_stream)
        f += m
    torch.cuda.synchronize()
    assert g.info().device_allocs == a0
    # one stream: the stamped state (reserved too), through a k_rng_sync
    for m in [1, 1, 1, 16, 1, 16, 16, 16, 4, 1]:
        if m == 1:
            r.render_device(outs[0].data_ptr(), f, stream=streams[0].cuda_stream)
        else:
            r.render_device_frames(outs[0].data_ptr(), f, m, h * w, stream=streams[0].cuda_stream)
        f += m
    torch.cuda.synchronize()
    assert g.info().device_allocs == a0
    # without the reservation the first 16-frame call grows the per-call buffers
    g2 = bihrt_mod.GPUArrayManager(tris)
    r2 = bihrt_mod.Renderer(g2, w, h)
    r2.render_device_frames(outs[0].data_ptr(), 0, 5, h * w)
    r2.sync()
    b0 = g2.info().device_allocs
    r2.render_device_frames(outs[1].data_ptr(), 5, 16, h * w)
    r2.sync()
    assert g2.info().device_allocs > b0


def test_reserved_share_calls_of_every_length_allocate_nothing(gpu, bihrt_mod):
    """A rank's share of an 8-way band split has few tiles, so a call's items
    are split over its frames, and the split count is not monotone in the
    frame count (item_split).  bih_reserve(max_frames=16) sizes what calls of
    every length 1..16 need -- the XORWOW ring, the tile queues of every camera
    set, the fallback records (one per packet and frame) and the stamps: no
    allocation in the loop, on one stream (stamped state) or alternating two
    (the ring)."""
    import torch
    from bihrt.tiling import band_rows
    tris = bihrt_mod.scenes.soup(100_000, seed=5)
    w, h, G = 1920, 1080, 16
    rows = band_rows(h, 8, 3, 8)
    g = bihrt_mod.GPUArrayManager(tris)
    g.reserve(w, h, 4, rows, G)
    r = bihrt_mod.Renderer(g, w, h)
    out = torch.zeros(G * rows.nrows * w, dtype=torch.int32, device="cuda")
    r.render_device_frames(out.data_ptr(), 0, 2, rows.nrows * w, rows=rows)   # camera structures
    r.sync()
    a0 = g.info().device_allocs
    f = 2
    for m in [3, 5, 7, 1, 9, 11, 13, 16, 6, 2]:
        r.render_device_frames(out.data_ptr(), f, m, rows.nrows * w, rows=rows)
        f += m
    r.sync()
    assert g.info().device_allocs == a0
    streams = [torch.cuda.Stream() for _ in range(2)]
    torch.cuda.synchronize()
    for k, m in enumerate([16, 4, 1, 16, 7, 2]):
        r.render_device_frames(out.data_ptr(), f, m, rows.nrows * w, rows=rows, stream=streams[k % 2].cuda_stream)
        f += m
    torch.cuda.synchronize()
    assert g.info().device_allocs == a0


def test_failed_back_tree_allocation_leaves_tree_usable(gpu, bihrt_mod, oracle_mod):
    """The first bih_rebuild allocates the second tree buffer; when that
    allocation fails part-way (BIH_PARAM_TEST_ALLOC_FAIL) the rebuild reports
    BIH_ERR_OOM, the partial buffers are freed, and the following rebuilds
    (the first in place, the next into a freshly allocated buffer) and renders
    are exact (a half-allocated buffer would be read through null pointers)."""
    tris = bihrt_mod.scenes.soup(20_000, seed=9)
    w, h = 128, 96
    ot = oracle_mod.OracleTree(tris)
    for k in (1, 5, 24):   # fail at the header, in the middle, at the last buffer
        g = bihrt_mod.GPUArrayManager(tris)
        r = bihrt_mod.Renderer(g, w, h)
        g.set_param(bihrt_mod.PARAM_TEST_ALLOC_FAIL, k)
        with pytest.raises(bihrt_mod.BihError) as ei:
            g.rebuild()
        assert ei.value.code == -4, ei.value          # BIH_ERR_OOM
        g.rebuild()
        g.rebuild()
        for f in range(2):
            img = r.render(f)
            ref, _ = ot.render(w, h, frame=f)
            assert np.array_equal(img, ref), (k, f)
        g.close()


@pytest.mark.gpu
def test_stamped_state_panning_sequence_matches_oracle(gpu, bihrt_mod, oracle_mod):
    """Frustum-bin launches on one stream keep each tile's XORWOW state with
    a stamp (bih_capi.cpp stamped mode): a tile no triangle covers is not
    stepped and catches up when it turns live, every 64 frames all tiles are
    brought level (k_rng_sync), and a render of another kind takes the state
    back into the ring.  A small object crosses the view over 160 frames in
    calls of 1 .. 16 frames, so tiles turn live after long background runs;
    sampled frames equal the oracle's, then a Whitted frame, a jump back and
    a frame after it continue the sequence."""
    import torch
    S = bihrt_mod.scenes
    tris = S.soup(20_000, seed=3).copy()
    v = tris.reshape(-1, 3)
    v[:] = 0.25 * (v - v.mean(0)) + v.mean(0)     # the object covers a small part of the view
    g = bihrt_mod.GPUArrayManager(tris)
    ot = oracle_mod.OracleTree(tris)
    w, h = 96, 64
    r = bihrt_mod.Renderer(g, w, h)
    sizes = [1, 16, 3, 1, 8, 16, 2, 1, 16, 5]
    stride = h * w
    shapes, frame = [], 0
    while frame < 160:
        n = min(sizes[len(shapes) % len(sizes)], 160 - frame)
        shapes.append((frame, n))
        frame += n
    # (filled before any render: the library's stream does not order after
    # torch's default stream)
    bufs = [torch.full((n * stride,), -1, dtype=torch.int32, device="cuda") for _, n in shapes]
    torch.cuda.synchronize()
    calls = []
    for (frame, n), buf in zip(shapes, bufs):
        cam = _moved_camera(bihrt_mod, w, h, -0.9 + 1.8 * frame / 160, 0.0, 0.0)
        r.camera = cam
        if n == 1:
            r.render_device(buf.data_ptr(), frame)
        else:
            r.render_device_frames(buf.data_ptr(), frame, n, stride)
        calls.append((frame, n, cam, buf))
    r.sync()
    checked = 0
    for k, (f0, n, cam, buf) in enumerate(calls):
        if k % 3 and k != len(calls) - 1:
            continue
        b = buf.cpu().numpy().view(np.uint32)
        for j in sorted({0, n - 1}):
            ref, _ = ot.render(w, h, frame=f0 + j, cam=np.array(cam.as_list(), np.float32))
            got = b[j * stride:(j + 1) * stride].reshape(h, w)
            assert np.array_equal(got, ref), (f0 + j, int((got != ref).sum()))
            checked += 1
    assert checked >= 10
    # another kind of render, then back
    cam = calls[-1][2]
    r.camera = cam
    camf = np.array(cam.as_list(), np.float32)
    out = torch.zeros(h * w, dtype=torch.int32, device="cuda")
    side = torch.cuda.Stream()
    torch.cuda.synchronize()
    # a Whitted frame, a frame on another stream, four in a row (back into
    # stamped mode), a gap of two sync runs (whole-run jumps), a jump back
    plan = [(160, "whitted", None), (161, "bins", side), (162, "bins", None), (163, "bins", None),
            (164, "bins", None), (165, "bins", None), (300, "bins", None), (301, "bins", None),
            (40, "bins", None), (41, "bins", None)]
    for f, kind, stream in plan:
        if kind == "whitted":
            r.render_whitted_device(out.data_ptr(), f)
            ref, _ = ot.render_whitted(w, h, frame=f, cam=camf)
        else:
            r.render_device(out.data_ptr(), f, stream=stream.cuda_stream if stream else None)
            ref, _ = ot.render(w, h, frame=f, cam=camf)
        if stream is not None:
            stream.synchronize()
        r.sync()
        got = out.cpu().numpy().view(np.uint32).reshape(h, w)
        assert np.array_equal(got, ref), (f, kind, int((got != ref).sum()))
    g.close()


@pytest.mark.gpu
def test_ring_advance_jump_tables_match_oracle(gpu, bihrt_mod, oracle_mod):
    """Frames on two streams in turn (the XORWOW ring, not the stamped
    state) with gaps of 48 and 148 frames: the ring's advance jumps the
    powers 2^7 .. 2^13 of the step count through its nibble tables (one or
    two of them) and steps the rest (bih_render.hip k_rng_advance); a
    16-frame call advances by exactly one table.  Every frame equals the
    oracle's."""
    import torch
    tris = bihrt_mod.scenes.soup(20_000, seed=4)
    g = bihrt_mod.GPUArrayManager(tris)
    ot = oracle_mod.OracleTree(tris)
    w, h = 96, 64
    r = bihrt_mod.Renderer(g, w, h)
    streams = [torch.cuda.Stream() for _ in range(2)]
    torch.cuda.synchronize()
    stride = h * w
    plan = [(0, 1), (1, 1), (50, 1), (51, 16), (67, 1), (216, 1), (217, 1)]
    # (filled before any render: the renders' streams do not order after
    # torch's default stream)
    bufs = [torch.full((n * stride,), -1, dtype=torch.int32, device="cuda") for _, n in plan]
    torch.cuda.synchronize()
    for k, (f, n) in enumerate(plan):
        buf = bufs[k]
        s = streams[k % 2].cuda_stream
        if n == 1:
            r.render_device(buf.data_ptr(), f, stream=s)
        else:
            r.render_device_frames(buf.data_ptr(), f, n, stride, stream=s)
    torch.cuda.synchronize()
    for (f, n), buf in zip(plan, bufs):
        b = buf.cpu().numpy().view(np.uint32)
        for j in sorted({0, n - 1}):
            ref, _ = ot.render(w, h, frame=f + j)
            got = b[j * stride:(j + 1) * stride].reshape(h, w)
            assert np.array_equal(got, ref), (f + j, int((got != ref).sum()), int((got == 0xFFFFFFFF).sum()))
    g.close()


@pytest.mark.gpu
def test_reserve_growing_stamps_mid_stamped_run(gpu, bihrt_mod, oracle_mod):
    """bih_reserve of a shape with more tiles (a higher spp: smaller packet
    tiles) while a one-stream frame loop runs on the stamped XORWOW state:
    the stamp array grows, and the stamped state is first folded back into
    the ring, so the next frames continue the sequence (before the
    fix the ring still held the state stamped mode started from).  Frames
    before and after equal the oracle's."""
    tris = bihrt_mod.scenes.soup(20_000, seed=12)
    ot = oracle_mod.OracleTree(tris)
    w, h = 96, 64
    g = bihrt_mod.GPUArrayManager(tris)
    r = bihrt_mod.Renderer(g, w, h)
    imgs = {}
    for f in range(6):                      # one stream: stamped from the fourth render on
        imgs[f] = r.render(f)
    g.reserve(w, h, 16, None, 4)            # 16 spp: 2x2 tiles, 4x the stamps
    for f in range(6, 9):
        imgs[f] = r.render(f)
    g.reserve(w * 2, h, 64, None, 1)        # the ring grows too (more pixels): re-seeded
    for f in (9, 10, 40):
        imgs[f] = r.render(f)
    for f, img in imgs.items():
        ref, _ = ot.render(w, h, frame=f)
        assert np.array_equal(img, ref), (f, int((img != ref).sum()))
    g.close()


@pytest.mark.gpu
def test_one_stream_1m_1080p_stamped_across_syncs(gpu, bihrt_mod, oracle_mod, soup1m):
    """The stamped XORWOW state at the BASELINE size: the
    1M soup at 1920x1080 on ONE stream, 140 frames in calls of 1 and 16
    frames -- stamped launches (k_render_bins<L, 4>) from the fourth render
    on, two k_rng_sync runs (every 64 frames) -- as INTEGRATION.md's frame
    loop issues them.  Frames 0, 70 and 139 equal the oracle on every row
    (cudaRender's persistent per-pixel curandState, CUDAKernels.cu:391-423)."""
    import torch
    tris, ot = soup1m
    w, h = 1920, 1080
    d = torch.from_numpy(tris).cuda()
    g = bihrt_mod.GPUArrayManager.from_device(d.data_ptr(), tris.shape[0])
    g.reserve(w, h, 4, None, 16)
    r = bihrt_mod.Renderer(g, w, h)
    want = (0, 70, 139)
    sizes = [1, 1, 1, 1, 16, 16, 1, 16, 16, 1, 1, 16, 16, 16, 1, 16]
    plan, f = [], 0
    while f < 140:
        n = min(sizes[len(plan) % len(sizes)], 140 - f)
        plan.append((f, n))
        f += n
    scratch = torch.zeros(16 * h * w, dtype=torch.int32, device="cuda")
    kept = {}
    torch.cuda.synchronize()
    for f0, n in plan:
        hit = [q for q in want if f0 <= q < f0 + n]
        buf = torch.full((n * h * w,), -1, dtype=torch.int32, device="cuda") if hit else scratch
        if hit:
            torch.cuda.synchronize()       # (the fill, on torch's stream, before the library's)
        if n == 1:
            r.render_device(buf.data_ptr(), f0)
        else:
            r.render_device_frames(buf.data_ptr(), f0, n, h * w)
        for q in hit:
            kept[q] = (buf, q - f0)
    r.sync()
    assert g.bins_stats().usable
    for q in want:
        buf, j = kept[q]
        got = buf[j * h * w:(j + 1) * h * w].cpu().numpy().view(np.uint32).reshape(h, w)
        ref, _ = ot.render(w, h, frame=q, mode=oracle_mod.MODE_GPU_ANYHIT, threads=0)
        assert np.array_equal(got, ref), (q, int((got != ref).sum()))
    g.close()


@pytest.mark.gpu
def test_dynamic_soup_1m_540p_rebuild_equals_oracle(gpu, bihrt_mod, oracle_mod, soup1m):
    """Geometry that changes every frame (bench `dynamic_rebuild`, VERDICT r5
    item 5): the tree's device soup is overwritten with another 1M soup and
    rebuilt (src/App.cpp:174-183 -> src/Renderer.cpp:415-501), and the next
    frames -- whose camera structures must follow the new tree -- equal the
    oracle of the new soup; then back to the first soup, frames in flight on
    two streams."""
    import torch
    tris_a, ot_a = soup1m
    tris_b = bihrt_mod.scenes.soup(1_000_000, seed=2)
    ot_b = oracle_mod.OracleTree(tris_b)
    w, h = 960, 540
    d = torch.from_numpy(tris_a).cuda()
    d_b = torch.from_numpy(tris_b).cuda()
    d_a = d.clone()
    g = bihrt_mod.GPUArrayManager.from_device(d.data_ptr(), tris_a.shape[0])
    r = bihrt_mod.Renderer(g, w, h)
    streams = [torch.cuda.Stream() for _ in range(2)]
    outs = [torch.zeros(4 * h * w, dtype=torch.int32, device="cuda") for _ in range(6)]
    torch.cuda.synchronize()
    seq = [("A", 0, 1), ("A", 1, 4), ("B", 5, 1), ("B", 6, 4), ("A", 10, 4), ("B", 14, 1)]
    cur = "A"
    for k, (soup, f0, n) in enumerate(seq):
        if soup != cur:
            torch.cuda.synchronize()
            d.copy_(d_b if soup == "B" else d_a)
            torch.cuda.synchronize()
            g.rebuild()
            cur = soup
        s = streams[k % 2].cuda_stream
        if n == 1:
            r.render_device(outs[k].data_ptr(), f0, stream=s)
        else:
            r.render_device_frames(outs[k].data_ptr(), f0, n, h * w, stream=s)
    torch.cuda.synchronize()
    for k, (soup, f0, n) in enumerate(seq):
        ot = ot_b if soup == "B" else ot_a
        for j in sorted({0, n - 1}):
            got = outs[k][j * h * w:(j + 1) * h * w].cpu().numpy().view(np.uint32).reshape(h, w)
            ref, _ = ot.render(w, h, frame=f0 + j, mode=oracle_mod.MODE_GPU_ANYHIT, threads=0)
            assert np.array_equal(got, ref), (soup, f0 + j, int((got != ref).sum()))
    g.close()


@pytest.mark.gpu
def test_host_loop_registered_framebuffer(gpu, bihrt_mod, oracle_mod):
    """INTEGRATION.md's loop (bih_rebuild + bih_render into a host
    framebuffer) into one reused buffer, pageable and then page-locked with
    bih_host_register: every frame equals the oracle's."""
    tris = bihrt_mod.scenes.soup(50_000, seed=4)
    ot = oracle_mod.OracleTree(tris)
    w, h = 320, 180
    g = bihrt_mod.GPUArrayManager(tris)
    r = bihrt_mod.Renderer(g, w, h)
    fb = np.zeros((h, w), np.uint32)
    for f in range(3):
        g.rebuild()
        r.render(f, out=fb)
        ref, _ = ot.render(w, h, frame=f)
        assert np.array_equal(fb, ref), f
    bihrt_mod.host_register(fb)
    try:
        for f in range(3, 7):
            g.rebuild()
            r.render(f, out=fb)
            ref, _ = ot.render(w, h, frame=f)
            assert np.array_equal(fb, ref), f
    finally:
        bihrt_mod.host_unregister(fb)
    with pytest.raises(ValueError):
        r.render(7, out=np.zeros((h, w + 1), np.uint32))
    g.close()


@pytest.mark.gpu
def test_destroyed_streams_keep_order(gpu, bihrt_mod, oracle_mod):
    """Streams created and destroyed through the HIP runtime (not torch's
    pool), each destroyed with its renders possibly still queued and the next
    created at once (the handle may come back): the library orders every
    render after the last one's state by events, never by stream identity, so
    every frame equals the oracle's."""
    import ctypes
    import torch
    torch.cuda.init()
    hip = ctypes.CDLL("libamdhip64.so.7")          # (the runtime torch loaded)
    tris = bihrt_mod.scenes.soup(30_000, seed=17)
    ot = oracle_mod.OracleTree(tris)
    w, h = 128, 96
    g = bihrt_mod.GPUArrayManager(tris)
    r = bihrt_mod.Renderer(g, w, h)
    outs = [torch.full((h * w,), -1, dtype=torch.int32, device="cuda") for _ in range(20)]
    torch.cuda.synchronize()
    f = 0
    for rnd in range(4):
        s = ctypes.c_void_p()
        assert hip.hipStreamCreate(ctypes.byref(s)) == 0
        for _ in range(5):
            r.render_device(outs[f].data_ptr(), f, stream=s.value)
            f += 1
        assert hip.hipStreamDestroy(s) == 0     # (its renders may still be queued)
    torch.cuda.synchronize()
    for k in range(f):
        got = outs[k].cpu().numpy().view(np.uint32).reshape(h, w)
        ref, _ = ot.render(w, h, frame=k)
        assert np.array_equal(got, ref), (k, int((got != ref).sum()))
    g.close()


def test_recycled_stream_handles_keep_order(gpu, bihrt_mod, oracle_mod):
    """Stamped mode and the shared-grid rule key on the raw hipStream_t of
    the last render.  A stream the caller destroys and
    creates again may come back with the same handle: the library must not
    rely on that identity for ordering (every render waits on ev_rng, the
    event after the last stamped launch or ring advance).  One-frame calls
    on a stream (stamped from the fourth on), the stream destroyed and a new
    one created (often the same handle) for the next frames, then a frame on
    a fresh stream: every frame equals the oracle's."""
    import torch
    tris = bihrt_mod.scenes.soup(30_000, seed=13)
    ot = oracle_mod.OracleTree(tris)
    w, h = 128, 96
    g = bihrt_mod.GPUArrayManager(tris)
    r = bihrt_mod.Renderer(g, w, h)
    outs = [torch.full((h * w,), -1, dtype=torch.int32, device="cuda") for _ in range(16)]
    torch.cuda.synchronize()
    f = 0
    plan = []
    for rnd in range(3):
        s = torch.cuda.Stream()
        for _ in range(5):
            r.render_device(outs[f].data_ptr(), f, stream=s.cuda_stream)
            plan.append(f)
            f += 1
        s.synchronize()
        del s                                  # (the handle may be reused by the next stream)
    for k in range(1):
        a = torch.cuda.Stream()
        r.render_device(outs[f].data_ptr(), f, stream=a.cuda_stream)
        plan.append(f)
        f += 1
    torch.cuda.synchronize()
    for f in plan:
        got = outs[f].cpu().numpy().view(np.uint32).reshape(h, w)
        ref, _ = ot.render(w, h, frame=f)
        assert np.array_equal(got, ref), (f, int((got != ref).sum()))
    g.close()
