"""The frustum bins' edge pre-test (csrc/bih_bins.hip, edge_pretest; the
render loop's bin_walk) may only drop a lane for a triangle when the exact f32
intersector (RayTriangleIntersection, CUDAKernels.cu:17-50, as prim_hits
evaluates it) rejects that lane's ray: for every accepted (ray, triangle),
K0' + Ku u + Kv v >= 0 for all three edges, with u, v the f32 values the
kernel forms and D its f32 camera_dir.  A numpy restatement of the pre-test
(f64 coefficients, f32 rounding, fmaf evaluation emulated), checked on
near-edge-on triangles and a soup for the reference camera and cameras far
from the origin, at the library's own dmax (bih_camera_ray_bound)."""
import numpy as np
import pytest

from test_miss_box import F, _barycentric_bounds, _camera_dir, _mt, _offset_cameras, _tri_prim

E = 2.0 ** -24


def _f32_up(x):
    f = x.astype(np.float32)
    low = f.astype(np.float64) < x
    f[low] = np.nextafter(f[low], np.float32(np.inf))
    return f


def _pretest_coeffs(e1, e2, s, a, b, c, cam):
    """edge_pretest: per triangle 3 x (K0 + M rounded up, Ku, Kv) as f32."""
    cam = np.asarray(cam, np.float64)
    O, llc, h, vert = cam[:3], cam[3:6], cam[6:9], cam[9:12]
    A = llc - O
    delta = 8.0 * E * (np.abs(llc) + np.abs(h) + np.abs(vert) + np.abs(O))
    e1, e2, s = (x.astype(np.float64) for x in (e1, e2, s))
    Nu, Nd, Q = np.cross(e2, s), np.cross(e2, e1), np.cross(s, e1)
    a, b, c = (x.astype(np.float64)[:, None] for x in (a, b, c))
    G = [Nu + a * Nd, Q + b * Nd, (1.0 + c) * Nd - Nu - Q]
    out = []
    for g in G:
        K0, Ku, Kv = g @ A, g @ h, g @ vert
        dg = np.abs(g) @ delta
        M = 4.0 * (dg + 8.0 * E * (np.abs(K0) + np.abs(Ku) + np.abs(Kv)) + 1e-30)
        out.append((_f32_up(K0 + M + 8.0 * E * M), Ku.astype(np.float32), Kv.astype(np.float32)))
    return out


def _fmaf(x, y, z):
    return (x.astype(np.float64) * y.astype(np.float64) + z.astype(np.float64)).astype(np.float32)


def _check(cam, dmax, v0, v1, v2, u, v):
    """Accepted rays all pass the pre-test; returns (accepted, rejected by
    MT, of those dropped by the pre-test)."""
    O = np.asarray(cam[:3], F)
    D = _camera_dir(cam, u, v)
    v0, v1, v2 = (np.asarray(x, F) for x in (v0, v1, v2))
    e1, e2 = (v1 - v0).astype(F), (v2 - v0).astype(F)
    s, q, tn = _tri_prim(v0, e1, e2, O)
    with np.errstate(all="ignore"):
        hit, _ = _mt(e1, e2, s, q, tn, D)
        dm = np.broadcast_to(np.asarray(dmax, F), D.shape)
        a, b, c = _barycentric_bounds(e1, e2, s, dm)
        den_ok = (F(0.99e-6) - _ed(e1, e2, dm)) > F(0.5e-6)
        ok = den_ok & (a < F(1e30)) & (b < F(1e30)) & (c < F(1e30)) & (tn > 0)
        co = _pretest_coeffs(e1, e2, s, a, b, c, cam)
        passed = np.ones(len(u), bool)
        for K0, Ku, Kv in co:
            f = _fmaf(Kv, v, _fmaf(Ku, u, K0))
            passed &= ~(f < 0)
    h = hit & ok
    assert not np.any(h & ~passed), int((h & ~passed).sum())
    miss = ok & ~hit
    return int(h.sum()), int(miss.sum()), int((miss & ~passed).sum())


def _ed(e1, e2, dmax):
    Em = F(6.0 * 2.0 ** -24)
    ae1, ae2 = np.abs(e1), np.abs(e2)
    P = np.stack([dmax[:, 1] * ae2[:, 2] + ae2[:, 1] * dmax[:, 2],
                  dmax[:, 2] * ae2[:, 0] + ae2[:, 2] * dmax[:, 0],
                  dmax[:, 0] * ae2[:, 1] + ae2[:, 0] * dmax[:, 1]], 1).astype(F)
    return Em * ((ae1[:, 0] * P[:, 0] + ae1[:, 1] * P[:, 1]) + ae1[:, 2] * P[:, 2])


def _scene_on_rays(cam, n, rng, edge_on):
    u = rng.random(n).astype(F)
    v = rng.random(n).astype(F)
    D = _camera_dir(cam, u, v).astype(np.float64)
    O = np.asarray(cam[:3], np.float64)
    X = O + rng.uniform(0.5, 3.0, (n, 1)) * D
    dh = D / np.linalg.norm(D, axis=1, keepdims=True)
    aa = np.cross(dh, rng.normal(size=(n, 3)))
    aa /= np.linalg.norm(aa, axis=1, keepdims=True)
    lo = -6 if edge_on else -0.5
    th = 10.0 ** rng.uniform(lo, -0.2, n)[:, None]
    bb = np.cos(th) * dh + np.sin(th) * np.cross(dh, aa)
    size = rng.uniform(0.005, 0.08, (n, 1))
    al, be = rng.uniform(-0.3, 1.3, (n, 1)), rng.uniform(-0.3, 1.3, (n, 1))
    v0 = X - size * (al * aa + be * bb)
    v1, v2 = v0 + size * bb, v0 + size * aa
    flip = rng.random(n) < 0.5
    v1[flip], v2[flip] = v2[flip].copy(), v1[flip].copy()
    # jitter the sample within a few pixels (rays that miss nearby)
    du = (rng.normal(size=n) * 10.0 ** rng.uniform(-6, -2, n)).astype(F)
    dv = (rng.normal(size=n) * 10.0 ** rng.uniform(-6, -2, n)).astype(F)
    return v0, v1, v2, np.clip(u + du, 0, 1).astype(F), np.clip(v + dv, 0, 1).astype(F)


def test_edge_pretest_keeps_every_accepted_ray(bihrt_mod):
    rng = np.random.default_rng(21)
    acc = rej = dropped = 0
    for cam in _offset_cameras()[:3]:
        dmax = bihrt_mod.camera_ray_bound(bihrt_mod.Camera.from_list(cam.tolist()))
        for edge_on in (True, False):
            h, m, d = _check(cam, dmax, *_scene_on_rays(cam, 150_000, rng, edge_on))
            acc, rej, dropped = acc + h, rej + m, dropped + d
    assert acc > 50_000
    # the pre-test has teeth: it drops most of the rays MT rejects
    assert dropped > 0.25 * rej, (dropped, rej)


def test_edge_pretest_soup_reference_camera(bihrt_mod):
    """Bench-like soup (SURVEY 8d C3 shape) at 1080p's reference camera."""
    rng = np.random.default_rng(4)
    cam = np.asarray(bihrt_mod.camera_reference(1920, 1080).as_list(), F)
    dmax = bihrt_mod.camera_ray_bound(bihrt_mod.Camera.from_list(cam.tolist()))
    n = 400_000
    c = np.stack([rng.uniform(0, 2.6667, n), rng.uniform(-1, 1, n), rng.uniform(0, 2, n)], 1)
    v = c[:, None, :] + rng.uniform(-0.02, 0.02, (n, 3, 3))
    # samples aimed at points in and around each triangle
    w = rng.uniform(-0.3, 1.3, (n, 2))
    X = v[:, 0] + w[:, :1] * (v[:, 1] - v[:, 0]) + w[:, 1:] * (v[:, 2] - v[:, 0])
    O, llc, hh, vv = (cam[3 * k:3 * k + 3].astype(np.float64) for k in range(4))
    d = X - O
    lam = (llc - O)[2] / d[:, 2]
    Y = d * lam[:, None] - (llc - O)
    u = np.clip(Y[:, 0] / hh[0], 0, 1).astype(F)
    vq = np.clip(Y[:, 1] / vv[1], 0, 1).astype(F)
    h, m, dr = _check(cam, dmax, v[:, 0], v[:, 1], v[:, 2], u, vq)
    assert h > 20_000 and dr > 0.5 * m, (h, m, dr)


def _bin_camera(cam):
    """bin_camera's n (A.n > 0), A.n and dn_lb (bih_bins.hip)."""
    cam = np.asarray(cam, np.float64)
    O, llc, h, vert = cam[:3], cam[3:6], cam[6:9], cam[9:12]
    A = llc - O
    n = np.cross(h, vert)
    if A @ n < 0:
        n = -n
    delta = 8.0 * E * (np.abs(llc) + np.abs(h) + np.abs(vert) + np.abs(O))
    an = A @ n
    return n, an, an - 2.0 * (delta @ np.abs(n))


def _refined_bounds(e1, e2, s, tn, dmax, cam):
    """k_bin_fp's refinement: coarse a, b, c; when every corner of the
    inflated triangle lies in front, det >= 0.99 (tnum_c - 8e |e2|.Q) dn_lb /
    max depth (det_lower_bound, bih_bound.h), and a, b, c are recomputed with
    that den (miss_bary's den_lb).  Returns a, b, c, the mask where the
    refinement applied."""
    n, an, dn_lb = _bin_camera(cam)
    a, b, c = _barycentric_bounds(e1, e2, s, dmax)
    e164, e264, s64 = (x.astype(np.float64) for x in (e1, e2, s))
    cu = [-a.astype(np.float64), 1.0 + b.astype(np.float64) + c.astype(np.float64), -a.astype(np.float64)]
    cv = [-b.astype(np.float64), -b.astype(np.float64), 1.0 + a.astype(np.float64) + c.astype(np.float64)]
    front = np.ones(len(a), bool)
    maxd = np.zeros(len(a))
    for j in range(3):
        X = cu[j][:, None] * e164 + cv[j][:, None] * e264 - s64
        d = X @ n
        front &= d > 1e-9 * np.linalg.norm(X, axis=1) * np.linalg.norm(n)
        maxd = np.maximum(maxd, d)
    as_, ae1 = np.abs(s64), np.abs(e164)
    Q = np.stack([as_[:, 1] * ae1[:, 2] + ae1[:, 1] * as_[:, 2],
                  as_[:, 2] * ae1[:, 0] + ae1[:, 2] * as_[:, 0],
                  as_[:, 0] * ae1[:, 1] + ae1[:, 0] * as_[:, 1]], 1)
    et = 8.0 * E * np.einsum("ij,ij->i", np.abs(e264), Q)
    tlb = tn.astype(np.float64) - et
    with np.errstate(all="ignore"):
        L = 0.99 * tlb * dn_lb / maxd
    use = front & (tlb > 0) & (maxd > 0) & (L < 1e30)
    Em = F(6.0 * 2.0 ** -24)
    ae1f, ae2f, asf = np.abs(e1), np.abs(e2), np.abs(s)
    P = np.stack([dmax[:, 1] * ae2f[:, 2] + ae2f[:, 1] * dmax[:, 2],
                  dmax[:, 2] * ae2f[:, 0] + ae2f[:, 2] * dmax[:, 0],
                  dmax[:, 0] * ae2f[:, 1] + ae2f[:, 0] * dmax[:, 1]], 1).astype(F)
    Qf = np.stack([asf[:, 1] * ae1f[:, 2] + ae1f[:, 1] * asf[:, 2],
                   asf[:, 2] * ae1f[:, 0] + ae1f[:, 2] * asf[:, 0],
                   asf[:, 0] * ae1f[:, 1] + ae1f[:, 0] * asf[:, 1]], 1).astype(F)
    dot = lambda x, y: (x[:, 0] * y[:, 0] + x[:, 1] * y[:, 1]) + x[:, 2] * y[:, 2]
    Eu, Ed, Ev = Em * dot(asf, P), Em * dot(ae1f, P), Em * dot(dmax, Qf)
    den0 = F(0.99e-6) - Ed
    Lf = np.where(use, L, 0).astype(F)
    den = np.maximum(den0, Lf)
    a2 = F(4) * Em + Eu / den
    b2 = F(4) * Em + Ev / den
    c2 = F(8) * Em + F(1.01) * (Eu + Ev + F(2) * Ed) / den
    take = use & (a2 <= a) & (b2 <= b) & (c2 <= c)
    return np.where(take, a2, a), np.where(take, b2, b), np.where(take, c2, c), take


def _check_refined(cam, dmax, v0, v1, v2, u, v):
    """Accepted rays: exact-line barycentrics inside the refined inflated
    triangle and the refined pre-test passed.  Returns (accepted, accepted
    under a refined bound, largest excursion / refined bound)."""
    O = np.asarray(cam[:3], F)
    D = _camera_dir(cam, u, v)
    v0, v1, v2 = (np.asarray(x, F) for x in (v0, v1, v2))
    e1, e2 = (v1 - v0).astype(F), (v2 - v0).astype(F)
    s, q, tn = _tri_prim(v0, e1, e2, O)
    with np.errstate(all="ignore"):
        hit, _ = _mt(e1, e2, s, q, tn, D)
        dm = np.broadcast_to(np.asarray(dmax, F), D.shape)
        a0, b0, c0 = _barycentric_bounds(e1, e2, s, dm)
        ok = ((F(0.99e-6) - _ed(e1, e2, dm)) > F(0.5e-6)) & (a0 < F(1e30)) & (b0 < F(1e30)) & \
            (c0 < F(1e30)) & (tn > 0)
        a, b, c, ref = _refined_bounds(e1, e2, s, tn, dm, cam)
        co = _pretest_coeffs(e1, e2, s, a, b, c, cam)
        passed = np.ones(len(u), bool)
        for K0, Ku, Kv in co:
            f = _fmaf(Kv, v, _fmaf(Ku, u, K0))
            passed &= ~(f < 0)
        s64, e164, e264, D64 = (x.astype(np.float64) for x in (s, e1, e2, D))
        p = np.cross(D64, e264)
        det64 = np.einsum("ij,ij->i", e164, p)
        uu = np.einsum("ij,ij->i", s64, p) / det64
        vv = np.einsum("ij,ij->i", D64, np.cross(s64, e164)) / det64
    h = hit & ok
    a, b, c = (x.astype(np.float64) for x in (a, b, c))
    assert np.all(uu[h] >= -a[h]) and np.all(vv[h] >= -b[h]) and np.all(uu[h] + vv[h] <= 1 + c[h])
    assert not np.any(h & ~passed), int((h & ~passed).sum())
    hr = h & ref
    ratio = np.max(np.concatenate([(-uu[hr]) / a[hr], (-vv[hr]) / b[hr], (uu[hr] + vv[hr] - 1) / c[hr],
                                   [0.0]]))
    return int(h.sum()), int(hr.sum()), ratio


def test_refined_bound_keeps_every_accepted_ray(bihrt_mod):
    """det_lower_bound (bih_bound.h): the tighter inflation still contains the
    exact-line barycentrics of every accepted ray and the pre-test built from
    it keeps them -- near-edge-on triangles (det down to 1e-6), offset cameras."""
    rng = np.random.default_rng(33)
    acc = refd = 0
    worst = 0.0
    for cam in _offset_cameras()[:3]:
        dmax = bihrt_mod.camera_ray_bound(bihrt_mod.Camera.from_list(cam.tolist()))
        for edge_on in (True, False):
            h, r, w = _check_refined(cam, dmax, *_scene_on_rays(cam, 150_000, rng, edge_on))
            acc, refd, worst = acc + h, refd + r, max(worst, w)
    assert acc > 50_000 and refd > 0.5 * acc, (acc, refd)
    assert worst > 0.005, worst        # accepted rays do approach the refined bound


def test_refined_bound_soup_reference_camera(bihrt_mod):
    """The bench's soup shape: the refinement applies to nearly every
    triangle and shrinks the inflation by orders of magnitude."""
    rng = np.random.default_rng(8)
    cam = np.asarray(bihrt_mod.camera_reference(1920, 1080).as_list(), F)
    dmax = bihrt_mod.camera_ray_bound(bihrt_mod.Camera.from_list(cam.tolist()))
    n = 300_000
    c = np.stack([rng.uniform(0, 2.6667, n), rng.uniform(-1, 1, n), rng.uniform(0, 2, n)], 1)
    v = c[:, None, :] + rng.uniform(-0.02, 0.02, (n, 3, 3))
    w = rng.uniform(-0.01, 1.01, (n, 2))
    X = v[:, 0] + w[:, :1] * (v[:, 1] - v[:, 0]) + w[:, 1:] * (v[:, 2] - v[:, 0])
    O, llc, hh, vv = (cam[3 * k:3 * k + 3].astype(np.float64) for k in range(4))
    d = X - O
    lam = (llc - O)[2] / d[:, 2]
    Y = d * lam[:, None] - (llc - O)
    u = np.clip(Y[:, 0] / hh[0], 0, 1).astype(F)
    vq = np.clip(Y[:, 1] / vv[1], 0, 1).astype(F)
    h, r, _ = _check_refined(cam, dmax, v[:, 0], v[:, 1], v[:, 2], u, vq)
    assert h > 50_000 and r > 0.95 * h, (h, r)


def _edge_margin(K0, Ku, Kv):
    """edge_margin (bih_bins.hip): 2^-21 fl(|K0| + |Ku| + |Kv|) + 2^-125, f32."""
    S = (np.abs(K0) + np.abs(Ku)).astype(F) + np.abs(Kv)
    return (F(2.0 ** -21) * S.astype(F)).astype(F) + F(2.0 ** -125)


def _tile_class(K, bx, by, w, h, tw, th):
    """tile_class (bih_bins.hip), op for op in f32, on coefficient triples
    K = [(K0, Ku, Kv)] x 3."""
    pad = F(2.0 ** -20)
    iw, ih = F(1.0) / F(w), F(1.0) / F(h)
    xe = np.minimum((bx + 1) * tw, w)
    ye = np.minimum((by + 1) * th, h)
    u0 = (bx * tw).astype(F) * iw - pad
    u1 = xe.astype(F) * iw + pad
    v0 = (by * th).astype(F) * ih - pad
    v1 = ye.astype(F) * ih + pad
    out = np.full(len(bx), 2)
    with np.errstate(all="ignore"):
        for K0, Ku, Kv in K:
            K0, Ku, Kv = (np.asarray(x, F) for x in (K0, Ku, Kv))
            T = _edge_margin(K0, Ku, Kv)
            au0, au1, bv0, bv1 = Ku * u0, Ku * u1, Kv * v0, Kv * v1
            hi = (K0 + np.fmax(au0, au1)) + np.fmax(bv0, bv1)
            lo = (K0 + np.fmin(au0, au1)) + np.fmin(bv0, bv1)
            out = np.where(hi < -T, 0, np.where(~(lo > T), np.minimum(out, 1), out))
    return out


def _pixel_mask(K, bx, by, w, h):
    """pixel_mask (bih_bins.hip) of 4 x 4 tiles, op for op in f32."""
    pad = F(2.0 ** -20)
    iw, ih = F(1.0) / F(w), F(1.0) / F(h)
    x = bx[:, None] * 4 + np.arange(4)[None, :]
    y = by[:, None] * 4 + np.arange(4)[None, :]
    ua, ub = x.astype(F) * iw - pad, (x + 1).astype(F) * iw + pad
    va, vb = y.astype(F) * ih - pad, (y + 1).astype(F) * ih + pad
    m = np.full(len(bx), 0xFFFF, np.int64)
    with np.errstate(all="ignore"):
        for K0, Ku, Kv in K:
            K0, Ku, Kv = (np.asarray(z, F)[:, None] for z in (K0, Ku, Kv))
            T = _edge_margin(K0, Ku, Kv)
            cu = K0 + np.fmax(Ku * ua, Ku * ub)
            cv = np.fmax(Kv * va, Kv * vb)
            for py in range(4):
                for px in range(4):
                    out = (cu[:, px] + cv[:, py]) < -T[:, 0]
                    m = np.where(out, m & ~(1 << (4 * py + px)), m)
    return m


@pytest.mark.parametrize("size", [0.02, 0.3])
def test_tile_class_keeps_passing_samples(bihrt_mod, size):
    """A tile is dropped from a triangle's list only when no sample of it can
    pass the pre-test; a tile classed 'every sample passes' has every sample
    pass.  Samples at the kernel's f32 (x + r) / W, r in (0, 1].  Bench-size
    triangles (~5 px) and large ones (~80 px, tiles inside them)."""
    rng = np.random.default_rng(12)
    W, H, tw, th = 1920, 1080, 4, 4
    cam = np.asarray(bihrt_mod.camera_reference(W, H).as_list(), F)
    dmax = bihrt_mod.camera_ray_bound(bihrt_mod.Camera.from_list(cam.tolist()))
    n = 200_000
    c = np.stack([rng.uniform(0, 2.6667, n), rng.uniform(-1, 1, n), rng.uniform(0, 2, n)], 1)
    v = (c[:, None, :] + rng.uniform(-size, size, (n, 3, 3))).astype(F)
    O = cam[:3]
    e1, e2 = (v[:, 1] - v[:, 0]).astype(F), (v[:, 2] - v[:, 0]).astype(F)
    s, q, tn = _tri_prim(v[:, 0], e1, e2, O)
    dm = np.broadcast_to(np.asarray(dmax, F), e1.shape)
    with np.errstate(all="ignore"):
        a, b, cc, _ = _refined_bounds(e1, e2, s, tn, dm, cam)
        K = _pretest_coeffs(e1, e2, s, a, b, cc, cam)
    # a sample pixel near each triangle's projection, random jitter
    Xc = v.mean(1).astype(np.float64)
    llc, hh, vv = (cam[3 * k:3 * k + 3].astype(np.float64) for k in (1, 2, 3))
    d = Xc - O
    lam = (llc - O)[2] / d[:, 2]
    Y = d * lam[:, None] - (llc - O)
    sp = int(400 * size)
    px = np.clip((Y[:, 0] / hh[0] * W).astype(np.int64) + rng.integers(-sp, sp + 1, n), 0, W - 1)
    py = np.clip((Y[:, 1] / vv[1] * H).astype(np.int64) + rng.integers(-sp, sp + 1, n), 0, H - 1)
    r1 = np.maximum(rng.random(n).astype(F), F(2.0 ** -32))
    r2 = np.maximum(rng.random(n).astype(F), F(2.0 ** -32))
    u = ((px.astype(F) + r1).astype(F) / F(W)).astype(F)
    vq = ((py.astype(F) + r2).astype(F) / F(H)).astype(F)
    passed = np.ones(n, bool)
    with np.errstate(all="ignore"):
        for K0, Ku, Kv in K:
            passed &= ~(_fmaf(Kv, vq, _fmaf(Ku, u, K0)) < 0)
    cls = _tile_class(K, px // tw, py // th, W, H, tw, th)
    assert not np.any(passed & (cls == 0)), int((passed & (cls == 0)).sum())
    assert np.all(passed[cls == 2])
    # the pixel mask of the sample's tile keeps the sample's pixel
    m = _pixel_mask(K, px // tw, py // th, W, H)
    bit = (m >> (4 * (py % th) + (px % tw))) & 1
    assert not np.any(passed & (bit == 0)), int((passed & (bit == 0)).sum())
    assert (bit[cls == 1] == 0).sum() > 0.05 * (cls == 1).sum(), np.bincount(bit[cls == 1])
    # the test has teeth: many tiles are dropped (and, for the large
    # triangles, many are fully covered)
    assert (cls == 0).sum() > 0.1 * n, np.bincount(cls)
    if size > 0.1:
        assert (cls == 2).sum() > 1000, np.bincount(cls)
