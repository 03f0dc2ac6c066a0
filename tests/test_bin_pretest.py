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
