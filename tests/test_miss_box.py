"""The miss-proof boxes of the any-hit walk (csrc/bih_render.hip, miss_box)
must contain, for every ray the exact f32 intersector accepts
(RayTriangleIntersection, CUDAKernels.cu:17-50, in the primary-ray record
form of prim_hits / k_tri_prim), a point of that ray's line -- as the
kernel's slab test sees it.  Checked on near-edge-on triangles (det down to
the 1e-6 threshold, where the intersector's rounding error is largest) and
on a random soup, with dmax = |D| per component (the tightest bound the
kernel may use).  A restatement in numpy f32 (every op rounded, no FMA), in
the kernel's operation order."""
import numpy as np

F = np.float32
EPS = F(np.uint32(0x358637BD).view(np.float32))
FMAX = F(np.finfo(np.float32).max)


def _tri_prim(v0, e1, e2, O):
    """k_tri_prim: s = O - v0, q = cross(s, e1), tnum = dot(e2, q)."""
    s = (O[None, :] - v0).astype(F)
    sx, sy, sz = s[:, 0], s[:, 1], s[:, 2]
    qx = sy * e1[:, 2] - e1[:, 1] * sz
    qy = sz * e1[:, 0] - e1[:, 2] * sx
    qz = sx * e1[:, 1] - e1[:, 0] * sy
    q = np.stack([qx, qy, qz], 1).astype(F)
    tn = (e2[:, 0] * qx + e2[:, 1] * qy) + e2[:, 2] * qz
    return s, q, tn.astype(F)


def _mt(e1, e2, s, q, tn, D):
    """prim_hits for one ray per triangle."""
    dx, dy, dz = D[:, 0], D[:, 1], D[:, 2]
    px = dy * e2[:, 2] - e2[:, 1] * dz
    py = dz * e2[:, 0] - e2[:, 2] * dx
    pz = dx * e2[:, 1] - e2[:, 0] * dy
    det = (e1[:, 0] * px + e1[:, 1] * py) + e1[:, 2] * pz
    ok = ~(det <= EPS)
    inv = F(1) / det
    u = ((s[:, 0] * px + s[:, 1] * py) + s[:, 2] * pz) * inv
    ok &= ~((u < 0) | (u > 1))
    v = ((dx * q[:, 0] + dy * q[:, 1]) + dz * q[:, 2]) * inv
    t = tn * inv
    ok &= ~((v < 0) | (u + v > 1)) & (t > 0) & (t < FMAX)
    return ok, det


def _miss_box(e1, e2, s, dmax):
    """miss_box, same f32 expressions."""
    E = F(6.0 * 2.0 ** -24)
    ae1, ae2, a_s = np.abs(e1), np.abs(e2), np.abs(s)
    P = np.stack([dmax[:, 1] * ae2[:, 2] + ae2[:, 1] * dmax[:, 2],
                  dmax[:, 2] * ae2[:, 0] + ae2[:, 2] * dmax[:, 0],
                  dmax[:, 0] * ae2[:, 1] + ae2[:, 0] * dmax[:, 1]], 1).astype(F)
    Q = np.stack([a_s[:, 1] * ae1[:, 2] + ae1[:, 1] * a_s[:, 2],
                  a_s[:, 2] * ae1[:, 0] + ae1[:, 2] * a_s[:, 0],
                  a_s[:, 0] * ae1[:, 1] + ae1[:, 0] * a_s[:, 1]], 1).astype(F)
    dot = lambda a, b: (a[:, 0] * b[:, 0] + a[:, 1] * b[:, 1]) + a[:, 2] * b[:, 2]
    Eu, Ed, Ev = E * dot(a_s, P), E * dot(ae1, P), E * dot(dmax, Q)
    den = F(0.99e-6) - Ed
    a = F(4) * E + Eu / den
    b = F(4) * E + Ev / den
    c = F(8) * E + F(1.01) * (Eu + Ev + F(2) * Ed) / den
    ok = (den > F(0.5e-6)) & (a < F(1e30)) & (b < F(1e30)) & (c < F(1e30))
    cu = [-a, F(1) + b + c, -a]
    cv = [-b, -b, F(1) + a + c]
    lo = np.empty_like(s)
    hi = np.empty_like(s)
    for ax in range(3):
        xs = [(cu[j] * e1[:, ax] + cv[j] * e2[:, ax]) - s[:, ax] for j in range(3)]
        l = np.minimum(np.minimum(xs[0], xs[1]), xs[2])
        h = np.maximum(np.maximum(xs[0], xs[1]), xs[2])
        lo[:, ax] = l - (F(1e-5) + F(1e-6) * np.abs(l))
        hi[:, ax] = h + (F(1e-5) + F(1e-6) * np.abs(h))
        ok &= (lo[:, ax] > F(-1e30)) & (hi[:, ax] < F(1e30))
    lo[~ok] = -np.inf
    hi[~ok] = np.inf
    return lo, hi


def _slab(lo, hi, D):
    """fast_walk's test with cons = true: tn <= tf over the whole line."""
    inv = (F(1) / D).astype(F)
    t0, t1 = lo * inv, hi * inv
    tn = np.max(np.minimum(t0, t1), axis=1)
    tf = np.min(np.maximum(t0, t1), axis=1)
    return tn <= tf


def _barycentric_bounds(e1, e2, s, dmax):
    """miss_box's a, b, c (f32, same expressions)."""
    E = F(6.0 * 2.0 ** -24)
    ae1, ae2, a_s = np.abs(e1), np.abs(e2), np.abs(s)
    P = np.stack([dmax[:, 1] * ae2[:, 2] + ae2[:, 1] * dmax[:, 2],
                  dmax[:, 2] * ae2[:, 0] + ae2[:, 2] * dmax[:, 0],
                  dmax[:, 0] * ae2[:, 1] + ae2[:, 0] * dmax[:, 1]], 1).astype(F)
    Q = np.stack([a_s[:, 1] * ae1[:, 2] + ae1[:, 1] * a_s[:, 2],
                  a_s[:, 2] * ae1[:, 0] + ae1[:, 2] * a_s[:, 0],
                  a_s[:, 0] * ae1[:, 1] + ae1[:, 0] * a_s[:, 1]], 1).astype(F)
    dot = lambda a, b: (a[:, 0] * b[:, 0] + a[:, 1] * b[:, 1]) + a[:, 2] * b[:, 2]
    Eu, Ed, Ev = E * dot(a_s, P), E * dot(ae1, P), E * dot(dmax, Q)
    den = F(0.99e-6) - Ed
    return (F(4) * E + Eu / den, F(4) * E + Ev / den,
            F(8) * E + F(1.01) * (Eu + Ev + F(2) * Ed) / den)


def _check(v0, v1, v2, O, D, dmax=None):
    """Every accepted ray: (1) its exact line meets the triangle's plane at
    barycentrics inside miss_box's inflated triangle (float64, exact enough:
    the claim the box rests on); (2) the kernel's slab test passes on the box.
    Returns the hit count, their det, and the largest violation of the plain
    triangle relative to the bound (how close the data comes to the bound)."""
    v0, v1, v2, D = (np.asarray(x, F) for x in (v0, v1, v2, D))
    e1, e2 = (v1 - v0).astype(F), (v2 - v0).astype(F)
    s, q, tn = _tri_prim(v0, e1, e2, O)
    with np.errstate(all="ignore"):
        hit, det = _mt(e1, e2, s, q, tn, D)
        if dmax is None:
            dmax = (np.abs(D) * F(1.001) + F(1e-6)).astype(F)
        else:
            dmax = np.broadcast_to(np.asarray(dmax, F), D.shape)
        lo, hi = _miss_box(e1, e2, s, dmax)
        inside = _slab(lo, hi, D)
        a, b, c = (x.astype(np.float64) for x in _barycentric_bounds(e1, e2, s, dmax))
    bad = hit & ~inside
    assert not bad.any(), (int(bad.sum()), det[bad][:5])
    # exact-line barycentrics (f64 from the f32 inputs MT used)
    s64, e164, e264, D64 = (x.astype(np.float64) for x in (s, e1, e2, D))
    p = np.cross(D64, e264)
    det64 = np.einsum("ij,ij->i", e164, p)
    u = np.einsum("ij,ij->i", s64, p) / det64
    v = np.einsum("ij,ij->i", D64, np.cross(s64, e164)) / det64
    h = hit
    assert np.all(det64[h] > 0)
    assert np.all(u[h] >= -a[h]) and np.all(v[h] >= -b[h]) and np.all(u[h] + v[h] <= 1 + c[h])
    ratio = np.max(np.concatenate([(-u[h]) / a[h], (-v[h]) / b[h], (u[h] + v[h] - 1) / c[h],
                                   [0.0]]))
    return int(hit.sum()), det[hit], ratio


def _edge_on(n, rng, O):
    """Triangle around a target point X with the ray O -> X meeting its plane
    at an angle of 1e-7 .. 0.3 rad."""
    X = np.stack([rng.uniform(0, 2.6667, n), rng.uniform(-1, 1, n), rng.uniform(0, 2, n)], 1)
    d = X - O
    D = d / d[:, 2:3]                                   # the camera's D.z = 1
    dh = d / np.linalg.norm(d, axis=1, keepdims=True)
    a = np.cross(dh, rng.normal(size=(n, 3)))
    a /= np.linalg.norm(a, axis=1, keepdims=True)
    th = 10.0 ** rng.uniform(-7, -0.5, n)[:, None]
    b = np.cos(th) * dh + np.sin(th) * np.cross(dh, a)
    size = rng.uniform(0.005, 0.08, (n, 1))
    al, be = rng.uniform(-0.3, 1.3, (n, 1)), rng.uniform(-0.3, 1.3, (n, 1))
    v0 = X - size * (al * a + be * b)
    v1, v2 = v0 + size * b, v0 + size * a
    flip = rng.random(n) < 0.5
    v1[flip], v2[flip] = v2[flip].copy(), v1[flip].copy()
    return v0, v1, v2, D


def test_miss_box_contains_every_accepted_ray_edge_on():
    rng = np.random.default_rng(5)
    O = np.array([2.0, 0.0, -2.0], F)
    hits, dets, worst = 0, [], 0.0
    for _ in range(8):
        v0, v1, v2, D = _edge_on(250_000, rng, O)
        # jitter the direction by a few ulps to a few 1e-4: rays that graze
        # the plane at other points
        D = D * (1 + rng.normal(size=D.shape) * 10.0 ** rng.uniform(-7, -3, (len(D), 1)))
        D[:, 2] = 1.0
        h, d, r = _check(v0, v1, v2, O, D)
        hits += h
        dets.append(d)
        worst = max(worst, r)
    dets = np.concatenate(dets)
    assert hits > 50_000
    assert (dets < 1e-5).sum() > 1000        # the near-threshold regime is exercised
    # accepted rays do land outside the plain triangle (rounding), by up to a
    # visible fraction of the bound: the check has teeth
    assert worst > 0.01, worst


def test_miss_box_contains_every_accepted_ray_soup():
    rng = np.random.default_rng(9)
    O = np.array([2.0, 0.0, -2.0], F)
    n = 400_000
    c = np.stack([rng.uniform(0, 2.6667, n), rng.uniform(-1, 1, n), rng.uniform(0, 2, n)], 1)
    v = c[:, None, :] + rng.uniform(-0.02, 0.02, (n, 3, 3))
    # rays aimed at points in and around each triangle
    w = rng.uniform(-0.2, 1.2, (n, 2))
    X = v[:, 0] + w[:, :1] * (v[:, 1] - v[:, 0]) + w[:, 1:] * (v[:, 2] - v[:, 0])
    D = (X - O) / (X - O)[:, 2:3]
    h, _, _ = _check(v[:, 0], v[:, 1], v[:, 2], O, D)
    assert h > 50_000


def _camera_dir(cam, u, v):
    """camera_dir (csrc/bih_render.hip), f32, no FMA: D = ((llc + u h) + v vert) - O."""
    c = np.asarray(cam, F)
    return np.stack([((c[3 + k] + u * c[6 + k]) + v * c[9 + k]) - c[k] for k in range(3)], 1).astype(F)


def _offset_cameras():
    """Reference-shaped cameras moved far from the origin (|O| up to 1e5 x |D|)
    and turned, where the f32 evaluation of D rounds by ulp(|llc|+|O|)."""
    out = []
    for o, hx, vy, sz in [((2.0, 0.0, -2.0), 3.5555556, 2.0, 1.0),
                          ((1000.0, -2000.0, 500.0), 3.5555556, 2.0, 1.0),
                          ((123456.7, 0.5, -98765.4), 2.6666667, 2.0, 1.0),
                          ((-3.0e4, 7.0e4, 1.0e3), 0.004, 0.003, 0.002)]:
        o = np.array(o, np.float64)
        llc = o + np.array([-hx / 2, -vy / 2, sz])
        out.append(np.concatenate([o, llc, [hx, 0, 0], [0, vy, 0]]).astype(F))
    return out


def test_camera_ray_bound_covers_kernel_directions(bihrt_mod):
    """bih_camera_ray_bound (the dmax the library sizes the miss-proof boxes
    with) bounds |D| of every primary ray as the kernel computes it, also for
    cameras far from the origin, whose f32 D rounds by ulp(|llc| + |O|)."""
    rng = np.random.default_rng(3)
    for cam in _offset_cameras():
        dmax = bihrt_mod.camera_ray_bound(bihrt_mod.Camera.from_list(cam.tolist()))
        g = np.linspace(0, 1, 257, dtype=F)
        u = np.concatenate([np.repeat(g, 257), rng.random(200_000).astype(F), [F(1), F(0)]])
        v = np.concatenate([np.tile(g, 257), rng.random(200_000).astype(F), [F(1), F(1)]])
        # the (u, v) the kernel forms: (x + r) / W with r in (0, 1]
        D = _camera_dir(cam, u.astype(F), v.astype(F))
        assert np.all(np.abs(D) <= dmax[None, :]), (cam, dmax, np.abs(D).max(0))


def test_miss_box_offset_origin_at_library_bound(bihrt_mod):
    """The miss-proof property at the library's own dmax (one bound for all
    rays of the camera, not the per-ray |D|) with an origin far from zero:
    near-edge-on triangles placed on the camera's own rays."""
    rng = np.random.default_rng(17)
    hits = 0
    for cam in _offset_cameras()[:3]:
        dmax = bihrt_mod.camera_ray_bound(bihrt_mod.Camera.from_list(cam.tolist()))
        O = cam[:3]
        n = 200_000
        D = _camera_dir(cam, rng.random(n).astype(F), rng.random(n).astype(F))
        X = O.astype(np.float64) + rng.uniform(0.5, 3.0, (n, 1)) * D.astype(np.float64)
        dh = D / np.linalg.norm(D.astype(np.float64), axis=1, keepdims=True)
        a = np.cross(dh, rng.normal(size=(n, 3)))
        a /= np.linalg.norm(a, axis=1, keepdims=True)
        th = 10.0 ** rng.uniform(-6, -0.5, n)[:, None]
        b = np.cos(th) * dh + np.sin(th) * np.cross(dh, a)
        size = rng.uniform(0.005, 0.08, (n, 1))
        al, be = rng.uniform(-0.3, 1.3, (n, 1)), rng.uniform(-0.3, 1.3, (n, 1))
        v0 = X - size * (al * a + be * b)
        v1, v2 = v0 + size * b, v0 + size * a
        flip = rng.random(n) < 0.5
        v1[flip], v2[flip] = v2[flip].copy(), v1[flip].copy()
        h, _, _ = _check(v0, v1, v2, O, D, dmax=dmax)
        hits += h
    assert hits > 20_000
