"""Deterministic synthetic scenes for the BASELINE.json configs.

Scenes are flat triangle soups: float32 arrays of shape (n, 9) holding
v0, v1, v2 per triangle in "file order" -- the layout App::LoadModels builds
(reference src/App.cpp:108-121).  Every generator is counter-based
(splitmix64), so this container and the GPU box produce identical bytes.

C1 cornell():   32-tri Cornell box (5 walls, 2 blocks x 5 faces, light).
C2 torus():     ~70k-tri closed torus (procedural stand-in: the Stanford
                Bunny is not available offline).
C3 soup():      1M random-triangle soup, centroids U([0,2.667]x[-1,1]x[0,2]),
                vertices = centroid + U(-0.02,0.02)^3, seed 1.
"""
from __future__ import annotations

import numpy as np

_GOLD = np.uint64(0x9E3779B97F4A7C15)


def splitmix64(seed: int, start: int, count: int) -> np.ndarray:
    """Outputs start..start+count-1 of splitmix64 seeded with `seed`."""
    k = np.arange(start + 1, start + count + 1, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = np.uint64(seed) + k * _GOLD
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    return z


def uniform01(seed: int, start: int, count: int) -> np.ndarray:
    """24-bit uniforms in [0,1), exact in float32 and float64."""
    return (splitmix64(seed, start, count) >> np.uint64(40)).astype(np.float64) * (2.0 ** -24)


def soup(n: int = 1_000_000, seed: int = 1, lo=(0.0, -1.0, 0.0), size=(2.6666667, 2.0, 2.0),
         half: float = 0.02) -> np.ndarray:
    """Random triangle soup (config C3/C5).  12 uniforms per triangle:
    3 for the centroid, then 9 for the vertex offsets (v0.xyz, v1.xyz, v2.xyz)."""
    u = uniform01(seed, 0, 12 * n).reshape(n, 12)
    c = np.asarray(lo, np.float64) + u[:, 0:3] * np.asarray(size, np.float64)
    off = (u[:, 3:12] * (2.0 * half) - half).reshape(n, 3, 3)
    v = c[:, None, :] + off
    return np.ascontiguousarray(v.reshape(n, 9).astype(np.float32))


def _quad(a, b, c, d):
    """Two CCW triangles (a,b,c), (a,c,d) of the quad a-b-c-d."""
    return [a + b + c, a + c + d]


def cornell() -> np.ndarray:
    """32 triangles: 5 walls x2, 2 blocks x 5 faces x2, ceiling light x2.
    Front faces (CCW seen from inside) point into the box, towards the
    reference camera at (2,0,-2) looking down +z (MT culls back faces)."""
    x0, x1, y0, y1, z0, z1 = -1.0, 1.9, -1.0, 1.0, 0.0, 2.4
    P = lambda x, y, z: [x, y, z]  # noqa: E731
    tris = []
    # back wall z=z1, normal -z (faces the camera)
    tris += _quad(P(x0, y0, z1), P(x0, y1, z1), P(x1, y1, z1), P(x1, y0, z1))
    # floor y=y0, normal +y
    tris += _quad(P(x0, y0, z0), P(x0, y0, z1), P(x1, y0, z1), P(x1, y0, z0))
    # ceiling y=y1, normal -y
    tris += _quad(P(x0, y1, z0), P(x1, y1, z0), P(x1, y1, z1), P(x0, y1, z1))
    # left wall x=x0, normal +x
    tris += _quad(P(x0, y0, z0), P(x0, y1, z0), P(x0, y1, z1), P(x0, y0, z1))
    # right wall x=x1, normal -x
    tris += _quad(P(x1, y0, z0), P(x1, y0, z1), P(x1, y1, z1), P(x1, y1, z0))

    def block(cx, cz, hw, hgt, rot):
        cs, sn = np.cos(rot), np.sin(rot)

        def p(dx, y, dz):
            return [cx + cs * dx - sn * dz, y, cz + sn * dx + cs * dz]
        a, b, c, d = (-hw, -hw), (hw, -hw), (hw, hw), (-hw, hw)
        yb, yt = y0, y0 + hgt
        out = []
        # top, normal +y
        out += _quad(p(a[0], yt, a[1]), p(d[0], yt, d[1]), p(c[0], yt, c[1]), p(b[0], yt, b[1]))
        # four sides, outward normals
        for (u0, u1) in ((a, b), (b, c), (c, d), (d, a)):
            out += _quad(p(u0[0], yb, u0[1]), p(u1[0], yb, u1[1]), p(u1[0], yt, u1[1]), p(u0[0], yt, u0[1]))
        return out
    tris += block(-0.2, 1.6, 0.35, 1.2, 0.3)
    tris += block(0.9, 0.9, 0.3, 0.6, -0.3)
    # light, just below the ceiling, normal -y
    ly = y1 - 0.01
    tris += _quad(P(0.1, ly, 1.0), P(0.7, ly, 1.0), P(0.7, ly, 1.6), P(0.1, ly, 1.6))
    v = np.asarray(tris, np.float64).astype(np.float32)
    assert v.shape == (32, 9), v.shape
    return np.ascontiguousarray(v)


def torus(nu: int = 263, nv: int = 132, R: float = 1.0, r: float = 0.35,
          center=(0.3, 0.0, 1.5), tilt: float = 0.6) -> np.ndarray:
    """Closed torus, 2*nu*nv triangles (69,432 at the defaults), outward CCW."""
    iu, iv = np.meshgrid(np.arange(nu), np.arange(nv), indexing="ij")
    th = 2 * np.pi * np.arange(nu + 1) / nu
    ph = 2 * np.pi * np.arange(nv + 1) / nv
    T, Pm = np.meshgrid(th, ph, indexing="ij")
    X = (R + r * np.cos(Pm)) * np.cos(T)
    Y = (R + r * np.cos(Pm)) * np.sin(T)
    Z = r * np.sin(Pm)
    ct, st = np.cos(tilt), np.sin(tilt)
    Y, Z = ct * Y - st * Z, st * Y + ct * Z
    pts = np.stack([X + center[0], Y + center[1], Z + center[2]], -1)
    a = pts[iu, iv]
    b = pts[iu + 1, iv]
    c = pts[iu + 1, iv + 1]
    d = pts[iu, iv + 1]
    t1 = np.concatenate([a, b, c], -1)
    t2 = np.concatenate([a, c, d], -1)
    v = np.stack([t1, t2], 2).reshape(-1, 9)
    return np.ascontiguousarray(v.astype(np.float32))


def dodecahedron(start=None, variant: int = 0) -> np.ndarray:
    """Regular dodecahedron, circumradius 1, 12 pentagons fan-triangulated
    (assimp aiProcess_Triangulate, reference src/Model.cpp:13) -> 36 tris.
    `start[f]` picks the fan apex of face f (0..4); variant selects one of the
    two standard axis orientations."""
    phi = (1 + 5 ** 0.5) / 2
    s = 1 / 3 ** 0.5
    V = []
    for x in (-1, 1):
        for y in (-1, 1):
            for z in (-1, 1):
                V.append((x, y, z))
    a, b = 1 / phi, phi
    if variant == 1:
        a, b = b, a
    for i in (-1, 1):
        for j in (-1, 1):
            V.append((0, i * a, j * b))
            V.append((i * a, j * b, 0))
            V.append((i * b, 0, j * a))
    V = np.asarray(V, np.float64) * s
    faces = _dodeca_faces(V)
    if start is None:
        start = [0] * 12
    tris = []
    for f, st in zip(faces, start):
        f = list(f[st:]) + list(f[:st])
        for k in range(1, 4):
            tris.append(np.concatenate([V[f[0]], V[f[k]], V[f[k + 1]]]))
    return np.ascontiguousarray(np.asarray(tris).astype(np.float32)), faces, V


# Fan apex per face (variant 1) of the one triangulation, out of 5^12 per
# orientation and vertex precision, whose BIH reproduces the reference's own
# tree dump node for node (BIH1.txt:1-348; search: tests/golden/
# make_bih1_soup.py, record: tests/golden/bih1_dodecahedron.json).
BIH1_APEX = (1, 4, 4, 0, 3, 3, 3, 1, 3, 0, 4, 1)


def dodecahedron_bih1() -> np.ndarray:
    """The reference's 36-triangle dodecahedron (the mesh behind BIH1.txt),
    recovered by exhaustive search; 36 x 9 float32."""
    return dodecahedron(start=BIH1_APEX, variant=1)[0]


def _dodeca_faces(V):
    """12 pentagonal faces as CCW (outward) vertex cycles."""
    d = np.linalg.norm(V[:, None] - V[None], axis=-1)
    edge = np.min(d[d > 1e-9])
    adj = np.abs(d - edge) < 1e-6
    seen, out = set(), []
    for i in range(len(V)):
        nb = np.nonzero(adj[i])[0]
        for a_ in range(len(nb)):
            for b_ in range(a_ + 1, len(nb)):
                j, k = nb[a_], nb[b_]
                nrm = np.cross(V[j] - V[i], V[k] - V[i])
                nrm /= np.linalg.norm(nrm)
                if np.dot(nrm, V[i]) < 0:
                    nrm = -nrm
                on = np.nonzero(np.abs((V - V[i]) @ nrm) < 1e-6)[0]
                key = frozenset(int(x) for x in on)
                if len(on) != 5 or key in seen:
                    continue
                seen.add(key)
                cen = V[on].mean(0)
                e0 = V[on[0]] - cen
                e0 /= np.linalg.norm(e0)
                e1 = np.cross(nrm, e0)
                ang = np.arctan2((V[on] - cen) @ e1, (V[on] - cen) @ e0)
                out.append([int(x) for x in on[np.argsort(ang)]])
    assert len(out) == 12, len(out)
    return out


def write_obj(path: str, tris: np.ndarray, shared: bool = False):
    """Writes a soup as Wavefront OBJ (numpy's shortest round-trip float32
    repr per coordinate).  shared=False: three `v` lines + one `f` per triangle;
    shared=True: identical vertices are written once and referenced by index."""
    tris = np.asarray(tris, np.float32).reshape(-1, 3, 3)
    with open(path, "w") as f:
        f.write(f"# {tris.shape[0]} triangles\no soup\n")
        if not shared:
            for t in tris:
                for p in t:
                    f.write("v %s %s %s\n" % tuple(str(x) for x in p))
            for i in range(tris.shape[0]):
                f.write("f %d %d %d\n" % (3 * i + 1, 3 * i + 2, 3 * i + 3))
            return
        verts, idx = np.unique(tris.reshape(-1, 3).view(np.uint32), axis=0, return_inverse=True)
        for p in verts.view(np.float32):
            f.write("v %s %s %s\n" % tuple(str(x) for x in p))
        for t in idx.reshape(-1, 3):
            f.write("f %d %d %d\n" % tuple(int(k) + 1 for k in t))
