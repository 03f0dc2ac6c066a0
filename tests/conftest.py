"""Shared test setup.

`-m "not gpu"` tests run anywhere (oracle vs golden vectors, host logic, the
C-ABI library's exports).  `-m gpu` tests are the parity tests proper: they
call the HIP path through the C ABI and compare with the oracle.
"""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "bih-gpu-raytracer_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a HIP device (MI355X); runs the HIP path")


@pytest.fixture(scope="session")
def oracle_mod():
    import oracle
    return oracle


@pytest.fixture(scope="session")
def bihrt_mod():
    import bihrt
    return bihrt


@pytest.fixture(scope="session")
def gpu(bihrt_mod):
    """Skips nothing: a gpu-marked test on a box without a device must fail."""
    n = bihrt_mod.device_count()
    assert n > 0, "no HIP device visible to libbih_amd.so"
    return 0


def edge_scenes():
    """Small scenes exercising the reference's corner cases."""
    from bihrt import scenes as S
    out = {}
    out["one_tri"] = np.array([[0.2, -0.5, 1.0, 1.5, -0.5, 1.0, 0.8, 0.6, 1.0]], np.float32)
    out["two_tris"] = np.concatenate([out["one_tri"], out["one_tri"] + np.float32(0.3)])
    # all triangles share one Morton code (duplicates, U=1 with N>1)
    base = out["one_tri"][0]
    out["dup_all"] = np.stack([base, base, base], 0).astype(np.float32)
    # many duplicates (counts > 3 exercise the escape path)
    rng = np.random.default_rng(7)
    cells = rng.integers(0, 6, size=(300, 3)).astype(np.float32) * np.float32(0.4)
    jit = rng.uniform(-0.01, 0.01, size=(300, 9)).astype(np.float32)
    tri = np.tile(cells, 3) + jit
    tri[:, 3] += 0.05
    tri[:, 7] += 0.05
    out["clustered"] = tri.astype(np.float32)
    # flat scene (zero extent in z): normalisation divides 0/0 -> NaN -> code 0
    flat = S.soup(500, seed=3)
    flat[:, 2::3] = np.float32(1.0)
    out["flat_z"] = flat
    # signed zeros on bounding coordinates
    sz = S.soup(200, seed=5, lo=(-1.0, -1.0, 0.0), size=(2.0, 2.0, 2.0))
    sz[::7, 0] = np.float32(-0.0)
    sz[::11, 4] = np.float32(0.0)
    sz[3, :] = np.array([-0.0, -1.0, 0.0, 0.0, 1.0, 0.0, 0.5, 0.0, -0.0], np.float32)
    out["signed_zero"] = sz
    out["cornell"] = S.cornell()
    out["dodeca"] = S.dodecahedron()[0]
    out["bih1_dodeca"] = S.dodecahedron_bih1()
    return out


def parse_bih1_dump(path=None):
    """The reference's tree dump (BIH1.txt:1-348): one dict per node."""
    nodes, cur = [], None
    for line in open(path or os.path.join(GOLDEN, "reference_BIH1.txt")):
        line = line.strip()
        if line.startswith("NODE"):
            cur = {"id": int(line.split()[1])}
            nodes.append(cur)
        elif ":" in line and cur is not None:
            k, v = [x.strip() for x in line.split(":", 1)]
            cur[k] = v
    return nodes


def bih1_mismatches(parent, children, axis, is_leaf, clip):
    """(node, field) pairs where a built tree differs from BIH1.txt.  All 8
    printed fields per node; clip planes compared at the dump's printed
    precision (std::cout default, %g with 6 significant digits, as the
    reference's printer at src/Renderer.cpp:617-636 writes them)."""
    bad = []
    for n in parse_bih1_dump():
        i = n["id"]
        got = {"parent": str(int(parent[i])), "leftChild": str(int(children[i][0])),
               "rightChild": str(int(children[i][1])), "axis": str(int(axis[i])),
               "isLeftLeaf": "TRUE" if is_leaf[i][0] else "FALSE",
               "isRightLeaf": "TRUE" if is_leaf[i][1] else "FALSE",
               "clipPlaneLEFT": "%g" % float(clip[i][0]),
               "clipPlaneRIGHT": "%g" % float(clip[i][1])}
        bad += [(i, k) for k, v in got.items() if n[k] != v]
    return bad
