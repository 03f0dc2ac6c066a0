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
    return out
