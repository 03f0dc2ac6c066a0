"""The division-free pre-test of the packet walk's Moeller-Trumbore
(csrc/bih_packet_asm.h, BIH_MT) may only drop lanes the exact test drops:
un < -det*2^-20 must give u = un * (1/det) < 0, and un > det*(1+2^-20) must
give u > 1, in f32 with IEEE division (CUDAKernels.cu:33-40).  Checked on
dense f32 neighbourhoods of both thresholds over det spanning (eps, 2^40)."""
import numpy as np

EPS = np.float32(np.uint32(0x358637BD).view(np.float32))
LO = np.float32(2.0 ** -20)
HI = np.float32(1.0 + 2.0 ** -20)


def _around(x, k=64):
    """x and its k f32 neighbours on each side."""
    x = np.asarray(x, np.float32)
    bits = x.view(np.int32)[:, None] + np.arange(-k, k + 1, dtype=np.int32)[None, :]
    return bits.astype(np.int32).view(np.float32)


def test_prefilter_drops_only_exact_misses():
    rng = np.random.default_rng(7)
    det = np.concatenate([
        np.float32(EPS) * (1 + rng.random(2000, dtype=np.float32)),
        (2.0 ** rng.uniform(-19, 40, 20000)).astype(np.float32),
        np.array([np.nextafter(EPS, np.float32(np.inf))], np.float32),
    ]).astype(np.float32)
    with np.errstate(over="ignore", invalid="ignore"):
        inv = (np.float32(1.0) / det).astype(np.float32)
        lo = (det * LO).astype(np.float32)
        hi = (det * HI).astype(np.float32)
        for centre, at_threshold in ((-lo, True), (hi, True), (np.float32(0) * det, False),
                                     (det, False)):
            un = _around(centre)
            u = (un * inv[:, None]).astype(np.float32)
            drop = (un < -lo[:, None]) | (un > hi[:, None])
            exact_drop = (u < 0) | (u > 1)
            assert not np.any(drop & ~exact_drop)
            if at_threshold:
                assert drop.sum() > 0


def test_prefilter_keeps_nonfinite():
    det = np.array([np.inf, np.nan, 1.0], np.float32)
    un = np.array([1e30, 0.5, np.nan], np.float32)
    with np.errstate(invalid="ignore"):
        lo = det * LO
        hi = det * HI
        drop = (un < -lo) | (un > hi)
    assert not drop.any()
