"""yakmo's prefix-chain fast path on the GPU against the sequential f32 chain.

The DLL's k-means++ seeding keeps the running f32 total cum[n] = fl(cum[n-1]
+ d[n]) over every point of a pick (yakmo_single.dll @0x1800016f0, SURVEY.md
App. C.1; restated in oracle/yakmo_oracle.c), and the next pick's
lower_bound searches it.  gsc_yakmo.hip's chain_fast replaces whole 64-point
blocks of that chain by one integer prefix sum while the total stays in one
binade, resolves round-half-even ties in place, runs negative totals on the
negated points and accepts leading all-zero blocks at a zero total.  The
whole-frame seeding tests cover it only through their end results; here the
kernel's own outputs -- accepted block count, checkpoints, per-block min /
max, the run after the accepted blocks -- are compared with numpy's
sequential float32 chain on crafted rings (tests/test_yakmo_chain_math.py
checks the same arithmetic on the CPU), through the C ABI
(gsc_yakmo_chain_test)."""
from __future__ import annotations

import ctypes

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def seq_chain(run: float, pts: np.ndarray):
    """cum after every point, sequential float32 (the DLL's order)."""
    cum = np.empty(len(pts), dtype=np.float32)
    r = np.float32(run)
    with np.errstate(all="ignore"):
        for i, d in enumerate(pts.astype(np.float32)):
            r = np.float32(r + d)
            cum[i] = r
    return cum


def gpu_chain(ppl: int, run: float, pts: np.ndarray):
    from soundchunks_amd import _lib

    lib = _lib.load()
    pts = np.ascontiguousarray(pts, dtype=np.float32)
    nbk = len(pts) // 64
    k = ctypes.c_int(-1)
    run_out = np.zeros(1, np.float32)
    ck, bmn, bmx = (np.zeros(nbk, np.float32) for _ in range(3))
    fp = lambda a: a.ctypes.data_as(ctypes.POINTER(ctypes.c_float))  # noqa: E731
    _lib.check(lib.gsc_yakmo_chain_test(ppl, fp(pts), nbk, ctypes.c_float(run), ctypes.byref(k), fp(run_out), fp(ck),
                                        fp(bmn), fp(bmx)))
    return k.value, float(run_out[0]), ck, bmn, bmx


def check(ppl: int, run: float, pts: np.ndarray, min_accept: int = 0):
    """Every accepted block equals the sequential chain bit for bit; returns k."""
    nbk = len(pts) // 64
    k, r, ck, bmn, bmx = gpu_chain(ppl, run, pts)
    assert 0 <= k <= nbk
    assert k >= min_accept, (k, min_accept)
    cum = seq_chain(run, pts)
    bits = lambda x: np.asarray(x, np.float32).view(np.uint32)  # noqa: E731
    for b in range(k):
        blk = cum[64 * b: 64 * b + 64]
        assert bits(ck[b]) == bits(blk[-1]), (b, ck[b], blk[-1])
        assert bits(bmn[b]) == bits(blk.min()), (b, bmn[b], blk.min())
        assert bits(bmx[b]) == bits(blk.max()), (b, bmx[b], blk.max())
    want_run = np.float32(run) if k == 0 else cum[64 * k - 1]
    assert bits(r) == bits(want_run), (r, want_run)
    return k


@pytest.mark.parametrize("ppl", [8, 16])
def test_ties_on_both_sides_of_a_lane_boundary(ppl):
    # run = 2^23 + 7: u = 1, d = +-0.5 are exact ties; put them at the last
    # point of lane 0 / first of lane 1, and across a 64-point block boundary
    nbk = ppl
    pts = np.ones(64 * nbk, np.float32) * np.float32(2.0)
    for i in (ppl - 1, ppl, 63, 64, 64 + ppl - 1, 64 + ppl):
        pts[i] = np.float32(0.5)
    pts[3 * ppl] = np.float32(-0.5)
    pts[3 * ppl + 1] = np.float32(0.5)
    check(ppl, 8388615.0, pts, min_accept=nbk)


@pytest.mark.parametrize("ppl", [8, 16])
def test_zero_run_with_signed_zero_points(ppl):
    nbk = ppl
    pts = np.zeros(64 * nbk, np.float32)
    pts[1::3] = np.float32(-0.0)
    pts[64 * 2 + 5] = np.float32(3.0)  # the first nonzero point: blocks 0 and 1 stay at +0
    k = check(ppl, 0.0, pts)
    assert k == 2
    # (a pick's total starts at +0 and a sum that cancels exactly is +0, so the
    # chain never runs from -0)


@pytest.mark.parametrize("ppl", [8, 16])
def test_negative_run(ppl):
    rng = np.random.default_rng(11)
    nbk = ppl
    pts = (rng.integers(-3, 4, 64 * nbk).astype(np.float32) * np.float32(0.25))
    pts[::17] = np.float32(-0.5)  # ties on the negated grid (u = 1 for |run| in [2^23, 2^24))
    check(ppl, -12000000.0, pts, min_accept=nbk)


@pytest.mark.parametrize("ppl", [8, 16])
@pytest.mark.parametrize("bad", [np.nan, np.inf, -np.inf])
def test_nonfinite_point_at_a_lane_start(ppl, bad):
    nbk = ppl
    pts = np.ones(64 * nbk, np.float32)
    pts[64 + ppl] = np.float32(bad)  # lane LPB + 1 starts with it: block 1 is refused, block 0 kept
    k = check(ppl, 9000000.0, pts)
    assert k == 1


@pytest.mark.parametrize("ppl", [8, 16])
def test_binade_crossing_mid_lane(ppl):
    nbk = ppl
    run = float(np.float32(2.0 ** 24 - 700.0))
    pts = np.ones(64 * nbk, np.float32) * np.float32(3.0)
    # block 0 adds 192 (stays below 2^24), block 1 crosses 2^24 - 2 in its middle
    pts[64:128] = np.float32(9.0)
    k = check(ppl, run, pts)
    assert k == 1


@pytest.mark.parametrize("ppl", [8, 16])
def test_random_rings_in_many_binades(ppl):
    rng = np.random.default_rng(2026)
    for trial in range(40):
        nbk = int(rng.integers(1, ppl + 1))
        e = int(rng.integers(-30, 40))
        run = float(np.float32(rng.uniform(1.0, 2.0) * 2.0 ** e * (1 if trial % 3 else -1)))
        u = 2.0 ** (e - 23)
        # multiples of u/2 (ties included), small against the run: long accepted prefixes
        pts = (rng.integers(-40, 41, 64 * nbk) * (u / 2)).astype(np.float32)
        check(ppl, run, pts)
