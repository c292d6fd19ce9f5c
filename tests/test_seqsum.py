"""gsc_seqsum.h: the parallel evaluation of a sequential f64 sum must be
bit-identical to the one-term-at-a-time loop (PrepareFrames' power sums,
encoder.lpr:1374-1389) -- including ties to even on the binade grid, binade
crossings inside a block, sign changes, and non-finite terms."""
from __future__ import annotations

import ctypes
import subprocess
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parents[1]

HARNESS = r'''
#include "%s"
#include <thread>
#include <atomic>
static gsc::SeqSumStats g_st;
extern "C" long stat_fast() { return long(g_st.fast_blocks); }
extern "C" long stat_ties() { return long(g_st.ties); }
extern "C" double par_sum(const double* t, long n, double s0, long block) {
    auto par = [](int nb, const auto& fn) {
        std::atomic<int> next{0};
        std::vector<std::thread> th;
        for (int k = 0; k < 4; ++k) th.emplace_back([&] { for (int i; (i = next++) < nb;) fn(i); });
        for (auto& x : th) x.join();
    };
    return gsc::exact_seq_sum(n, s0, [&](int64_t a, int64_t b, double* o) { for (int64_t i = a; i < b; ++i) o[i - a] = t[i]; }, par, block, &g_st);
}
extern "C" double seq_sum(const double* t, long n, double s0) {
    double s = s0;
    for (long i = 0; i < n; ++i) s = s + t[i];
    return s;
}
'''


@pytest.fixture(scope="module")
def lib(tmp_path_factory):
    d = tmp_path_factory.mktemp("seqsum")
    src = d / "h.cpp"
    src.write_text(HARNESS % (ROOT / "soundchunks_amd" / "csrc" / "gsc_seqsum.h"))
    so = d / "h.so"
    subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-shared", "-fPIC", "-pthread", "-o", str(so),
                    str(src)], check=True)
    L = ctypes.CDLL(str(so))
    L.par_sum.restype = ctypes.c_double
    L.par_sum.argtypes = [ctypes.c_void_p, ctypes.c_long, ctypes.c_double, ctypes.c_long]
    L.seq_sum.restype = ctypes.c_double
    L.seq_sum.argtypes = [ctypes.c_void_p, ctypes.c_long, ctypes.c_double]
    L.stat_fast.restype = ctypes.c_long
    L.stat_ties.restype = ctypes.c_long
    return L


def _gen(kind, rng, n):
    if kind == "squares":  # avgPower's terms: (s/32767)^2
        v = rng.integers(-32768, 32768, n) / 32767.0
        return v * v
    if kind == "dyadic":  # few-bit terms: exact ties on the binade grid
        return rng.integers(0, 64, n) * np.ldexp(1.0, -int(rng.integers(1, 12)))
    if kind == "dyadic_mixed":
        return rng.integers(-40, 64, n) * np.ldexp(1.0, -int(rng.integers(1, 12)))
    if kind == "pw":  # 1 - RMS, in [0, 1], a few tiny negatives
        v = 1.0 - np.abs(rng.standard_normal(n)) * 0.3
        v[rng.integers(0, n, 5)] = -2e-16
        return v
    if kind == "wide":  # magnitudes over many binades, both signs
        return rng.standard_normal(n) * np.exp(rng.uniform(-30, 30, n))
    if kind == "dyadic_tie":  # used with s0 = 2^50 (grid 1/4): half the terms are exact ties
        return rng.integers(-3, 16, n) * 0.125
    if kind == "nonfinite":
        v = rng.random(n)
        v[n // 2] = np.inf
        return v
    raise ValueError(kind)


@pytest.mark.parametrize("kind", ["squares", "dyadic", "dyadic_mixed", "dyadic_tie", "pw", "wide", "nonfinite"])
def test_parallel_sum_is_the_sequential_sum(lib, kind):
    rng = np.random.default_rng(sum(map(ord, kind)))
    f0, t0 = lib.stat_fast(), lib.stat_ties()
    for trial in range(12):
        n = int(rng.integers(1, 300_000))
        t = np.ascontiguousarray(_gen(kind, rng, n))
        s0 = [0.0, 1.0, 1e6, -3.5, 0.0][trial % 5]
        if kind == "dyadic_tie":
            s0 = 2.0**50 + [0.0, 0.25, 0.5, 1.75][trial % 4]
        for block in (64, 1000, 8192):
            got = lib.par_sum(t.ctypes.data, n, s0, block)
            want = lib.seq_sum(t.ctypes.data, n, s0)
            assert np.float64(got).tobytes() == np.float64(want).tobytes() or (np.isnan(got) and np.isnan(want)), \
                (kind, trial, block, got, want)
    if kind in ("squares", "pw", "dyadic_tie"):
        assert lib.stat_fast() > f0  # the grid path ran (not only the term-by-term fallback)
    if kind == "dyadic_tie":
        assert lib.stat_ties() > t0
