"""Batched speculative KNNScanReduce (gsc_scan.hip) and yakmo seeding
(gsc_yakmo.hip) at the benchmark shape K = 4096 / D = 16, against the oracle
(pytest -m gpu).  Stage parity on a real C2 frame, plus the generic kernel
forced through the same cases (GSC_SCAN_GENERIC) so both paths stay green.
"""
from __future__ import annotations

import os
import subprocess
import sys
from pathlib import Path

import numpy as np
import pytest

from golden.cases import CASES

pytestmark = pytest.mark.gpu
ROOT = Path(__file__).resolve().parents[1]


def _bits(a):
    return np.ascontiguousarray(a).view(np.uint32)


@pytest.fixture(scope="module")
def c2_trace(oracle):
    make, argv = CASES["syn2s_c2_cs8_cpf4096"]
    return oracle.trace_frame(make(), argv, 0)


def test_yakmo_k4096_bit_exact(c2_trace):
    import soundchunks_amd as sc

    c = sc.yakmo_seed_means(c2_trace["dataset"], c2_trace["K"])
    np.testing.assert_array_equal(_bits(c), _bits(c2_trace["yakmo"]))


@pytest.mark.parametrize("passes", [1, 3])
def test_scan_k4096_first_passes(oracle, c2_trace, passes):
    import soundchunks_amd as sc

    os.environ["GSC_SCAN_MAX_PASSES"] = str(passes)
    try:
        gc, gcl, gn = sc.scan_reduce(c2_trace["dataset"], c2_trace["yakmo"], precision=3)
    finally:
        del os.environ["GSC_SCAN_MAX_PASSES"]
    oc, ocl, on = oracle.scan_reduce(c2_trace["dataset"], c2_trace["yakmo"], 3, passes)
    assert gn == on == passes
    np.testing.assert_array_equal(gcl, ocl)
    np.testing.assert_array_equal(_bits(gc), _bits(oc))


def test_scan_k4096_full(c2_trace):
    import soundchunks_amd as sc

    gc, gcl, gn = sc.scan_reduce(c2_trace["dataset"], c2_trace["yakmo"], precision=3)
    assert gn == c2_trace["scan_iters"]
    np.testing.assert_array_equal(gcl, c2_trace["clusters"])
    np.testing.assert_array_equal(_bits(gc), _bits(c2_trace["scan"]))


@pytest.fixture(scope="module")
def c3_trace(oracle):
    make, argv = CASES["syn8s_c3_cs16_cpf4096_cbd12"]
    return oracle.trace_frame(make(), argv, 0)


@pytest.mark.parametrize("passes", [1, 3])
def test_scan_k4096_d32_first_passes(oracle, c3_trace, passes):
    """D = 32 (ChunkSize 16) at K = 4096: one CU per frame in the split layout
    (DCT half of each centroid in VGPRs, cepstrum half in the frame's tail array)."""
    import soundchunks_amd as sc

    os.environ["GSC_SCAN_MAX_PASSES"] = str(passes)
    try:
        gc, gcl, gn = sc.scan_reduce(c3_trace["dataset"], c3_trace["yakmo"], precision=3)
    finally:
        del os.environ["GSC_SCAN_MAX_PASSES"]
    oc, ocl, on = oracle.scan_reduce(c3_trace["dataset"], c3_trace["yakmo"], 3, passes)
    assert gn == on == passes
    np.testing.assert_array_equal(gcl, ocl)
    np.testing.assert_array_equal(_bits(gc), _bits(oc))


def test_scan_k4096_d32_full(c3_trace):
    import soundchunks_amd as sc

    gc, gcl, gn = sc.scan_reduce(c3_trace["dataset"], c3_trace["yakmo"], precision=3)
    assert gn == c3_trace["scan_iters"]
    np.testing.assert_array_equal(gcl, c3_trace["clusters"])
    np.testing.assert_array_equal(_bits(gc), _bits(c3_trace["scan"]))


@pytest.mark.parametrize("k", [256, 2048, 3000])
def test_scan_d32_one_cu(oracle, c3_trace, k):
    """D = 32: K <= 2048 keeps every feature in VGPRs (4 leaves per lane); K = 3000
    runs the split layout over the padded 4096-leaf tree."""
    import soundchunks_amd as sc

    x = c3_trace["dataset"][:6000]
    c0 = sc.yakmo_seed_means(x, k)
    gc, gcl, gn = sc.scan_reduce(x, c0, precision=3)
    oc, ocl, on = oracle.scan_reduce(x, c0, 3, 100)
    assert gn == on
    np.testing.assert_array_equal(gcl, ocl)
    np.testing.assert_array_equal(_bits(gc), _bits(oc))


@pytest.mark.parametrize("name", ["hihat_cs8_cpf256", "silence_tone_cs8_cpf256", "quiet_tone_cs8_cpf1024"])
def test_generic_scan_kernel_still_exact(name):
    # the generic per-search kernel (non-power-of-2 K, NaN passes) on its own
    code = (f"import sys; sys.path[:0]=[{str(ROOT)!r},{str(ROOT / 'tests')!r}];"
            "import soundchunks_amd as sc; from golden.cases import CASES, golden_path;"
            f"m,a=CASES[{name!r}]; assert sc.Encoder(a).encode(m())==golden_path({name!r}).read_bytes()")
    env = dict(os.environ, GSC_SCAN_GENERIC="1")
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]


def test_scan_nan_centroids_k4096(oracle):
    """A frame with NaN centroids (the corpus' 60.wav: yakmo 0/0 means of seeds
    that won no point) in the batched kernel: NaN-first descents, dead low
    children of NaN cuts, the NaN-exact tree build and the exact LDS-stack DFS,
    first passes against the oracle (NaN rows compared as NaN)."""
    import soundchunks_amd as sc

    wav = (ROOT / "tests" / "golden" / "lame_test" / "60.wav").read_bytes()
    t = oracle.trace_frame(wav, ["-cs8", "-cpf4096"], 1)
    assert int(np.isnan(t["yakmo"]).any(axis=1).sum()) > 1000
    os.environ["GSC_SCAN_MAX_PASSES"] = "3"
    try:
        gc, gcl, gn = sc.scan_reduce(t["dataset"], t["yakmo"], precision=3)
    finally:
        del os.environ["GSC_SCAN_MAX_PASSES"]
    oc, ocl, on = oracle.scan_reduce(t["dataset"], t["yakmo"], 3, 3)
    assert gn == on == 3
    np.testing.assert_array_equal(gcl, ocl)
    nan = np.isnan(oc)
    np.testing.assert_array_equal(np.isnan(gc), nan)
    np.testing.assert_array_equal(_bits(np.where(nan, 0, gc)), _bits(np.where(nan, 0, oc)))


@pytest.mark.parametrize("d,k", [(8, 1024), (8, 4096), (16, 4096)])
def test_scan_integer_grid_ties_match_oracle(oracle, d, k):
    """Integer-valued features with duplicate points: exact distance ties
    everywhere, so many batch queries get no certificate (no unique minimum)
    and take ANN's own DFS answer on the snapshot (gsc_scan.hip's in-batch
    DFS answers, checked at the commit by dfs_keeps), and moved centroids
    land on exact ties with them.  Three passes, bit-exact against the oracle's
    KNNScanReduce (encoder.lpr:699-765 over ANN's stale tree)."""
    import soundchunks_amd as sc

    rng = np.random.default_rng(7 + d + k)
    n = 24000
    x = rng.integers(-6, 7, size=(n, d)).astype(np.float32)
    x[::5] = x[1::5][: len(x[::5])]  # runs of duplicate points
    c0 = x[rng.choice(n, k, replace=False)] + rng.integers(-1, 2, size=(k, d)).astype(np.float32) * 0.5
    os.environ["GSC_SCAN_MAX_PASSES"] = "3"
    try:
        gc, gcl, gn = sc.scan_reduce(x, c0, precision=3)
    finally:
        del os.environ["GSC_SCAN_MAX_PASSES"]
    oc, ocl, on = oracle.scan_reduce(x, c0, 3, 3)
    assert gn == on
    np.testing.assert_array_equal(gcl, ocl)
    np.testing.assert_array_equal(_bits(gc), _bits(oc))
