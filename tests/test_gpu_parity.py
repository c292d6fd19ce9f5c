"""HIP path vs oracle, byte for byte (run on a real MI355X: pytest -m gpu).

Stage-level parity (yakmo seeding, KNNScanReduce, KNNFit) on oracle traces
of real frames, and whole-file .gsc parity against the committed golden
fixtures (tests/golden, produced by the C oracle).
"""
from __future__ import annotations

import numpy as np
import pytest

from golden.cases import CASES, golden_path

pytestmark = pytest.mark.gpu


def _bits(a):
    return np.ascontiguousarray(a).view(np.uint32)


def _trace(oracle, name, frame=0):
    make, argv = CASES[name]
    return oracle.trace_frame(make(), argv, frame)


@pytest.mark.parametrize("name", ["c1_test_cs8_cpf256", "silence_tone_cs8_cpf256"])
def test_yakmo_seed_means_bit_exact(oracle, name):
    import soundchunks_amd as sc

    tr = _trace(oracle, name)
    if tr["N"] <= tr["K"]:
        pytest.skip("passthrough frame")
    c = sc.yakmo_seed_means(tr["dataset"], tr["K"])
    np.testing.assert_array_equal(_bits(c), _bits(tr["yakmo"]))


@pytest.mark.parametrize("name", ["c1_test_cs8_cpf256", "silence_tone_cs8_cpf256", "hihat_cs4_default"])
def test_scan_reduce_bit_exact(oracle, name):
    import soundchunks_amd as sc

    tr = _trace(oracle, name)
    if tr["N"] <= tr["K"]:
        pytest.skip("passthrough frame")
    c, cl, passes = sc.scan_reduce(tr["dataset"], tr["yakmo"], precision=3)
    assert passes == tr["scan_iters"]
    np.testing.assert_array_equal(cl, tr["clusters"])
    np.testing.assert_array_equal(_bits(c), _bits(tr["scan"]))


@pytest.mark.parametrize("name", ["c1_test_cs8_cpf256", "hihat_cs8_cpf256", "silence_tone_cs8_cpf256"])
def test_knnfit_bit_exact(oracle, name):
    import soundchunks_amd as sc

    tr = _trace(oracle, name)
    cand = tr["knn_cand"]
    fwd = cand[0::4]  # forward, non-negated variant of every reduced chunk
    best = sc.knnfit_assign(fwd, tr["knn_query"], tr["knn_eps"])
    np.testing.assert_array_equal(best, tr["knn_best"])


@pytest.mark.parametrize("name", ["quiet_tone_cs8_cpf1024", "quiet_tone_cs4_cpf1024"])
def test_knnfit_bucket_overflow_follows_ann_order(oracle, name):
    """Queries in near-silence tie with thousands of all-zero candidates: the
    64-NN bucket holds the first 64 ANN's priority search meets, and the tie
    rule picks the smallest index among those (encoder.lpr:945-958) -- the
    GPU path replays that search for exactly these queries."""
    import soundchunks_amd as sc

    tr = _trace(oracle, name)
    cand, q, eps, cs = tr["knn_cand"], tr["knn_query"], tr["knn_eps"], tr["CS"]
    # the case must actually overflow the bucket (> 64 candidates within eps)
    zero = int((np.abs(cand).sum(axis=1) == 0).sum())
    assert zero > 64
    best = sc.knnfit_assign(cand[0::4], q, eps)
    np.testing.assert_array_equal(best, tr["knn_best"])
    # a brute-force "smallest index among all ties" differs on some of them
    quiet = np.abs(q).sum(axis=1) == 0
    assert quiet.any()
    assert (tr["knn_best"][quiet] > np.flatnonzero(np.abs(cand).sum(axis=1) == 0)[0]).any()


def test_knnfit_overflow_replay_twice_per_stream(oracle):
    """ADVICE r04 regression: the ANN replay of bucket-overflow queries runs
    twice in one process on the null stream (the synchronous stage entry
    point) and twice on the encoder's non-blocking post-processing stream,
    interleaved.  Its device scratch is poison-filled before every replay
    (gsc_runtime.cpp DevArena) and the replay kernel bounds-checks every node,
    segment and point index, so a stale or uninitialised read shows up as a
    wrong answer or a -4 failure here instead of hiding behind zero pages."""
    import soundchunks_amd as sc

    name = "quiet_tone_cs8_cpf1024"
    tr = _trace(oracle, name)
    make, argv = CASES[name]
    wav, expected = make(), golden_path(name).read_bytes()
    for _ in range(2):
        best = sc.knnfit_assign(tr["knn_cand"][0::4], tr["knn_query"], tr["knn_eps"])
        np.testing.assert_array_equal(best, tr["knn_best"])
        assert sc.Encoder(argv).encode(wav) == expected
        assert sc.Encoder.last_timing()["knnfit_overflow"] > 0  # the encoder's stream did replay


@pytest.mark.parametrize("name", sorted(CASES))
def test_gsc_matches_golden(name):
    import soundchunks_amd as sc

    make, argv = CASES[name]
    expected = golden_path(name).read_bytes()
    got = sc.Encoder(argv).encode(make())
    assert len(got) == len(expected)
    assert got == expected


def _yakmo_dataset(kind, n, d, seed):
    rng = np.random.default_rng(seed)
    if kind == "gauss":
        return rng.standard_normal((n, d)).astype(np.float32) * 50.0
    if kind == "integer":  # many equal distances and duplicate points (zero / tiny negative d)
        return rng.integers(-3, 4, size=(n, d)).astype(np.float32)
    if kind == "outliers":  # a few huge points: the prefix jumps across many binades at once
        x = rng.standard_normal((n, d)).astype(np.float32)
        x[rng.integers(0, n, size=n // 500)] *= 1e4
        return x
    raise ValueError(kind)


@pytest.mark.parametrize("kind,n,d,k", [("gauss", 5000, 16, 256), ("integer", 3000, 16, 512),
                                        ("outliers", 7000, 8, 256), ("gauss", 20000, 16, 1024),
                                        # more than 262,144 points: bitmap and prefix summaries in HBM
                                        ("gauss", 300000, 8, 256), ("integer", 270000, 16, 256)])
def test_yakmo_seed_means_synthetic(oracle, kind, n, d, k):
    """The binade-exact prefix fast path (gsc_yakmo.hip) against the oracle's sequential f32 chain."""
    import ctypes

    import soundchunks_amd as sc

    x = _yakmo_dataset(kind, n, d, 1234 + n)
    want = np.zeros((k, d), dtype=np.float32)
    labels = np.zeros(n, dtype=np.int32)
    fp = ctypes.POINTER(ctypes.c_float)
    rc = oracle.load().ora_yakmo_seed_means(n, d, x.ctypes.data_as(fp), k, want.ctypes.data_as(fp),
                                            labels.ctypes.data_as(ctypes.POINTER(ctypes.c_int)))
    assert rc == 0
    got = sc.yakmo_seed_means(x, k)
    np.testing.assert_array_equal(_bits(got), _bits(want))


@pytest.mark.parametrize("cs,r,n,eps,seed", [(8, 600, 3000, 0.0026, 1), (8, 4096, 2000, 1.0 / 32767, 2),
                                             (4, 300, 2500, 0.01, 3), (16, 1000, 1500, 0.004, 4)])
def test_knnfit_synthetic_ties(oracle, cs, r, n, eps, seed):
    """Bound-then-exact KNNFit (gsc_kernels.hip) vs the oracle's ANN 64-NN + tie rule on
    8-bit-quantised candidates with duplicates and queries on / near the candidates."""
    import ctypes

    import soundchunks_amd as sc

    rng = np.random.default_rng(seed)
    base = np.round(rng.uniform(-1, 1, size=(r // 2, cs)) * 127) / 127
    fwd = np.concatenate([base, base[rng.integers(0, len(base), size=r - len(base))]]).astype(np.float32)
    rng.shuffle(fwd)
    pick = fwd[rng.integers(0, r, size=n)]
    flip = rng.integers(0, 4, size=n)  # queries near every variant: fwd, rev, neg, neg rev
    pick = np.where((flip & 1)[:, None] == 1, pick[:, ::-1], pick) * np.where(flip >= 2, -1.0, 1.0)[:, None]
    noise = rng.normal(0, 0.002, size=pick.shape) * (rng.uniform(size=(n, 1)) < 0.7)
    q = (pick + noise).astype(np.float32)
    cand4 = np.empty((4 * r, cs), dtype=np.float32)
    cand4[0::4], cand4[1::4], cand4[2::4], cand4[3::4] = fwd, fwd[:, ::-1], -fwd, -fwd[:, ::-1]
    want = np.zeros(n, dtype=np.int32)
    fp = ctypes.POINTER(ctypes.c_float)
    oracle.load().ora_knnfit_assign(4 * r, cs, np.ascontiguousarray(cand4).ctypes.data_as(fp), n,
                                    q.ctypes.data_as(fp), ctypes.c_float(eps),
                                    want.ctypes.data_as(ctypes.POINTER(ctypes.c_int)))
    got = sc.knnfit_assign(fwd, q, eps)
    np.testing.assert_array_equal(got, want)


def _u32(*h):
    return np.array(h, dtype=np.uint32).view(np.float32)


def test_knnfit_eps_tie_needs_ieee_sqrt(oracle):
    """Frame 7 of the C2 bench (1024 s synthetic): |sqrt(e1/8) - sqrt(e0/8)| lands
    0.3 ulp below eps, so the reference keeps the smaller index 2 (chunk 0,
    negated).  A 1-ulp sqrt (HIP's __fsqrt_rn is v_sqrt_f32) rounds s1 up,
    misses the tie and keeps index 6."""
    import soundchunks_amd as sc

    fwd = np.stack([_u32(0x3d8be665, 0x3d8f274a, 0x3d503926, 0x3dbff4af, 0x3e12682f, 0x3e1408a1, 0x3e1dcb4f,
                         0x3e467678),
                    _u32(0x3d281020, 0x3d5c3871, 0x3d566cda, 0x3e0f6ede, 0x3e1254a9, 0x3e199326, 0x3dfefdfc,
                         0x3e2af5ec)])
    q = _u32(0xbd5ae1b6, 0xbd86810d, 0xbd95b12b, 0xbdfb71f7, 0xbe02d106, 0xbe012902, 0xbe1a3134, 0xbe2ec15e)[None]
    eps = float(_u32(0x3a24b306)[0])
    assert oracle.knnfit_assign(fwd, q, eps).tolist() == [2]
    assert sc.knnfit_assign(fwd, q, eps).tolist() == [2]


def test_knnfit_eps_boundary_sweep(oracle):
    """eps one ulp below, at and above the exact f32 gap sqrt(e1/CS) - sqrt(e0/CS)
    for random query / candidate pairs: the choice flips exactly where the
    oracle's does."""
    import soundchunks_amd as sc

    rng = np.random.default_rng(77)
    f32 = np.float32
    flips = 0
    for t in range(24):
        cs = (4, 8, 16)[t % 3]
        fwd = rng.uniform(-0.3, 0.3, size=(2, cs)).astype(np.float32)
        q = (fwd[1] + rng.normal(0, 0.01, size=cs)).astype(np.float32)[None]
        var = [v for c in fwd for v in (c, c[::-1], -c, -c[::-1])]  # f = 4c + 2neg + rev
        s = []
        for v in var:
            e = f32(0)
            for j in range(cs):  # sequential f32 distance, as ANN
                d = f32(q[0, j] - v[j])
                e = f32(e + f32(d * d))
            s.append(f32(np.sqrt(f32(e / f32(cs)))))
        assert min(s[4:]) < min(s[:4])  # the nearest is a variant of chunk 1
        gap = f32(min(s[:4]) - min(s[4:]))
        for eps in (np.nextafter(gap, f32(0)), gap, np.nextafter(gap, f32(1))):
            want = oracle.knnfit_assign(fwd, q, float(eps))
            got = sc.knnfit_assign(fwd, q, float(eps))
            assert got.tolist() == want.tolist(), (t, float(eps))
        flips += int(oracle.knnfit_assign(fwd, q, float(np.nextafter(gap, f32(0))))[0] !=
                     oracle.knnfit_assign(fwd, q, float(gap))[0])
    assert flips >= 20  # the sweep does sit on the decision boundary


# C4: the reference's lame_test corpus (tests/golden/lame_test, copied from the
# reference as data) at -cs8 -cpf4096 (corpus_meta.json) and at the encoder
# defaults -cs4 -cpf4096 (corpus_default_meta.json: SURVEY.md §8d's C4 flags,
# encoder.lpr:1486-1509, and encoder.lps:260 `mstest.wav -v`); expected
# digests from the oracle (tests/golden/make_corpus.py)
CORPUS_SETS = {"cs8": "corpus_meta.json", "default": "corpus_default_meta.json"}


def _corpus(which="cs8"):
    import json
    from golden.cases import HERE

    return json.loads((HERE / CORPUS_SETS[which]).read_text())


@pytest.mark.parametrize("name", sorted(_corpus()["files"]))
def test_corpus_matches_oracle(name):
    import hashlib

    import soundchunks_amd as sc
    from golden.cases import HERE

    meta = _corpus()
    want = meta["files"][name]
    wav = (HERE / "lame_test" / name).read_bytes()
    assert hashlib.sha256(wav).hexdigest() == want["wav_sha256"]
    got = sc.Encoder(meta["argv"]).encode(wav)
    assert len(got) == want["gsc_bytes"]
    assert hashlib.sha256(got).hexdigest() == want["gsc_sha256"]


@pytest.mark.parametrize("which", sorted(CORPUS_SETS))
def test_corpus_as_one_batch_matches_oracle(which):
    """C4 (BASELINE configs[3]): all 22 corpus files in ONE batched encode --
    every frame of every file in one launch per stage (gsc_prepare_many /
    gsc_encode_prepared_files) -- and each file's .gsc equals the oracle's;
    at -cs8 -cpf4096 and at the encoder defaults (-cs4 -cpf4096, D = 8)."""
    import hashlib

    import soundchunks_amd as sc
    from golden.cases import HERE

    meta = _corpus(which)
    names = sorted(meta["files"])
    assert len(names) == 22
    wavs = [(HERE / "lame_test" / n).read_bytes() for n in names]
    outs = sc.encode_many(wavs, meta["argv"])
    tm = sc.Encoder.last_timing()
    assert tm["frames"] == sum(meta["files"][n]["frames"] for n in names)
    # launch rounds are bounded by the pass count (a NaN pass hands a frame to the
    # generic kernel for one round), not multiplied by the number of files
    assert tm["scan_launches"] <= 100
    for n, got in zip(names, outs):
        assert len(got) == meta["files"][n]["gsc_bytes"], n
        assert hashlib.sha256(got).hexdigest() == meta["files"][n]["gsc_sha256"], n


# f4: reconstruction (TBand/TEncoder.MakeDstData) and PsyADelta on the device
@pytest.mark.parametrize("name", ["c1_test_cs8_cpf256", "hihat_cs4_default", "syn3s_cs8_cpf1000_cbd12",
                                  "syn8s_c3_cs16_cpf4096_cbd12", "tiny_passthrough_cs8", "quiet_tone_cs8_cpf1024"])
def test_reconstruction_matches_oracle(oracle, name):
    import soundchunks_amd as sc

    make, argv = CASES[name]
    wav = make()
    gsc, rec, psy = sc.Encoder(argv).encode_recon(wav)
    ogsc, orec, opsy = oracle.encode_recon(wav, argv, threads=8)
    assert gsc == ogsc == golden_path(name).read_bytes()
    np.testing.assert_array_equal(rec, orec)
    assert psy == opsy  # bit-identical f64


# a9: the -py reducer (cluster.py Birch, sklearn 1.7.2) on the datasets the
# reference hands it; labels from the real cluster.py (tests/golden/make_birch.py),
# bit for bit (the numpy / scipy BLAS summation orders: gsc_npblas.h)
_BIRCH = ["mstest_fl500_f0", "mstest_fl500_f2", "silence_tone_cs8_cpf256_f0", "c1_test_cs8_cpf256_f1",
          "hihat_cs8_cpf256_f0"]


@pytest.mark.parametrize("name", _BIRCH)
def test_birch_labels_match_cluster_py(name):
    from golden.cases import HERE
    from soundchunks_amd.encoder import birch_labels

    z = np.load(HERE / f"birch_{name}.npz")
    got = birch_labels(z["dataset"], int(z["k"]))
    assert int((got != z["labels"]).sum()) == 0


@pytest.mark.parametrize("name", ["mstest_fl500_cpf256_py", "tone_lsb45_cs4_cpf256_py", "mstest_default_py"])
def test_python_reduce_file_matches_golden(name):
    import hashlib
    import json

    import soundchunks_amd as sc
    from golden.cases import HERE
    from golden.make_birch import PY_FILES, py_file_wav

    want = json.loads((HERE / "golden_meta.json").read_text())[name]
    wav = py_file_wav(PY_FILES[name][0])
    assert hashlib.sha256(wav).hexdigest() == want["wav_sha256"]
    got = sc.Encoder(want["argv"]).encode(wav)
    assert got == (HERE / f"{name}.gsc").read_bytes()
    assert hashlib.sha256(got).hexdigest() == want["gsc_sha256"]




def test_failed_encode_drains_before_next_encode():
    """An encode whose KNNFit/pack post-processing fails while its scan may
    still be running drains its stream and the device before the shared pinned
    arena is released (gsc_runtime.cpp: lock, drain, PostCtx in that order), so
    a concurrent encode on another thread, which then takes the arena, is
    unaffected.  GSC_TEST_FAIL_POST fails exactly one post_group call."""
    import os
    import threading
    import time

    import soundchunks_amd as sc

    make, argv = CASES["syn8s_c2_cs8_cpf4096"]
    wav = make()
    expected = golden_path("syn8s_c2_cs8_cpf4096").read_bytes()
    res = {}

    def run(tag):
        try:
            res[tag] = sc.Encoder(argv).encode(wav)
        except sc.GscError as e:
            res[tag] = str(e)

    os.environ["GSC_TEST_FAIL_POST"] = "1"
    try:
        ta = threading.Thread(target=run, args=("a",))
        ta.start()
        time.sleep(0.05)
        tb = threading.Thread(target=run, args=("b",))
        tb.start()
        ta.join()
        tb.join()
    finally:
        del os.environ["GSC_TEST_FAIL_POST"]
    failed = [k for k, v in res.items() if isinstance(v, str)]
    assert len(failed) == 1 and "injected" in res[failed[0]], res
    ok = "b" if failed[0] == "a" else "a"
    assert res[ok] == expected
    assert sc.Encoder(argv).encode(wav) == expected  # and the library stays usable
