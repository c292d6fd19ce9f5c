"""Oracle regression against the committed golden .gsc fixtures, .gsc format
checks through the decoder restatement (decoder/decoder.lpr:37-220), and the
ANN / yakmo restatements against brute force where their semantics are
exactly known (fresh tree => exact nearest neighbour, first-visited minimum).

Pinning: the golden .gsc files were produced by this oracle
(tests/golden/make_golden.py); the reference ships no .gsc and its encoder
cannot run here, so whole-file parity with the reference is
unpinned beyond the quantiser KAT and the decoder round trip.
"""
from __future__ import annotations

import ctypes
import struct

import numpy as np
import pytest

import oracle_ffi
from golden.cases import CASES, golden_path

FAST = ["tiny_passthrough_cs8", "silence_tone_cs8_cpf256", "hihat_cs8_cpf256", "hihat_cs4_default",
        "silence_burst_pr0_cs8"]


@pytest.mark.parametrize("name", FAST)
def test_oracle_reproduces_golden(name):
    make, argv = CASES[name]
    assert oracle_ffi.encode(make(), argv, threads=4) == golden_path(name).read_bytes()


def test_oracle_pr0_noise_fails_save_stream_assert():
    """-pr0 on noise: every chunk is its own reduced chunk (passthrough,
    encoder.lpr:891-905) and KNNFit keeps far more than 4096 of them, so
    SaveStream's Assert(reducedChunks.Count <= CMaxChunksPerFrame)
    (encoder.lpr:986, assertions on in encoder.lpi) stops the encode."""
    from soundchunks_amd.synth import synth_wav

    with pytest.raises(RuntimeError, match="-4"):
        oracle_ffi.encode(synth_wav(1.0, 44100, 1), ["-cs8", "-pr0"], threads=2)


def _frame_headers(gsc: bytes):
    """Walk TFrame.SaveStream headers (encoder.lpr:988-1106 / SURVEY App. B)."""
    pos, out = 0, []
    while pos < len(gsc):
        ver, ch = gsc[pos], gsc[pos + 1]
        kw, = struct.unpack_from("<H", gsc, pos + 2)
        bd, cs = gsc[pos + 4], gsc[pos + 5]
        sr, = struct.unpack_from("<I", gsc, pos + 6)
        div, = struct.unpack_from("<H", gsc, pos + 10)
        out.append(dict(ver=ver, ch=ch, K=kw & 0x1FFF, bd=bd, cs=cs, sr=sr & 0xFFFFFF, div=div))
        return out  # first frame is enough for header checks
    return out


@pytest.mark.parametrize("name", sorted(CASES))
def test_golden_decodes(name):
    make, argv = CASES[name]
    wav = make()
    gsc = golden_path(name).read_bytes()
    ch = struct.unpack_from("<H", wav, 22)[0]
    rate = struct.unpack_from("<I", wav, 24)[0]
    h = _frame_headers(gsc)[0]
    assert h["ver"] == 1 and h["ch"] == ch and h["sr"] == rate
    assert 1 <= h["div"] <= 64
    cs = int(next((a[3:] for a in argv if a.startswith("-cs")), "4"))
    assert h["cs"] == cs
    pcm, dch, drate = oracle_ffi.decode(gsc)
    assert dch == ch and drate == rate
    n_in = (len(wav) - 44) // 2
    # the encoder pads the sample count to a ChunkSize multiple (encoder.lpr:1318-1323)
    assert n_in <= pcm.size < n_in + cs * ch + 1
    src = np.frombuffer(wav[44:44 + 2 * n_in], dtype="<i2").astype(np.float64)
    dec = pcm[:n_in].astype(np.float64)
    if np.abs(src).max() > 1000:
        # vector quantisation keeps the waveform: clearly positive correlation
        c = np.corrcoef(src, dec)[0, 1]
        assert c > 0.5, c


def _ann(lib):
    fp = ctypes.POINTER(ctypes.c_float)
    lib.ora_kdtree_create.argtypes = [ctypes.POINTER(fp), ctypes.c_int, ctypes.c_int, ctypes.c_int]
    lib.ora_kdtree_create.restype = ctypes.c_void_p
    lib.ora_kdtree_destroy.argtypes = [ctypes.c_void_p]
    lib.ora_kdtree_search.argtypes = [ctypes.c_void_p, fp, ctypes.c_float, fp]
    lib.ora_kdtree_search.restype = ctypes.c_int
    lib.ora_kdtree_pri_search_multi.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_int), fp, ctypes.c_int, fp,
                                                ctypes.c_float]
    return lib


def _rows(a):
    fp = ctypes.POINTER(ctypes.c_float)
    rows = (fp * a.shape[0])(*[a[i].ctypes.data_as(fp) for i in range(a.shape[0])])
    return rows


def _seq_dist(p, q):
    d = np.float32(0)
    for k in range(p.shape[0]):
        t = np.float32(q[k] - p[k])
        d = np.float32(d + np.float32(t * t))
    return d


@pytest.mark.parametrize("n,dd", [(1, 4), (7, 3), (256, 16), (1000, 8)])
def test_ann_fresh_tree_is_exact_nn(n, dd):
    lib = _ann(oracle_ffi.load())
    rng = np.random.default_rng(n * 31 + dd)
    pts = rng.standard_normal((n, dd)).astype(np.float32)
    pts[n // 2:] = np.round(pts[n // 2:] * 4) / 4  # duplicates / exact ties
    rows = _rows(pts)
    t = lib.ora_kdtree_create(rows, n, dd, 1)
    fp = ctypes.POINTER(ctypes.c_float)
    try:
        for _ in range(200):
            q = (rng.standard_normal(dd) * 1.2).astype(np.float32)
            err = ctypes.c_float(0)
            idx = lib.ora_kdtree_search(t, q.ctypes.data_as(fp), 0.0, ctypes.byref(err))
            d = np.array([_seq_dist(p, q) for p in pts], dtype=np.float32)
            assert err.value == d.min() and d[idx] == d.min()
            k = min(8, n)
            idxs = np.zeros(k, np.int32)
            errs = np.zeros(k, np.float32)
            lib.ora_kdtree_pri_search_multi(t, idxs.ctypes.data_as(ctypes.POINTER(ctypes.c_int)),
                                            errs.ctypes.data_as(fp), k, q.ctypes.data_as(fp), 0.0)
            np.testing.assert_array_equal(errs, np.sort(d)[:k])
    finally:
        lib.ora_kdtree_destroy(t)


def test_yakmo_seed_means_properties():
    lib = oracle_ffi.load()
    fp = ctypes.POINTER(ctypes.c_float)
    rng = np.random.default_rng(3)
    N, D, K = 600, 8, 16
    x = rng.standard_normal((N, D)).astype(np.float32)
    c = np.zeros((K, D), np.float32)
    lab = np.zeros(N, np.int32)
    assert lib.ora_yakmo_seed_means(N, D, x.ctypes.data_as(fp), K, c.ctypes.data_as(fp),
                                    lab.ctypes.data_as(ctypes.POINTER(ctypes.c_int))) == 0
    # every centroid is the f32 mean (in point order) of its seeding cluster
    for k in range(K):
        m = x[lab == k]
        s = np.zeros(D, np.float32)
        for row in m:
            s = (s + row).astype(np.float32)
        np.testing.assert_array_equal(c[k], (s / np.float32(len(m))).astype(np.float32))
    # K >= N is rejected (the DLL would spin)
    assert lib.ora_yakmo_seed_means(4, D, x.ctypes.data_as(fp), 4, c.ctypes.data_as(fp),
                                    lab.ctypes.data_as(ctypes.POINTER(ctypes.c_int))) == -1


@pytest.mark.parametrize("meta_file", ["corpus_meta.json", "corpus_default_meta.json"])
@pytest.mark.parametrize("name", ["60.wav", "hihat.wav", "mstest.wav"])
def test_oracle_reproduces_corpus_digest(name, meta_file):
    """The committed C4 digests (tests/golden/corpus_meta.json at -cs8
    -cpf4096, corpus_default_meta.json at the encoder defaults) are what the
    oracle computes now (the three smallest corpus files, to stay fast)."""
    import hashlib
    import json

    import oracle_ffi
    from golden.cases import HERE

    meta = json.loads((HERE / meta_file).read_text())
    wav = (HERE / "lame_test" / name).read_bytes()
    gsc = oracle_ffi.encode(wav, meta["argv"], threads=8)
    assert hashlib.sha256(gsc).hexdigest() == meta["files"][name]["gsc_sha256"]


@pytest.mark.parametrize("name", ["c1_test_cs8_cpf256", "hihat_cs8_cpf256", "syn2s_c2_cs8_cpf4096"])
def test_oracle_reconstruction_agrees_with_decoder(name):
    """f4 pin: the encoder-side reconstruction (encoder.lpr:487-522,1518-1582)
    and the independently restated decoder (decoder.lpr:37-220) rebuild the
    same signal from the same .gsc, up to the decoder's integer lookup
    arithmetic (12-bit rescale, 15-bit attenuation table)."""
    make, argv = CASES[name]
    wav = make()
    gsc, rec, psy = oracle_ffi.encode_recon(wav, argv, threads=8)
    assert gsc == golden_path(name).read_bytes()
    pcm = np.asarray(oracle_ffi.decode(gsc)[0]).ravel().astype(np.int64)
    k = min(len(pcm), len(rec))
    assert k >= len(rec) - 64 * 2
    diff = np.abs(pcm[:k] - rec[:k].astype(np.int64))
    assert diff.max() <= 32
    src = np.zeros(len(rec))  # srcData padded with zeros to the block multiple (encoder.lpr:1317-1323)
    s = np.frombuffer(wav[44:44 + (len(wav) - 44) // 2 * 2], dtype="<i2").astype(np.float64)[:len(rec)]
    src[:len(s)] = s
    assert psy == pytest.approx(np.sqrt(((src - rec) ** 2).sum() / len(rec)), rel=1e-12)


# a9 (-py): the oracle fed cluster.py's labels reproduces the committed .gsc,
# and the datasets it hands cluster.py are the fixtures' (make_birch.py)
def test_oracle_python_reduce_reproduces_fixture():
    import json

    from golden.cases import HERE

    want = json.loads((HERE / "golden_meta.json").read_text())["mstest_fl500_cpf256_py"]
    z = np.load(HERE / "birch_file_mstest_fl500_cpf256_py.npz")
    wav = (HERE / "lame_test" / "mstest.wav").read_bytes()
    oracle_ffi.set_py_labels(z["labels"], z["offsets"])
    try:
        got = oracle_ffi.encode(wav, want["argv"], threads=8)
    finally:
        oracle_ffi.set_py_labels(None)
    assert got == (HERE / "mstest_fl500_cpf256_py.gsc").read_bytes()
    for name in ("mstest_fl500_f0", "mstest_fl500_f2"):
        b = np.load(HERE / f"birch_{name}.npz")
        tr = oracle_ffi.trace_frame(wav, [str(a) for a in b["argv"]], int(b["frame"]))
        np.testing.assert_array_equal(np.asarray(tr["dataset"], np.float32), b["dataset"])
        assert int(tr["K"]) == int(b["k"])


# the -py reducer's host part (gsc_birch_host.cpp: CF tree, linkage labelling,
# _hc_cut) with host restatements of its two device steps (tools/birch), built
# with g++ here, against cluster.py's labels
@pytest.mark.parametrize("name", ["mstest_fl500_f0", "mstest_fl500_f2"])
def test_birch_host_part_matches_cluster_py(tmp_path, name):
    import subprocess
    from pathlib import Path

    from golden.cases import HERE

    root = Path(__file__).resolve().parents[1]
    so = tmp_path / "birch_host.so"
    subprocess.run(["g++", "-O2", "-ffp-contract=off", "-shared", "-fPIC", "-o", str(so),
                    str(root / "tools" / "birch" / "host_check.cpp"),
                    str(root / "soundchunks_amd" / "csrc" / "gsc_birch_host.cpp")], check=True)
    lib = ctypes.CDLL(str(so))
    z = np.load(HERE / f"birch_{name}.npz")
    x = np.ascontiguousarray(z["dataset"], np.float32)
    out = np.zeros(x.shape[0], np.int32)
    assert lib.birch_host_labels(x.shape[0], x.shape[1], ctypes.c_void_p(x.ctypes.data), int(z["k"]),
                                 ctypes.c_void_p(out.ctypes.data)) == 0
    np.testing.assert_array_equal(out, z["labels"])


def test_oracle_frame_list_rejects_repeated_frames():
    """ora_encode_frame_list refuses an index listed twice (two workers would
    write the same frame's buffer) as it refuses one outside the file."""
    import oracle_ffi
    from soundchunks_amd.synth import synth_wav

    wav = synth_wav(0.5)
    with pytest.raises(RuntimeError, match="-2"):
        oracle_ffi.encode_frame_list(wav, ["-cs8", "-cpf256"], [0, 0])
    with pytest.raises(RuntimeError, match="-2"):
        oracle_ffi.encode_frame_list(wav, ["-cs8", "-cpf256"], [5])
