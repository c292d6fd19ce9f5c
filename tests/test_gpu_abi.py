"""The reference-named drop-in ABI (extern.pas:112-123) replayed exactly as
the Pascal host calls it (pytest -m gpu), against the oracle:

  TFrame.Reduce        yakmo_create(K,1,0,1,0,0,0) / load_train_data /
                       train_on_data / get_centroids / destroy (encoder.lpr:824-828)
  TFrame.KNNScanReduce per pass ann_kdtree_create on the LIVE centroid row
                       pointers, per point ann_kdtree_search + in-place
                       centroid move (encoder.lpr:725-761)
  TFrame.KNNFit        ann_kdtree_create over the 4R candidates,
                       ann_kdtree_pri_search_multi(64) + the tie rule
                       (encoder.lpr:945-965)

plus the other two search exports on fresh and stale trees.  Small N and K:
every search is one host->device round trip through these entry points.
"""
from __future__ import annotations

import ctypes
import math

import numpy as np
import pytest

from golden.cases import CASES

pytestmark = pytest.mark.gpu

FP = ctypes.POINTER(ctypes.c_float)
IP = ctypes.POINTER(ctypes.c_int)


def _rows(a: np.ndarray):
    """float** row-pointer array aliasing the rows of a (Pascal TFloatDynArray2)."""
    base = a.ctypes.data
    stride = a.strides[0]
    return (FP * a.shape[0])(*[ctypes.cast(base + i * stride, FP) for i in range(a.shape[0])])


def _row(a: np.ndarray, i: int):
    return ctypes.cast(a.ctypes.data + i * a.strides[0], FP)


def _ora_tree_api(lib):
    lib.ora_kdtree_create.restype = ctypes.c_void_p
    lib.ora_kdtree_create.argtypes = [ctypes.POINTER(FP), ctypes.c_int, ctypes.c_int, ctypes.c_int]
    lib.ora_kdtree_destroy.argtypes = [ctypes.c_void_p]
    for fn in (lib.ora_kdtree_search_multi, lib.ora_kdtree_pri_search_multi):
        fn.argtypes = [ctypes.c_void_p, IP, FP, ctypes.c_int, FP, ctypes.c_float]
    return lib


@pytest.fixture(scope="module")
def frame(oracle):
    make, argv = CASES["c1_test_cs8_cpf256"]
    return oracle.trace_frame(make(), argv, 0)


def test_yakmo_abi_matches_oracle(oracle, frame):
    import soundchunks_amd as sc

    lib = sc.load()
    x = np.ascontiguousarray(frame["dataset"][:3000])
    K = 64
    y = lib.yakmo_create(K, 1, 0, 1, 0, 0, 0)
    assert y
    lib.yakmo_load_train_data(y, x.shape[0], x.shape[1], _rows(x))
    labels = np.zeros(x.shape[0], dtype=np.int32)
    lib.yakmo_train_on_data(y, labels.ctypes.data_as(IP))
    c = np.zeros((K, x.shape[1]), dtype=np.float32)
    lib.yakmo_get_centroids(y, _rows(c))
    lib.yakmo_destroy(y)
    want = np.zeros_like(c)
    wl = np.zeros_like(labels)
    assert oracle.load().ora_yakmo_seed_means(x.shape[0], x.shape[1], x.ctypes.data_as(FP), K,
                                              want.ctypes.data_as(FP), wl.ctypes.data_as(IP)) == 0
    np.testing.assert_array_equal(c.view(np.uint32), want.view(np.uint32))
    np.testing.assert_array_equal(labels, wl)


def test_knn_scan_reduce_replay_matches_oracle(oracle, frame):
    """encoder.lpr:699-765 line by line over the ABI: the tree keeps the row
    pointers of Centroids and sees every in-place move (stale tree, live points)."""
    import soundchunks_amd as sc

    lib = sc.load()
    x = np.ascontiguousarray(frame["dataset"][:600])
    N, D = x.shape
    K = 32
    c = np.zeros((K, D), dtype=np.float32)
    assert oracle.load().ora_yakmo_seed_means(N, D, x.ctypes.data_as(FP), K, c.ctypes.data_as(FP),
                                              np.zeros(N, np.int32).ctypes.data_as(IP)) == 0
    want_c, want_cl, want_it = oracle.scan_reduce(x, c, 3, 100)
    pa = _rows(c)
    cnts = {False: np.ones(K, np.int64), True: np.ones(K, np.int64)}
    clusters = np.zeros(N, np.int32)
    it, err = 0, float(np.finfo(np.float32).max)
    best = ctypes.c_float()
    while True:
        prev, err = err, 0.0
        kdt = lib.ann_kdtree_create(pa, K, D, 1, 0)
        assert kdt
        odd = bool(it & 1)
        for i in range(N):
            b = lib.ann_kdtree_search(kdt, _row(x, i), 0.0, ctypes.byref(best))
            assert 0 <= b < K
            rate = np.float32(1.0 / math.sqrt(cnts[not odd][b]))
            v = x[i] - c[b]
            c[b] = c[b] + v * rate
            clusters[i] = b
            err += float(np.sqrt(np.float32(best.value) / np.float32(D)))
            cnts[odd][b] += 1
        cnts[not odd][:] = 1
        it += 1
        lib.ann_kdtree_destroy(kdt)
        if abs(err - prev) <= 1e-3 or it >= 100:
            break
    assert it == want_it
    np.testing.assert_array_equal(clusters, want_cl)
    np.testing.assert_array_equal(c.view(np.uint32), want_c.view(np.uint32))


def test_knnfit_replay_matches_oracle(oracle, frame):
    """encoder.lpr:945-965 over ann_kdtree_pri_search_multi(64)."""
    import soundchunks_amd as sc

    lib = sc.load()
    cand = np.ascontiguousarray(frame["knn_cand"])
    q = np.ascontiguousarray(frame["knn_query"][:1500])
    eps = np.float32(frame["knn_eps"])
    CS = cand.shape[1]
    pa = _rows(cand)  # the tree keeps the row-pointer array (ANN does not copy it): keep it alive
    kdt = lib.ann_kdtree_create(pa, cand.shape[0], CS, 1, 0)
    assert kdt
    idxs = np.zeros(64, np.int32)
    errs = np.zeros(64, np.float32)
    got = np.zeros(q.shape[0], np.int32)
    for i in range(q.shape[0]):
        lib.ann_kdtree_pri_search_multi(kdt, idxs.ctypes.data_as(IP), errs.ctypes.data_as(FP), 64, _row(q, i), 0.0)
        b = int(idxs[0])
        s0 = np.sqrt(errs[0] / np.float32(CS))
        for j in range(64):
            if 0 <= idxs[j] <= b - 1:
                sj = np.sqrt(errs[j] / np.float32(CS))
                if abs(s0 - sj) <= eps:
                    b = int(idxs[j])
        got[i] = b
    lib.ann_kdtree_destroy(kdt)
    want = np.zeros(q.shape[0], np.int32)
    oracle.load().ora_knnfit_assign(cand.shape[0], CS, cand.ctypes.data_as(FP), q.shape[0], q.ctypes.data_as(FP),
                                    ctypes.c_float(eps), want.ctypes.data_as(IP))
    np.testing.assert_array_equal(got, want)
    np.testing.assert_array_equal(got, frame["knn_best"][:1500])


@pytest.mark.parametrize("k,n", [(1, 300), (7, 300), (64, 300), (7, 3000)])
def test_search_exports_stale_tree(oracle, k, n):
    """ann_kdtree_search_multi / pri_search_multi / pri_search vs ANN's
    restatement, on a tree whose points then move (every search reads live rows).
    n = 3000 also runs the build's wave-per-node levels (segments >= 512)."""
    import soundchunks_amd as sc

    lib = sc.load()
    ora = _ora_tree_api(oracle.load())
    rng = np.random.default_rng(7 + k + n)
    pts = np.round(rng.normal(size=(n, 8)) * 8).astype(np.float32) / 8  # coarse grid: exact ties
    pa = _rows(pts)
    t = lib.ann_kdtree_create(pa, pts.shape[0], 8, 1, 0)
    o = ora.ora_kdtree_create(pa, pts.shape[0], 8, 1)
    assert t and o
    gi, ge = np.zeros(k, np.int32), np.zeros(k, np.float32)
    wi, we = np.zeros(k, np.int32), np.zeros(k, np.float32)
    for step in range(60):
        qv = np.round(rng.normal(size=8) * 8).astype(np.float32) / 8
        qp = qv.ctypes.data_as(FP)
        for ours, theirs in ((lib.ann_kdtree_search_multi, ora.ora_kdtree_search_multi),
                             (lib.ann_kdtree_pri_search_multi, ora.ora_kdtree_pri_search_multi)):
            ours(t, gi.ctypes.data_as(IP), ge.ctypes.data_as(FP), k, qp, 0.0)
            theirs(o, wi.ctypes.data_as(IP), we.ctypes.data_as(FP), k, qp, 0.0)
            np.testing.assert_array_equal(gi, wi)
            np.testing.assert_array_equal(ge.view(np.uint32), we.view(np.uint32))
        if k == 1:
            e = ctypes.c_float()
            assert lib.ann_kdtree_pri_search(t, qp, 0.0, ctypes.byref(e)) == wi[0]
        pts[rng.integers(0, pts.shape[0])] += np.float32(0.25)  # in place: the trees stay stale
    lib.ann_kdtree_destroy(t)
    ora.ora_kdtree_destroy(o)


def test_invalid_tree_arguments_return_null():
    import soundchunks_amd as sc

    lib = sc.load()
    assert lib.ann_kdtree_create(None, 10, 8, 2, 0) is None  # bs != 1
    assert lib.ann_kdtree_create(None, 10, 8, 1, 3) is None  # split rule other than ANN_KD_STD
