"""The NaN-centroid model the batched scan kernel relies on (gsc_scan.hip,
DESIGN.md §4 "NaN centroids"), checked against the oracle's ANN restatement
(oracle/ann_oracle.c, ANN.dll annkSearch @0x1800124b0) on a frame whose yakmo
means include 0/0 NaN rows: one KNNScanReduce pass replayed search by search
(encoder.lpr:729-745, live centroids, stale tree).  For every search:
  - the leaf of the near-child descent is the answer when it is a NaN row;
  - otherwise the answer is a real centroid;
  - a leaf below the low child of a NaN cut value is never the answer.
CPU only (the checker, not the product)."""
from __future__ import annotations

import ctypes

import numpy as np
import pytest

from golden.cases import CASES


@pytest.mark.parametrize("name,frame", [("quiet_tone_cs4_cpf1024", 0)])
def test_nan_centroid_model_against_oracle_ann(oracle, name, frame):
    lib = oracle.load()
    lib.ora_kdtree_create.restype = ctypes.c_void_p
    lib.ora_kdtree_create.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int]
    lib.ora_kdtree_search.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_float, ctypes.POINTER(ctypes.c_float)]
    lib.ora_kdtree_search.restype = ctypes.c_int
    lib.ora_kdtree_destroy.argtypes = [ctypes.c_void_p]
    lib.ora_kdtree_node_count.argtypes = [ctypes.c_void_p]
    lib.ora_kdtree_export.argtypes = [ctypes.c_void_p] + [ctypes.c_void_p] * 7
    make, argv = CASES[name]
    t = oracle.trace_frame(make(), argv, frame)
    X = np.ascontiguousarray(t["dataset"], np.float32)
    C = np.ascontiguousarray(t["yakmo"], np.float32).copy()
    N, D = X.shape
    K = C.shape[0]
    nanrow = np.isnan(C).any(axis=1)
    assert nanrow.sum() > 0, "the case must have NaN seeding means"
    fp = ctypes.POINTER(ctypes.c_float)
    rows = (fp * K)(*[C[i].ctypes.data_as(fp) for i in range(K)])
    tree = lib.ora_kdtree_create(ctypes.cast(rows, ctypes.c_void_p), K, D, 1)
    try:
        nn = lib.ora_kdtree_node_count(tree)
        cd = np.zeros(nn, np.int32)
        cv = np.zeros(nn, np.float32)
        lo = np.zeros(nn, np.float32)
        hi = np.zeros(nn, np.float32)
        lc = np.zeros(nn, np.int32)
        hc = np.zeros(nn, np.int32)
        lp = np.zeros(nn, np.int32)
        lib.ora_kdtree_export(tree, *[a.ctypes.data for a in (cd, cv, lo, hi, lc, hc, lp)])
        dead = np.zeros(K, bool)  # below the low child of a NaN cut
        stack = [(0, False)]
        while stack:
            nd, d = stack.pop()
            if lp[nd] >= 0:
                dead[lp[nd]] = d
                continue
            stack.append((lc[nd], d or bool(np.isnan(cv[nd]))))
            stack.append((hc[nd], d))
        nan_first = 0
        for i in range(N):  # pass 0: rate = Single(1/sqrt(1)) = 1 (CCntStart)
            q = X[i]
            nd = 0
            while lp[nd] < 0:
                nd = lc[nd] if np.float32(q[cd[nd]] - cv[nd]) < 0 else hc[nd]
            first = lp[nd]
            err = ctypes.c_float(0)
            b = lib.ora_kdtree_search(tree, q.ctypes.data, 0.0, ctypes.byref(err))
            if nanrow[first]:
                nan_first += 1
                assert b == first, f"search {i}: NaN leaf {first} reached first, ANN returned {b}"
            else:
                assert not nanrow[b], f"search {i}: real first leaf, ANN returned NaN row {b}"
            assert not dead[b], f"search {i}: ANN returned {b} below a NaN cut's low child"
            C[b] = (X[i] - C[b]) * np.float32(1.0) + C[b]  # encoder.lpr:736-740 (in place: ANN sees it)
        assert nan_first > 0
    finally:
        lib.ora_kdtree_destroy(tree)
