"""ctypes access to the ORACLE (oracle/_build/liboracle.so) -- test infrastructure.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use this.
"""
from __future__ import annotations

import ctypes
import subprocess
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
ORACLE_DIR = ROOT / "oracle"
ORACLE_LIB = ORACLE_DIR / "_build" / "liboracle.so"
ORACLE_CLI = ORACLE_DIR / "_build" / "gsc_oracle"


class OraParams(ctypes.Structure):
    _fields_ = [
        ("bit_rate", ctypes.c_int), ("precision", ctypes.c_int), ("low_cut", ctypes.c_double),
        ("high_cut", ctypes.c_double), ("chunk_bit_depth", ctypes.c_int), ("chunk_size", ctypes.c_int),
        ("chunks_per_frame", ctypes.c_int), ("reduce_bass_band", ctypes.c_int), ("vfr", ctypes.c_double),
        ("chunk_blend", ctypes.c_int), ("frame_length", ctypes.c_double), ("python_reduce", ctypes.c_int),
        ("verbose", ctypes.c_int),
    ]


class OraStats(ctypes.Structure):
    _fields_ = [("frame_count", ctypes.c_int), ("total_chunks", ctypes.c_longlong),
                ("scan_iterations", ctypes.c_longlong), ("kd_searches", ctypes.c_longlong),
                ("kd_leaves", ctypes.c_longlong), ("kd_splits", ctypes.c_longlong)]


class OraTrace(ctypes.Structure):
    _fields_ = [("N", ctypes.c_int), ("K", ctypes.c_int), ("D", ctypes.c_int), ("CS", ctypes.c_int),
                ("atten_div", ctypes.c_int), ("scan_iters", ctypes.c_int), ("reduced_count", ctypes.c_int),
                ("dataset", ctypes.POINTER(ctypes.c_float)), ("yakmo_centroids", ctypes.POINTER(ctypes.c_float)),
                ("scan_centroids", ctypes.POINTER(ctypes.c_float)), ("clusters", ctypes.POINTER(ctypes.c_int)),
                ("knn_best", ctypes.POINTER(ctypes.c_int)), ("knn_cand", ctypes.POINTER(ctypes.c_float)),
                ("knn_query", ctypes.POINTER(ctypes.c_float)), ("knn_eps", ctypes.c_float)]


_lib = None


def build() -> None:
    subprocess.run(["make", "-s", "-C", str(ORACLE_DIR)], check=True)


def load():
    global _lib
    if _lib is None:
        if not ORACLE_LIB.exists():
            build()
        lib = ctypes.CDLL(str(ORACLE_LIB))
        u8p = ctypes.POINTER(ctypes.c_uint8)
        lib.ora_default_params.argtypes = [ctypes.POINTER(OraParams)]
        lib.ora_parse_params.argtypes = [ctypes.POINTER(OraParams), ctypes.c_int, ctypes.POINTER(ctypes.c_char_p)]
        lib.ora_encode.argtypes = [u8p, ctypes.c_size_t, ctypes.POINTER(OraParams), ctypes.c_int,
                                   ctypes.POINTER(u8p), ctypes.POINTER(ctypes.c_size_t)]
        lib.ora_encode.restype = ctypes.c_int
        lib.ora_encode_frames.argtypes = [u8p, ctypes.c_size_t, ctypes.POINTER(OraParams), ctypes.c_int, ctypes.c_int,
                                          ctypes.c_int, ctypes.POINTER(u8p), ctypes.POINTER(ctypes.c_size_t),
                                          ctypes.POINTER(ctypes.c_int)]
        lib.ora_encode_frames.restype = ctypes.c_int
        lib.ora_encode_frame_list.argtypes = [u8p, ctypes.c_size_t, ctypes.POINTER(OraParams), ctypes.c_void_p,
                                              ctypes.c_int, ctypes.c_int, ctypes.POINTER(u8p),
                                              ctypes.POINTER(ctypes.c_size_t), ctypes.c_void_p,
                                              ctypes.POINTER(ctypes.c_int)]
        lib.ora_encode_frame_list.restype = ctypes.c_int
        lib.ora_encode_recon.argtypes = [u8p, ctypes.c_size_t, ctypes.POINTER(OraParams), ctypes.c_int,
                                         ctypes.POINTER(u8p), ctypes.POINTER(ctypes.c_size_t),
                                         ctypes.POINTER(ctypes.POINTER(ctypes.c_int16)),
                                         ctypes.POINTER(ctypes.c_size_t), ctypes.POINTER(ctypes.c_double)]
        lib.ora_encode_recon.restype = ctypes.c_int
        lib.ora_set_py_labels.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
        lib.ora_free.argtypes = [ctypes.c_void_p]
        lib.ora_get_stats.argtypes = [ctypes.POINTER(OraStats)]
        lib.ora_trace_frame.argtypes = [u8p, ctypes.c_size_t, ctypes.POINTER(OraParams), ctypes.c_int,
                                        ctypes.POINTER(OraTrace)]
        lib.ora_frame_bounds.argtypes = [u8p, ctypes.c_size_t, ctypes.POINTER(OraParams), ctypes.c_void_p,
                                         ctypes.c_void_p, ctypes.c_int]
        lib.ora_frame_bounds.restype = ctypes.c_int
        lib.ora_decode.argtypes = [u8p, ctypes.c_size_t, ctypes.POINTER(ctypes.POINTER(ctypes.c_int16)),
                                   ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int)]
        lib.ora_decode.restype = ctypes.c_long
        lib.ora_make_output_sample.argtypes = [ctypes.c_double, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                               ctypes.c_double]
        lib.ora_make_output_sample.restype = ctypes.c_int16
        lib.ora_make_float_sample.argtypes = [ctypes.c_int16, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                              ctypes.c_double]
        lib.ora_make_float_sample.restype = ctypes.c_double
        for fn in ("fpc_sin", "fpc_cos", "fpc_ln", "fpc_log10"):
            getattr(lib, fn).argtypes = [ctypes.c_double]
            getattr(lib, fn).restype = ctypes.c_double
        fp = ctypes.POINTER(ctypes.c_float)
        ip = ctypes.POINTER(ctypes.c_int)
        lib.ora_yakmo_seed_means.argtypes = [ctypes.c_int, ctypes.c_int, fp, ctypes.c_int, fp, ip]
        lib.ora_scan_reduce.argtypes = [ctypes.c_int, ctypes.c_int, fp, ctypes.c_int, fp, ip, ctypes.c_int]
        lib.ora_scan_reduce_n.argtypes = [ctypes.c_int, ctypes.c_int, fp, ctypes.c_int, fp, ip, ctypes.c_int,
                                          ctypes.c_int]
        lib.ora_knnfit_assign.argtypes = [ctypes.c_int, ctypes.c_int, fp, ctypes.c_int, fp, ctypes.c_float, ip]
        _lib = lib
    return _lib


def params(argv=()) -> OraParams:
    lib = load()
    p = OraParams()
    lib.ora_default_params(ctypes.byref(p))
    arr = (ctypes.c_char_p * max(1, len(argv)))(*[a.encode() for a in argv])
    lib.ora_parse_params(ctypes.byref(p), len(argv), arr)
    return p


def _u8(b: bytes):
    a = np.frombuffer(b, dtype=np.uint8)
    return a, a.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8))


def encode(wav: bytes, argv=(), threads: int = 1) -> bytes:
    lib = load()
    p = params(argv)
    a, ptr = _u8(wav)
    out = ctypes.POINTER(ctypes.c_uint8)()
    n = ctypes.c_size_t(0)
    rc = lib.ora_encode(ptr, len(a), ctypes.byref(p), threads, ctypes.byref(out), ctypes.byref(n))
    if rc != 0:
        raise RuntimeError(f"oracle encode failed: {rc}")
    try:
        return ctypes.string_at(out, n.value)
    finally:
        lib.ora_free(out)


_py_keep = None


def set_py_labels(labels=None, offsets=None):
    """-py mode: per-frame cluster.py labels (concatenated, int32) and each
    frame's offset into them (int64); None clears."""
    global _py_keep
    lib = load()
    if labels is None:
        _py_keep = None
        lib.ora_set_py_labels(None, None, 0)
        return
    lab = np.ascontiguousarray(labels, dtype=np.int32)
    off = np.ascontiguousarray(offsets, dtype=np.int64)
    _py_keep = (lab, off)
    lib.ora_set_py_labels(lab.ctypes.data, off.ctypes.data, len(off))


def encode_recon(wav: bytes, argv=(), threads: int = 1):
    """(.gsc bytes, reconstruction int16 [samples x channels] interleaved, PsyADelta)."""
    lib = load()
    p = params(argv)
    a, ptr = _u8(wav)
    out = ctypes.POINTER(ctypes.c_uint8)()
    n = ctypes.c_size_t(0)
    rec = ctypes.POINTER(ctypes.c_int16)()
    rn = ctypes.c_size_t(0)
    psy = ctypes.c_double(0.0)
    rc = lib.ora_encode_recon(ptr, len(a), ctypes.byref(p), threads, ctypes.byref(out), ctypes.byref(n),
                              ctypes.byref(rec), ctypes.byref(rn), ctypes.byref(psy))
    if rc != 0:
        raise RuntimeError(f"oracle encode failed: {rc}")
    try:
        return (ctypes.string_at(out, n.value), np.ctypeslib.as_array(rec, (rn.value,)).copy(), psy.value)
    finally:
        lib.ora_free(out)
        lib.ora_free(rec)


def encode_frames(wav: bytes, argv=(), frame_begin: int = 0, frame_end: int = -1, threads: int = 1):
    """Frames [frame_begin, frame_end) -> (bytes, total frame count)."""
    lib = load()
    p = params(argv)
    a, ptr = _u8(wav)
    out = ctypes.POINTER(ctypes.c_uint8)()
    n = ctypes.c_size_t(0)
    fc = ctypes.c_int(0)
    rc = lib.ora_encode_frames(ptr, len(a), ctypes.byref(p), frame_begin, frame_end, threads, ctypes.byref(out),
                               ctypes.byref(n), ctypes.byref(fc))
    if rc != 0:
        raise RuntimeError(f"oracle encode failed: {rc}")
    try:
        return ctypes.string_at(out, n.value), fc.value
    finally:
        lib.ora_free(out)


def encode_frame_list(wav: bytes, argv, frames, threads: int = 1):
    """The listed frames of the whole-file encode: ([bytes of each frame], total frame count)."""
    lib = load()
    p = params(argv)
    a, ptr = _u8(wav)
    fl = np.ascontiguousarray(frames, dtype=np.int32)
    fb = np.zeros(max(1, len(fl)), dtype=np.uint64)
    out = ctypes.POINTER(ctypes.c_uint8)()
    n = ctypes.c_size_t(0)
    fc = ctypes.c_int(0)
    rc = lib.ora_encode_frame_list(ptr, len(a), ctypes.byref(p), fl.ctypes.data, len(fl), threads, ctypes.byref(out),
                                   ctypes.byref(n), fb.ctypes.data, ctypes.byref(fc))
    if rc != 0:
        raise RuntimeError(f"oracle encode failed: {rc}")
    try:
        blob = ctypes.string_at(out, n.value)
    finally:
        lib.ora_free(out)
    parts, o = [], 0
    for k in range(len(fl)):
        parts.append(blob[o:o + int(fb[k])])
        o += int(fb[k])
    return parts, fc.value


def scan_reduce(x, c0, precision=3, max_passes=100):
    """KNNScanReduce restatement: (centroids, clusters, passes)."""
    x = np.ascontiguousarray(x, dtype=np.float32)
    c = np.ascontiguousarray(c0, dtype=np.float32).copy()
    cl = np.zeros(x.shape[0], dtype=np.int32)
    fp, ip = ctypes.POINTER(ctypes.c_float), ctypes.POINTER(ctypes.c_int)
    n = load().ora_scan_reduce_n(x.shape[0], x.shape[1], x.ctypes.data_as(fp), c.shape[0], c.ctypes.data_as(fp),
                                 cl.ctypes.data_as(ip), precision, max_passes)
    return c, cl, n


def knnfit_assign(fwd, q, eps):
    """KNNFit's candidate choice f = 4c + 2neg + rev per query over the four
    variants (fwd, rev, -fwd, -rev) of every forward row."""
    fwd = np.ascontiguousarray(fwd, dtype=np.float32)
    q = np.ascontiguousarray(q, dtype=np.float32)
    r, cs = fwd.shape
    cand4 = np.empty((4 * r, cs), dtype=np.float32)
    cand4[0::4], cand4[1::4], cand4[2::4], cand4[3::4] = fwd, fwd[:, ::-1], -fwd, -fwd[:, ::-1]
    out = np.zeros(q.shape[0], dtype=np.int32)
    fp = ctypes.POINTER(ctypes.c_float)
    load().ora_knnfit_assign(4 * r, cs, cand4.ctypes.data_as(fp), q.shape[0], q.ctypes.data_as(fp),
                             ctypes.c_float(eps), out.ctypes.data_as(ctypes.POINTER(ctypes.c_int)))
    return out


def stats() -> dict:
    s = OraStats()
    load().ora_get_stats(ctypes.byref(s))
    return {k: getattr(s, k) for k, _ in s._fields_}


def decode(gsc: bytes):
    lib = load()
    a, ptr = _u8(gsc)
    pcm = ctypes.POINTER(ctypes.c_int16)()
    ch, rate = ctypes.c_int(0), ctypes.c_int(0)
    n = lib.ora_decode(ptr, len(a), ctypes.byref(pcm), ctypes.byref(ch), ctypes.byref(rate))
    out = np.ctypeslib.as_array(pcm, shape=(n,)).copy() if n > 0 else np.zeros(0, np.int16)
    lib.ora_free(pcm)
    return out, ch.value, rate.value


def frame_bounds(wav: bytes, argv=()):
    """PrepareFrames' frame boundaries: (starts, ends) int32 arrays."""
    lib = load()
    p = params(argv)
    a, ptr = _u8(wav)
    n = lib.ora_frame_bounds(ptr, len(a), ctypes.byref(p), None, None, 0)
    if n < 0:
        raise RuntimeError(f"oracle prepare failed: {n}")
    st = np.zeros(max(n, 1), np.int32)
    en = np.zeros(max(n, 1), np.int32)
    lib.ora_frame_bounds(ptr, len(a), ctypes.byref(p), st.ctypes.data_as(ctypes.c_void_p),
                         en.ctypes.data_as(ctypes.c_void_p), n)
    return st[:n], en[:n]


def trace_frame(wav: bytes, argv=(), frame: int = 0) -> dict:
    lib = load()
    p = params(argv)
    a, ptr = _u8(wav)
    t = OraTrace()
    rc = lib.ora_trace_frame(ptr, len(a), ctypes.byref(p), frame, ctypes.byref(t))
    if rc != 0:
        raise RuntimeError(f"oracle trace failed: {rc}")

    def arr(ptr, n, dt):
        return np.ctypeslib.as_array(ptr, shape=(n,)).astype(dt).copy()

    N, K, D, CS, R = t.N, t.K, t.D, t.CS, t.reduced_count
    res = {
        "N": N, "K": K, "D": D, "CS": CS, "atten_div": t.atten_div, "scan_iters": t.scan_iters, "R": R,
        "dataset": arr(t.dataset, N * D, np.float32).reshape(N, D),
        "yakmo": arr(t.yakmo_centroids, K * D, np.float32).reshape(K, D),
        "scan": arr(t.scan_centroids, K * D, np.float32).reshape(K, D),
        "clusters": arr(t.clusters, N, np.int32),
        "knn_best": arr(t.knn_best, N, np.int32),
        "knn_cand": arr(t.knn_cand, 4 * R * CS, np.float32).reshape(4 * R, CS),
        "knn_query": arr(t.knn_query, N * CS, np.float32).reshape(N, CS),
        "knn_eps": float(t.knn_eps),
    }
    for f in ("dataset", "yakmo_centroids", "scan_centroids", "clusters", "knn_best", "knn_cand", "knn_query"):
        lib.ora_free(ctypes.cast(getattr(t, f), ctypes.c_void_p))
    return res
