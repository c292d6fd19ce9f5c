"""ctypes binding of the in-tree C-ABI library (include/soundchunks.h).

The library is built in-tree by ``__graft_entry__.build()`` (or
``make -C soundchunks_amd/csrc``) into ``soundchunks_amd/lib/libsoundchunks_amd.so``.
There is no CPU fallback: if the library or a gfx950 device is missing, every
compute call raises.
"""
from __future__ import annotations

import ctypes
import os
from pathlib import Path

LIB_PATH = Path(__file__).resolve().parent / "lib" / "libsoundchunks_amd.so"


class GscOptions(ctypes.Structure):
    """Mirror of ``gsc_options`` (TEncoder fields, encoder.lpr:1486-1509)."""

    _fields_ = [
        ("bit_rate", ctypes.c_int),
        ("precision", ctypes.c_int),
        ("low_cut", ctypes.c_double),
        ("high_cut", ctypes.c_double),
        ("chunk_bit_depth", ctypes.c_int),
        ("chunk_size", ctypes.c_int),
        ("chunks_per_frame", ctypes.c_int),
        ("reduce_bass_band", ctypes.c_int),
        ("vfr", ctypes.c_double),
        ("chunk_blend", ctypes.c_int),
        ("frame_length", ctypes.c_double),
        ("python_reduce", ctypes.c_int),
        ("verbose", ctypes.c_int),
    ]


class GscTiming(ctypes.Structure):
    _fields_ = [
        ("host_prepare_ms", ctypes.c_double),
        ("host_frames_ms", ctypes.c_double),
        ("gpu_yakmo_ms", ctypes.c_double),
        ("gpu_scan_ms", ctypes.c_double),
        ("gpu_knnfit_ms", ctypes.c_double),
        ("host_post_ms", ctypes.c_double),
        ("total_ms", ctypes.c_double),
        ("frames", ctypes.c_int),
        ("reduce_frames", ctypes.c_int),
        ("points", ctypes.c_longlong),
        ("scan_passes", ctypes.c_longlong),
        ("scan_slow", ctypes.c_longlong),
        ("scan_point_passes", ctypes.c_longlong),
        ("knnfit_pairs", ctypes.c_longlong),
        ("scan_launches", ctypes.c_int),
        ("knnfit_launches", ctypes.c_int),
        ("scan_restarts", ctypes.c_longlong),
        ("gpu_dsp_ms", ctypes.c_double),
        ("post_overlap_ms", ctypes.c_double),
        ("post_groups", ctypes.c_int),
        ("gpu_recon_ms", ctypes.c_double),
        ("knnfit_overflow", ctypes.c_longlong),
    ]


_FP = ctypes.POINTER(ctypes.c_float)
_IP = ctypes.POINTER(ctypes.c_int)
_U8P = ctypes.POINTER(ctypes.c_uint8)

# name -> (restype, argtypes); every symbol declared in include/soundchunks.h
SIGNATURES = {
    "yakmo_create": (ctypes.c_void_p, [ctypes.c_uint, ctypes.c_uint, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                        ctypes.c_int, ctypes.c_int]),
    "yakmo_destroy": (None, [ctypes.c_void_p]),
    "yakmo_load_train_data": (None, [ctypes.c_void_p, ctypes.c_uint, ctypes.c_uint, ctypes.POINTER(_FP)]),
    "yakmo_train_on_data": (None, [ctypes.c_void_p, _IP]),
    "yakmo_get_centroids": (None, [ctypes.c_void_p, ctypes.POINTER(_FP)]),
    "ann_kdtree_create": (ctypes.c_void_p, [ctypes.POINTER(_FP), ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                             ctypes.c_int]),
    "ann_kdtree_destroy": (None, [ctypes.c_void_p]),
    "ann_kdtree_search": (ctypes.c_int, [ctypes.c_void_p, _FP, ctypes.c_float, _FP]),
    "ann_kdtree_pri_search": (ctypes.c_int, [ctypes.c_void_p, _FP, ctypes.c_float, _FP]),
    "ann_kdtree_search_multi": (None, [ctypes.c_void_p, _IP, _FP, ctypes.c_int, _FP, ctypes.c_float]),
    "ann_kdtree_pri_search_multi": (None, [ctypes.c_void_p, _IP, _FP, ctypes.c_int, _FP, ctypes.c_float]),
    "gsc_default_options": (None, [ctypes.POINTER(GscOptions)]),
    "gsc_parse_options": (None, [ctypes.POINTER(GscOptions), ctypes.c_int, ctypes.POINTER(ctypes.c_char_p)]),
    "gsc_encode_wav": (ctypes.c_int, [_U8P, ctypes.c_size_t, ctypes.POINTER(GscOptions), ctypes.POINTER(_U8P),
                                      ctypes.POINTER(ctypes.c_size_t)]),
    "gsc_encode_wav_frames": (ctypes.c_int, [_U8P, ctypes.c_size_t, ctypes.POINTER(GscOptions), ctypes.c_int,
                                             ctypes.c_int, ctypes.POINTER(_U8P), ctypes.POINTER(ctypes.c_size_t),
                                             _IP]),
    "gsc_encode_wav_recon": (ctypes.c_int, [_U8P, ctypes.c_size_t, ctypes.POINTER(GscOptions), ctypes.POINTER(_U8P),
                                            ctypes.POINTER(ctypes.c_size_t),
                                            ctypes.POINTER(ctypes.POINTER(ctypes.c_int16)),
                                            ctypes.POINTER(ctypes.c_size_t), ctypes.POINTER(ctypes.c_double)]),
    "gsc_count_frames": (ctypes.c_int, [_U8P, ctypes.c_size_t, ctypes.POINTER(GscOptions), _IP]),
    "gsc_prepare": (ctypes.c_void_p, [_U8P, ctypes.c_size_t, ctypes.POINTER(GscOptions)]),
    "gsc_prepared_frame_count": (ctypes.c_int, [ctypes.c_void_p]),
    "gsc_prepared_frame_chunks": (ctypes.c_int, [ctypes.c_void_p, _IP]),
    "gsc_prepared_frame_bounds": (ctypes.c_int, [ctypes.c_void_p, _IP, _IP]),
    "gsc_prepare_frames": (ctypes.c_void_p, [_U8P, ctypes.c_size_t, ctypes.POINTER(GscOptions), _IP, _IP, ctypes.c_int,
                                             ctypes.c_int, ctypes.c_int]),
    "gsc_prepare_many": (ctypes.c_void_p, [ctypes.POINTER(_U8P), ctypes.POINTER(ctypes.c_size_t), ctypes.c_int,
                                           ctypes.POINTER(GscOptions)]),
    "gsc_prepared_file_count": (ctypes.c_int, [ctypes.c_void_p]),
    "gsc_prepared_file_frames": (ctypes.c_int, [ctypes.c_void_p, _IP]),
    "gsc_encode_prepared_files": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.POINTER(_U8P),
                                                 ctypes.POINTER(ctypes.c_size_t), ctypes.POINTER(ctypes.c_size_t)]),
    "gsc_encode_prepared": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.POINTER(_U8P),
                                           ctypes.POINTER(ctypes.c_size_t)]),
    "gsc_encode_prepared_frames": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.POINTER(_U8P),
                                                  ctypes.POINTER(ctypes.c_size_t), ctypes.POINTER(ctypes.c_size_t)]),
    "gsc_prepared_prepare_ms": (ctypes.c_double, [ctypes.c_void_p]),
    "gsc_prepared_free": (None, [ctypes.c_void_p]),
    "gsc_frame_dsp": (ctypes.c_int, [_U8P, ctypes.c_size_t, ctypes.POINTER(GscOptions), ctypes.c_int, _IP,
                                     ctypes.POINTER(_FP), _IP]),
    "gsc_yakmo_seed_means": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, _FP, ctypes.c_int, _FP]),
    "gsc_yakmo_chain_test": (ctypes.c_int, [ctypes.c_int, _FP, ctypes.c_int, ctypes.c_float, _IP, _FP, _FP, _FP,
                                            _FP]),
    "gsc_scan_reduce": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, _FP, ctypes.c_int, _FP, _IP, ctypes.c_int, _IP]),
    "gsc_birch_labels": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, _FP, ctypes.c_int, _IP]),
    "gsc_knnfit_assign": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, _FP, ctypes.c_int, _FP, ctypes.c_float, _IP]),
    "gsc_last_timing": (None, [ctypes.POINTER(GscTiming)]),
    "gsc_device_count": (ctypes.c_int, []),
    "gsc_set_device": (ctypes.c_int, [ctypes.c_int]),
    "gsc_last_error": (ctypes.c_char_p, []),
    "gsc_free": (None, [ctypes.c_void_p]),
}

_lib = None


class GscError(RuntimeError):
    pass


def load(path: str | os.PathLike | None = None) -> ctypes.CDLL:
    """Load the product library (fails loudly if it has not been built)."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    p = Path(path) if path is not None else Path(os.environ.get("GSC_LIB", LIB_PATH))
    if not p.exists():
        raise GscError(f"{p} not built; run __graft_entry__.build() or make -C soundchunks_amd/csrc")
    lib = ctypes.CDLL(str(p))
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if path is None:
        _lib = lib
    return lib


def check(rc: int) -> None:
    if rc != 0:
        raise GscError(load().gsc_last_error().decode(errors="replace"))
