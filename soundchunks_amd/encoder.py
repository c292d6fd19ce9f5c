"""Host-side mirror of the reference ``TEncoder`` (encoder/encoder.lpr:121-196)
for the MI355X hot path.

``Encoder(argv).encode(wav_bytes)`` returns ``.gsc`` bytes, bit-identical to the
reference encoder on the same WAV and options.  Options use the reference's
argv syntax (values glued to the flag, prefix matching; encoder.lpr:201-227,
1985-1998), e.g. ``Encoder(["-cs8", "-cpf4096", "-cbd8"])``.
"""
from __future__ import annotations

import ctypes
from typing import Sequence

import numpy as np

from . import _lib


def parse_options(argv: Sequence[str] = ()) -> _lib.GscOptions:
    lib = _lib.load()
    o = _lib.GscOptions()
    lib.gsc_default_options(ctypes.byref(o))
    arr = (ctypes.c_char_p * max(1, len(argv)))(*[a.encode() for a in argv])
    lib.gsc_parse_options(ctypes.byref(o), len(argv), arr)
    return o


def _u8(buf: bytes):
    a = np.frombuffer(buf, dtype=np.uint8)
    return a, a.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8))


class Encoder:
    """TEncoder: Load -> PrepareFrames -> MakeFrames -> SaveStream, with
    TFrame.Reduce / TFrame.KNNFit on the GPU."""

    def __init__(self, argv: Sequence[str] = ()):
        self.argv = list(argv)
        self.options = parse_options(self.argv)

    # ChunkSize, ChunksPerFrame, ... exposed like the TEncoder fields
    def __getattr__(self, name):
        opts = self.__dict__.get("options")
        if opts is not None and name in dict(_lib.GscOptions._fields_):
            return getattr(opts, name)
        raise AttributeError(name)

    def frame_count(self, wav: bytes) -> int:
        lib = _lib.load()
        arr, ptr = _u8(wav)
        n = ctypes.c_int(0)
        _lib.check(lib.gsc_count_frames(ptr, len(arr), ctypes.byref(self.options), ctypes.byref(n)))
        return n.value

    def encode(self, wav: bytes, frame_begin: int = 0, frame_end: int = -1) -> bytes:
        """Encode frames [frame_begin, frame_end) (default: all) to .gsc bytes."""
        lib = _lib.load()
        arr, ptr = _u8(wav)
        out = ctypes.POINTER(ctypes.c_uint8)()
        n = ctypes.c_size_t(0)
        fc = ctypes.c_int(0)
        rc = lib.gsc_encode_wav_frames(ptr, len(arr), ctypes.byref(self.options), frame_begin, frame_end,
                                       ctypes.byref(out), ctypes.byref(n), ctypes.byref(fc))
        _lib.check(rc)
        try:
            return ctypes.string_at(out, n.value)
        finally:
            lib.gsc_free(out)

    def encode_recon(self, wav: bytes):
        """Encode, plus the reference's reconstruction and PsyADelta
        (encoder.lpr:2019-2031): (.gsc bytes, int16 samples interleaved
        [sample][channel] over the padded SampleCount, PsyADelta)."""
        lib = _lib.load()
        arr, ptr = _u8(wav)
        out = ctypes.POINTER(ctypes.c_uint8)()
        n = ctypes.c_size_t(0)
        rec = ctypes.POINTER(ctypes.c_int16)()
        rn = ctypes.c_size_t(0)
        psy = ctypes.c_double(0.0)
        rc = lib.gsc_encode_wav_recon(ptr, len(arr), ctypes.byref(self.options), ctypes.byref(out), ctypes.byref(n),
                                      ctypes.byref(rec), ctypes.byref(rn), ctypes.byref(psy))
        _lib.check(rc)
        try:
            return (ctypes.string_at(out, n.value), np.ctypeslib.as_array(rec, (rn.value,)).copy(), psy.value)
        finally:
            lib.gsc_free(out)
            lib.gsc_free(rec)

    def prepare(self, wav: bytes) -> "Prepared":
        """Load + PrepareFrames once (the frame boundaries of the whole file)."""
        return Prepared(self, wav)

    def prepare_frames(self, wav: bytes, starts, ends, frame_begin: int = 0, frame_end: int = -1) -> "Prepared":
        """A prepared encoder over frame boundaries computed elsewhere (e.g.
        broadcast from the rank that ran PrepareFrames); only the samples of
        frames [frame_begin, frame_end) are loaded and only they may be encoded."""
        return Prepared(self, wav, bounds=(starts, ends, frame_begin, frame_end))

    def prepare_many(self, wavs) -> "Prepared":
        """A batch of WAVs as one frame list (each file's own Load +
        PrepareFrames; every stage then runs one launch for the whole batch)."""
        return Prepared(self, None, many=list(wavs))

    @staticmethod
    def last_timing() -> dict:
        t = _lib.GscTiming()
        _lib.load().gsc_last_timing(ctypes.byref(t))
        return {k: getattr(t, k) for k, _ in t._fields_}


class Prepared:
    """A WAV after TEncoder.Load + PrepareFrames (encoder.lpr:1111-1152,
    1294-1429): frame boundaries computed once per job, then any frame range
    encodes without rescanning the file (multi-GPU sharding)."""

    def __init__(self, encoder: Encoder, wav: bytes | None, bounds=None, many=None):
        lib = _lib.load()
        if many is not None:
            arrs = [_u8(w) for w in many]
            ptrs = (ctypes.POINTER(ctypes.c_uint8) * len(arrs))(*[p for _, p in arrs])
            lens = (ctypes.c_size_t * len(arrs))(*[len(a) for a, _ in arrs])
            h = lib.gsc_prepare_many(ptrs, lens, len(arrs), ctypes.byref(encoder.options))
            if not h:
                raise _lib.GscError(lib.gsc_last_error().decode(errors="replace"))
            self._h = h
            self.frame_count = lib.gsc_prepared_frame_count(h)
            self.prepare_ms = lib.gsc_prepared_prepare_ms(h)
            return
        arr, ptr = _u8(wav)
        if bounds is None:
            h = lib.gsc_prepare(ptr, len(arr), ctypes.byref(encoder.options))
        else:
            st = np.ascontiguousarray(bounds[0], dtype=np.int32)
            en = np.ascontiguousarray(bounds[1], dtype=np.int32)
            h = lib.gsc_prepare_frames(ptr, len(arr), ctypes.byref(encoder.options), _ip(st), _ip(en), len(st),
                                       int(bounds[2]), int(bounds[3]))
        if not h:
            raise _lib.GscError(lib.gsc_last_error().decode(errors="replace"))
        self._h = h
        self.frame_count = lib.gsc_prepared_frame_count(h)
        self.prepare_ms = lib.gsc_prepared_prepare_ms(h)

    def frame_chunks(self) -> np.ndarray:
        """chunkRefs count (chunks x channels) per frame: the sharding weights."""
        out = np.zeros(max(1, self.frame_count), dtype=np.int32)
        _lib.check(_lib.load().gsc_prepared_frame_chunks(self._h, _ip(out)))
        return out[: self.frame_count]

    def frame_bounds(self) -> tuple[np.ndarray, np.ndarray]:
        """First and last sample of every frame (PrepareFrames' cut)."""
        st = np.zeros(max(1, self.frame_count), dtype=np.int32)
        en = np.zeros(max(1, self.frame_count), dtype=np.int32)
        _lib.check(_lib.load().gsc_prepared_frame_bounds(self._h, _ip(st), _ip(en)))
        return st[: self.frame_count], en[: self.frame_count]

    def encode(self, frame_begin: int = 0, frame_end: int = -1) -> bytes:
        lib = _lib.load()
        out = ctypes.POINTER(ctypes.c_uint8)()
        n = ctypes.c_size_t(0)
        _lib.check(lib.gsc_encode_prepared(self._h, frame_begin, frame_end, ctypes.byref(out), ctypes.byref(n)))
        try:
            return ctypes.string_at(out, n.value)
        finally:
            lib.gsc_free(out)

    def encode_frames(self, frame_begin: int = 0, frame_end: int = -1) -> tuple[bytes, list[int]]:
        """Frames [frame_begin, frame_end): (bytes, each frame's byte count)."""
        lib = _lib.load()
        fe = self.frame_count if frame_end < 0 else min(frame_end, self.frame_count)
        nb = max(0, fe - max(0, frame_begin))
        out = ctypes.POINTER(ctypes.c_uint8)()
        ln = ctypes.c_size_t(0)
        fb = (ctypes.c_size_t * max(1, nb))()
        _lib.check(lib.gsc_encode_prepared_frames(self._h, frame_begin, frame_end, ctypes.byref(out),
                                                  ctypes.byref(ln), fb))
        try:
            return ctypes.string_at(out, ln.value), [int(fb[i]) for i in range(nb)]
        finally:
            lib.gsc_free(out)

    def file_frames(self) -> np.ndarray:
        """First frame of every file of a batch, then the total frame count."""
        lib = _lib.load()
        n = lib.gsc_prepared_file_count(self._h)
        out = np.zeros(n + 1, dtype=np.int32)
        _lib.check(lib.gsc_prepared_file_frames(self._h, _ip(out)))
        return out

    def encode_files(self, frame_begin: int = 0, frame_end: int = -1) -> tuple[bytes, list[int]]:
        """Frames [frame_begin, frame_end) of the batch: (bytes, per-file byte counts)."""
        lib = _lib.load()
        n = lib.gsc_prepared_file_count(self._h)
        out = ctypes.POINTER(ctypes.c_uint8)()
        ln = ctypes.c_size_t(0)
        fb = (ctypes.c_size_t * max(1, n))()
        _lib.check(lib.gsc_encode_prepared_files(self._h, frame_begin, frame_end, ctypes.byref(out), ctypes.byref(ln),
                                                 fb))
        try:
            return ctypes.string_at(out, ln.value), [int(fb[i]) for i in range(n)]
        finally:
            lib.gsc_free(out)

    def close(self) -> None:
        if getattr(self, "_h", None):
            _lib.load().gsc_prepared_free(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def encode_many(wavs, argv: Sequence[str] = (), rank: int = 0, world_size: int = 1, device=None):
    """Encode a batch of WAVs (the C4 corpus case) as one job: every frame of
    every file in one launch per stage, the batch's frame list sharded across
    ranks by chunk count.  Returns one .gsc per file on rank 0
    (None on the others; world_size > 1 needs torch.distributed initialised).
    With a process group initialised the bytes always go through the
    collective gather, also for one rank (`device`: where its tensors live)."""
    from .shard import frame_range_weighted, gather_files

    wavs = list(wavs)
    p = Encoder(argv).prepare_many(wavs)
    try:
        b, e = frame_range_weighted(p.frame_chunks().tolist(), rank, world_size)
        blob, sizes = p.encode_files(b, e)
    finally:
        p.close()
    import torch.distributed as dist

    if world_size > 1 or (dist.is_available() and dist.is_initialized()):
        return gather_files(blob, sizes, device=device)
    outs, o = [], 0
    for n in sizes:
        outs.append(blob[o:o + n])
        o += n
    return outs


def set_device(device: int) -> None:
    """Bind this process's HIP context to `device` (one process per GPU)."""
    _lib.check(_lib.load().gsc_set_device(device))


def _fp(a: np.ndarray):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_float))


def _ip(a: np.ndarray):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_int))


def yakmo_seed_means(x: np.ndarray, k: int) -> np.ndarray:
    """yakmo k-means++ seeding means on the GPU (x: N x D float32)."""
    x = np.ascontiguousarray(x, dtype=np.float32)
    c = np.zeros((k, x.shape[1]), dtype=np.float32)
    _lib.check(_lib.load().gsc_yakmo_seed_means(x.shape[0], x.shape[1], _fp(x), k, _fp(c)))
    return c


def scan_reduce(x: np.ndarray, c0: np.ndarray, precision: int = 3):
    """KNNScanReduce on the GPU; returns (centroids, clusters, passes)."""
    x = np.ascontiguousarray(x, dtype=np.float32)
    c = np.ascontiguousarray(c0, dtype=np.float32).copy()
    cl = np.zeros(x.shape[0], dtype=np.int32)
    it = ctypes.c_int(0)
    _lib.check(_lib.load().gsc_scan_reduce(x.shape[0], x.shape[1], _fp(x), c.shape[0], _fp(c), _ip(cl), precision,
                                           ctypes.byref(it)))
    return c, cl, it.value


def birch_labels(x: np.ndarray, k: int) -> np.ndarray:
    """-py reducer stage: Birch labels of one frame's features (gsc_birch_host.cpp)."""
    lib = _lib.load()
    x = np.ascontiguousarray(x, dtype=np.float32)
    out = np.zeros(x.shape[0], dtype=np.int32)
    _lib.check(lib.gsc_birch_labels(x.shape[0], x.shape[1], _fp(x), k, _ip(out)))
    return out


def knnfit_assign(cand_fwd: np.ndarray, q: np.ndarray, eps: float) -> np.ndarray:
    """KNNFit candidate choice f = 4c + 2neg + rev per query on the GPU."""
    cand_fwd = np.ascontiguousarray(cand_fwd, dtype=np.float32)
    q = np.ascontiguousarray(q, dtype=np.float32)
    out = np.zeros(q.shape[0], dtype=np.int32)
    _lib.check(_lib.load().gsc_knnfit_assign(cand_fwd.shape[0], cand_fwd.shape[1], _fp(cand_fwd), q.shape[0],
                                             _fp(q), ctypes.c_float(eps), _ip(out)))
    return out


def frame_dsp(wav: bytes, frame: int = 0, argv: Sequence[str] = ()) -> tuple[int, np.ndarray]:
    """Device DSP of one frame: (attenuation divider, N x 2CS features)."""
    o = parse_options(argv)
    a, ptr = _u8(wav)
    att = ctypes.c_int(0)
    n = ctypes.c_int(0)
    feat = ctypes.POINTER(ctypes.c_float)()
    lib = _lib.load()
    _lib.check(lib.gsc_frame_dsp(ptr, len(a), ctypes.byref(o), frame, ctypes.byref(att), ctypes.byref(feat),
                                 ctypes.byref(n)))
    try:
        d = 2 * o.chunk_size
        x = np.ctypeslib.as_array(feat, shape=(n.value * d,)).copy().reshape(n.value, d)
    finally:
        lib.gsc_free(ctypes.cast(feat, ctypes.c_void_p))
    return att.value, x
