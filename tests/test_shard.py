"""Multi-rank frame sharding (world size 2, gloo on CPU): each rank encodes a
contiguous frame range and rank 0 gathers the bytes; the result must equal the
single-process encode.  The per-rank encoder here is the oracle (the CPU
checker); on the GPU box bench.py runs the same soundchunks_amd.shard code
with the HIP encoder over RCCL."""
from __future__ import annotations

import os
import sys
from pathlib import Path

import pytest
import torch.multiprocessing as mp

ROOT = Path(__file__).resolve().parents[1]


def _worker(rank, ws, port, argv, seconds, q):
    sys.path.insert(0, str(ROOT))
    sys.path.insert(0, str(ROOT / "tests"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist

    import oracle_ffi
    from soundchunks_amd.shard import frame_range, gather_streams
    from soundchunks_amd.synth import synth_wav

    dist.init_process_group("gloo", rank=rank, world_size=ws)
    try:
        wav = synth_wav(seconds, 44100, 1)
        _, fc = oracle_ffi.encode_frames(wav, argv, 0, 0)
        b, e = frame_range(fc, rank, ws)
        blob, _ = oracle_ffi.encode_frames(wav, argv, b, e, threads=2)
        out = gather_streams(blob)
        if rank == 0:
            q.put((fc, out))
    finally:
        dist.destroy_process_group()


def test_frame_range_partitions():
    from soundchunks_amd.shard import frame_range, frame_range_weighted

    for fc in (0, 1, 3, 7, 900):
        for ws in (1, 2, 3, 8):
            rs = [frame_range(fc, r, ws) for r in range(ws)]
            assert rs[0][0] == 0 and rs[-1][1] == fc
            assert all(rs[i][1] == rs[i + 1][0] for i in range(ws - 1))
            w = [((i * 7) % 5) + 1 for i in range(fc)]
            rw = [frame_range_weighted(w, r, ws) for r in range(ws)]
            assert rw[0][0] == 0 and rw[-1][1] == fc
            assert all(rw[i][1] == rw[i + 1][0] for i in range(ws - 1))


@pytest.mark.timeout(300)
def test_two_rank_gather_equals_single_encode():
    import oracle_ffi
    from soundchunks_amd.synth import synth_wav

    argv = ["-cs8", "-cpf256", "-fl500"]  # 0.5 s frames -> several frames from 2.2 s
    seconds = 2.2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29500 + (os.getpid() % 1000)
    procs = [ctx.Process(target=_worker, args=(r, 2, port, argv, seconds, q)) for r in range(2)]
    for p in procs:
        p.start()
    fc, got = q.get(timeout=280)
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    assert fc >= 3
    want = oracle_ffi.encode(synth_wav(seconds, 44100, 1), argv, threads=4)
    assert got == want


def _hip_worker(rank, ws, port, name, q):
    sys.path.insert(0, str(ROOT))
    sys.path.insert(0, str(ROOT / "tests"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist

    import soundchunks_amd as sc
    from golden.cases import CASES
    from soundchunks_amd.shard import gather_streams

    dist.init_process_group("gloo", rank=rank, world_size=ws)
    try:
        from soundchunks_amd.shard import bounds_range, broadcast_bounds

        make, argv = CASES[name]
        wav = make()
        enc = sc.Encoder(argv)
        prep = enc.prepare(wav) if rank == 0 else None  # PrepareFrames once per job, on rank 0
        st, en = broadcast_bounds(*(prep.frame_bounds() if prep is not None else (None, None)))
        b, e = bounds_range(st, en, enc.chunk_size, 1, rank, ws)
        if prep is None:  # the other ranks load only their frames' samples (bench.py's path)
            prep = enc.prepare_frames(wav, st, en, b, e)
        out = gather_streams(prep.encode(b, e))
        if rank == 0:
            q.put((prep.frame_count, (b, e), out))
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.timeout(300)
def test_two_rank_hip_encoder_matches_golden():
    """The HIP encoder in 2 gloo ranks (both on device 0): each rank encodes its
    chunk-count-balanced frame range; rank 0's gathered bytes equal the golden."""
    from golden.cases import golden_path

    name = "c1_test_cs8_cpf256"
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 30500 + (os.getpid() % 1000)
    procs = [ctx.Process(target=_hip_worker, args=(r, 2, port, name, q)) for r in range(2)]
    for p in procs:
        p.start()
    fc, rng0, got = q.get(timeout=280)
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    assert fc >= 3 and 0 < rng0[1] < fc
    assert got == golden_path(name).read_bytes()
