"""The multi-GPU plumbing bench.py uses (soundchunks_amd.shard), on CPU:
the --gpus N launcher, rank 0's PrepareFrames boundaries broadcast to every
rank, the chunk-count (LPT) frame ranges, a rank preparing only its own
frames from the broadcast bounds, and the frame-ordered / per-file gathers.
World size 2 over gloo; the per-rank encoder is the oracle (the CPU checker:
the HIP encoder needs the GPU, tests/test_shard.py runs it there)."""
from __future__ import annotations

import os
import subprocess
import sys
from pathlib import Path

import numpy as np
import pytest
import torch.multiprocessing as mp

ROOT = Path(__file__).resolve().parents[1]


def test_spawn_workers_sets_rank_env(tmp_path):
    from soundchunks_amd.shard import spawn_workers

    script = tmp_path / "w.py"
    out = tmp_path / "out"
    out.mkdir()
    script.write_text("import os, pathlib\n"
                      f"pathlib.Path(r'{out}', os.environ['RANK']).write_text("
                      "os.environ['WORLD_SIZE'] + ' ' + os.environ['LOCAL_RANK'] + ' ' + os.environ['MASTER_ADDR'])\n")
    assert spawn_workers(3, [sys.executable, str(script)]) == 0
    got = sorted((p.name, p.read_text()) for p in out.iterdir())
    assert got == [("0", "3 0 127.0.0.1"), ("1", "3 1 127.0.0.1"), ("2", "3 2 127.0.0.1")]
    bad = tmp_path / "bad.py"
    bad.write_text("import os, sys, time\nif os.environ['RANK'] == '1': sys.exit(7)\ntime.sleep(30)\n")
    assert spawn_workers(2, [sys.executable, str(bad)]) == 7  # rank 1 fails: rank 0 is ended, not waited for


def test_bench_refuses_mismatched_world_size():
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", "3", "--no-cpu-baseline"], env=env,
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 2 and "WORLD_SIZE=2" in r.stderr


def _job_worker(rank, ws, port, argv, q):
    sys.path[:0] = [str(ROOT), str(ROOT / "tests")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist

    import oracle_ffi
    import soundchunks_amd as sc
    from golden.cases import _tone_lsb
    from soundchunks_amd.shard import bounds_range, broadcast_bounds, gather_files, gather_streams

    dist.init_process_group("gloo", rank=rank, world_size=ws)
    try:
        wav = _tone_lsb(6.0)
        enc = sc.Encoder(argv)
        st = en = None
        if rank == 0:  # PrepareFrames of the whole file (the product's host code) on rank 0 only
            st, en = enc.prepare(wav).frame_bounds()
        st, en = broadcast_bounds(st, en)
        b, e = bounds_range(st, en, enc.chunk_size, 1, rank, ws)
        mine = enc.prepare_frames(wav, st, en, b, e)  # only this rank's samples
        assert mine.frame_count == len(st)
        blob, _ = oracle_ffi.encode_frames(wav, argv, b, e, threads=2)
        whole = gather_streams(blob)
        per_file = gather_files(b"r%d" % rank * 3, [2, 4])  # two files: 2 + 4 bytes from each rank
        if rank == 0:
            q.put((len(st), (b, e), whole, per_file))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_two_rank_job_equals_single_encode():
    import oracle_ffi
    from golden.cases import _tone_lsb

    argv = ["-cs8", "-cpf256", "-fl1000"]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 31500 + (os.getpid() % 1000)
    procs = [ctx.Process(target=_job_worker, args=(r, 2, port, argv, q)) for r in range(2)]
    for p in procs:
        p.start()
    nfr, rng0, whole, per_file = q.get(timeout=280)
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    assert nfr >= 4 and 0 < rng0[1] < nfr
    assert whole == oracle_ffi.encode(_tone_lsb(6.0), argv, threads=4)
    assert per_file == [b"r0" + b"r1", b"r0r0" + b"r1r1"]


def test_bench_frame_digest_check(tmp_path, monkeypatch):
    """bench.py's bit-exactness check splits a rank's output by the per-frame
    byte counts and compares SHA-256 digests of the frames the table lists
    (host logic; the GPU test runs it on real output)."""
    import hashlib
    import importlib.util
    import json

    spec = importlib.util.spec_from_file_location("bench_mod", ROOT / "bench.py")
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    frames = [b"frame-a" * 3, b"frame-bb", b"c" * 11]
    table = {"c2:8": {"frames": 5, "per_frame": {"2": hashlib.sha256(frames[0]).hexdigest(),
                                                 "4": hashlib.sha256(frames[2]).hexdigest()}}}
    db = tmp_path / "d.json"
    db.write_text(json.dumps(table))
    monkeypatch.setattr(bench, "DIGESTS", db)
    blob, sizes = b"".join(frames), [len(f) for f in frames]
    assert bench.frame_digest_check("c2:8", 2, blob, sizes, 5) == (2, 0, 2)  # frames 2..4, 2 and 4 listed
    bad = frames[0] + frames[1] + b"c" * 10 + b"x"
    assert bench.frame_digest_check("c2:8", 2, bad, sizes, 5) == (2, 1, 2)
    assert bench.frame_digest_check("c2:8", 2, blob, sizes, 6)[1] == 1  # another frame cut
    assert bench.frame_digest_check("c2:9", 0, blob, sizes, 5) == (0, 0, 0)  # no digests: unchecked
    assert bench.frame_digest_check("c2:8", 2, blob + b"!", sizes, 5)[1] == 1  # bytes past the frames


@pytest.mark.parametrize("args", [["--share", "1/8"], ["--share", "8/8", "--strong"],
                                  ["--share", "1/8", "--strong", "--gpus", "2"]])
def test_bench_refuses_bad_share(args):
    """--share R/N (one rank's share of the whole file on one GPU) needs
    --strong, --gpus 1 and 0 <= R < N; it is refused before any GPU call."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--no-cpu-baseline", *args], env=env,
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 2 and "--share" in r.stderr


def test_share_ranges_tile_the_whole_file():
    """Every rank's --share range of the whole file's frame cut, for N = 1, 2,
    4, 8: contiguous, in rank order, covering every frame once (the ranges an
    N-GPU strong run gives its ranks, bench.py's bounds_range)."""
    import oracle_ffi
    from soundchunks_amd.shard import bounds_range
    from soundchunks_amd.synth import synth_wav

    wav = synth_wav(120.0, 48000, 2)
    st, en = oracle_ffi.frame_bounds(wav, ["-cs4", "-cpf4096"])
    for n in (1, 2, 4, 8):
        rs = [bounds_range(st, en, 4, 2, r, n) for r in range(n)]
        assert rs[0][0] == 0 and rs[-1][1] == len(st)
        assert all(rs[r][1] == rs[r + 1][0] for r in range(n - 1))
        assert all(b < e for b, e in rs)  # 30 frames: every rank gets some


def _one_rank_worker(port, q):
    sys.path[:0] = [str(ROOT), str(ROOT / "tests")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist

    from soundchunks_amd.shard import broadcast_bounds, gather_files, gather_streams

    dist.init_process_group("gloo", rank=0, world_size=1)
    try:
        st, en = broadcast_bounds(np.array([0, 10, 20]), np.array([9, 19, 29]))
        q.put((st.tolist(), en.tolist(), gather_streams(b"abc"), gather_streams(b""),
               gather_files(b"aabbb", [2, 3])))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(120)
def test_one_rank_group_gathers():
    """bench.py at --gpus 1 under a launcher (or --dist) runs the same
    collectives in a one-rank group (RCCL on the GPU box, tests/test_gpu_rccl.py;
    gloo here): the broadcast and both gathers are the identity."""
    from soundchunks_amd.shard import free_port

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_one_rank_worker, args=(free_port(), q))
    p.start()
    st, en, whole, empty, files = q.get(timeout=100)
    p.join(30)
    assert p.exitcode == 0
    assert (st, en) == ([0, 10, 20], [9, 19, 29])
    assert whole == b"abc" and empty == b"" and files == [b"aa", b"bbb"]
