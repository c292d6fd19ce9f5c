"""The RCCL (torch.distributed "nccl") path on the GPU, at world size 1.

An 8-GPU driver run shards frames over ranks (encoder.lpr:1449 fan-out,
SURVEY.md §8e): rank 0's PrepareFrames bounds go out with `broadcast_bounds`,
the per-rank bytes come back with `gather_streams` / `gather_files`, all on
device tensors over RCCL.  The multi-rank tests elsewhere use gloo on host
tensors (two ranks cannot form an RCCL group on one GPU), so this file runs
the same functions in a one-rank RCCL group on device 0: the collectives,
the device-tensor staging and the byte reassembly execute exactly as they do
on every rank of an N-GPU run, and the result is checked against the goldens.
"""
from __future__ import annotations

import hashlib
import json
import os
import subprocess
import sys
from pathlib import Path

import pytest
import torch.multiprocessing as mp

ROOT = Path(__file__).resolve().parents[1]
GOLD = ROOT / "tests" / "golden"


def _rccl_worker(port, q):
    sys.path[:0] = [str(ROOT), str(ROOT / "tests")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import numpy as np
    import torch
    import torch.distributed as dist

    import soundchunks_amd as sc
    from soundchunks_amd.shard import bounds_range, broadcast_bounds, gather_files, gather_streams
    from soundchunks_amd.synth import synth_wav

    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1)
    dev = torch.device("cuda", 0)
    res = {"backend": dist.get_backend()}
    try:
        # bench.py's C2 job at 16 s: prepare, broadcast, encode the rank's range, gather
        enc = sc.Encoder(["-cs8", "-cpf4096", "-cbd8"])
        wav = synth_wav(16.0, 44100, 2)
        p = enc.prepare(wav)
        st, en = p.frame_bounds()
        st2, en2 = broadcast_bounds(st, en, device=dev)
        res["bounds_equal"] = bool(np.array_equal(np.asarray(st), st2) and np.array_equal(np.asarray(en), en2))
        b, e = bounds_range(st2, en2, 8, 2, 0, 1)
        out, sizes = p.encode_frames(b, e)
        whole = gather_streams(out, device=dev)
        res["frames"] = [b, e]
        o, digests = 0, []
        for n in sizes:
            digests.append(hashlib.sha256(whole[o:o + n]).hexdigest())
            o += n
        res["frame_digests"] = digests
        res["whole_len"] = len(whole)
        # an empty shard (a rank with no frames) still takes part in the gather
        res["empty_gather"] = gather_streams(b"", device=dev)
        # the corpus batch: per-file reassembly through gather_files on device tensors
        names = ["castanets.wav", "hihat.wav", "mstest.wav", "testsignal2.wav"]
        meta = json.loads((GOLD / "corpus_meta.json").read_text())
        wavs = [(GOLD / "lame_test" / n).read_bytes() for n in names]
        outs = sc.encode_many(wavs, meta["argv"], rank=0, world_size=1, device=dev)
        res["corpus"] = [hashlib.sha256(x).hexdigest() for x in outs]
        # gather_files with an explicit size table (files split at arbitrary byte counts)
        blob = b"".join(outs)
        res["files_roundtrip"] = gather_files(blob, [len(x) for x in outs], device=dev) == outs
        q.put(res)
    except Exception as ex:  # surface the failure to the test instead of a queue timeout
        q.put({"error": repr(ex)})
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.timeout(400)
def test_rccl_world1_broadcast_gather_match_goldens():
    from soundchunks_amd.shard import free_port

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_rccl_worker, args=(free_port(), q))
    p.start()
    res = q.get(timeout=380)
    p.join(60)
    assert "error" not in res, res.get("error")
    assert p.exitcode == 0
    assert res["backend"] == "nccl"
    assert res["bounds_equal"]
    db = json.loads((GOLD / "bench_digests.json").read_text())["c2:16"]
    b, e = res["frames"]
    assert (b, e) == (0, db["frames"])
    assert res["frame_digests"] == [db["per_frame"][str(f)] for f in range(b, e)]
    assert res["whole_len"] == db["total_bytes"]
    assert res["empty_gather"] == b""
    meta = json.loads((GOLD / "corpus_meta.json").read_text())
    names = ["castanets.wav", "hihat.wav", "mstest.wav", "testsignal2.wav"]
    assert res["corpus"] == [meta["files"][n]["gsc_sha256"] for n in names]
    assert res["files_roundtrip"]


@pytest.mark.gpu
@pytest.mark.timeout(420)
def test_bench_takes_the_rccl_path_at_world_size_1():
    """bench.py under a launcher's environment (WORLD_SIZE=1) initialises the
    RCCL group and runs broadcast + all-gather + the max-over-ranks timing on
    device tensors; the line stays bit-exact."""
    from soundchunks_amd.shard import free_port

    env = dict(os.environ, RANK="0", LOCAL_RANK="0", WORLD_SIZE="1", LOCAL_WORLD_SIZE="1",
               MASTER_ADDR="127.0.0.1", MASTER_PORT=str(free_port()))
    r = subprocess.run([sys.executable, "-u", str(ROOT / "bench.py"), "--steps", "1", "--warmup", "0",
                        "--no-cpu-baseline", "--seconds", "16"], capture_output=True, text=True, timeout=400,
                       env=env)
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert r.returncode == 0, r.stderr[-3000:]
    res = json.loads(lines[-1])
    assert res["config"]["collectives"] == "nccl"
    assert res["bit_exact"] is True and res["bit_exact_check"]["whole_file"]
