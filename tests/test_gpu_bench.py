"""bench.py and the multi-rank job on the GPU: the bench line proves its own
output bit-exact (per-frame oracle digests, tests/golden/bench_digests.json),
the --gpus N launcher runs N ranks over gloo on the one-GPU box (ranks share
device 0; the RCCL backend is the same code with device tensors), and the
C4-style corpus batch sharded over 2 ranks gives every file's oracle .gsc
(tests/golden/corpus_meta.json)."""
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


def _bench(*args, timeout=400):
    r = subprocess.run([sys.executable, "-u", str(ROOT / "bench.py"), "--steps", "1", "--warmup", "0",
                        "--no-cpu-baseline", *args], capture_output=True, text=True, timeout=timeout)
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert r.returncode == 0, r.stderr[-3000:]
    assert lines, r.stdout[-2000:]
    return json.loads(lines[-1])


def test_digest_table_covers_the_test_workloads():
    """The digests the GPU tests below check against exist (oracle output,
    generated in the build container by make_bench_digests.py)."""
    db = json.loads((GOLD / "bench_digests.json").read_text())
    for key in ("c2:16", "c2:32"):
        ent = db[key]
        assert len(ent["per_frame"]) == ent["frames"] and ent["total_bytes"] > 0


@pytest.mark.gpu
@pytest.mark.timeout(420)
def test_bench_line_is_bit_exact():
    res = _bench("--seconds", "16")
    assert res["n_gpus"] == 1 and res["bit_exact"] is True
    chk = res["bit_exact_check"]
    assert chk["whole_file"] and chk["frames_checked"] == chk["frames_total"] >= 4 and chk["frames_differing"] == 0


@pytest.mark.gpu
@pytest.mark.timeout(420)
def test_bench_two_ranks_over_gloo_is_bit_exact():
    """bench.py --gpus 2 spawns two ranks (both on device 0 here): rank 0 runs
    PrepareFrames and broadcasts the bounds, each rank encodes its frames, the
    bytes are gathered, and every frame of the 32-s weak-scaling file matches."""
    res = _bench("--gpus", "2", "--backend", "gloo", "--seconds", "16")
    assert res["n_gpus"] == 2 and res["bit_exact"] is True
    assert res["config"]["frames"] == res["bit_exact_check"]["frames_checked"]
    assert 0 < res["config"]["rank0_frames"][1] < res["config"]["frames"]


def _corpus_worker(rank, ws, port, names, q):
    sys.path[:0] = [str(ROOT), str(ROOT / "tests")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist

    import soundchunks_amd as sc

    dist.init_process_group("gloo", rank=rank, world_size=ws)
    try:
        wavs = [(GOLD / "lame_test" / n).read_bytes() for n in names]
        meta = json.loads((GOLD / "corpus_meta.json").read_text())
        outs = sc.encode_many(wavs, meta["argv"], rank=rank, world_size=ws)
        if rank == 0:
            q.put([hashlib.sha256(o).hexdigest() for o in outs])
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.timeout(400)
def test_corpus_batch_two_ranks_matches_oracle():
    """encode_many(world_size=2): 4 corpus files as one frame list, sharded by
    chunk count across 2 ranks, gathered per file on rank 0."""
    names = ["castanets.wav", "hihat.wav", "mstest.wav", "testsignal2.wav"]
    meta = json.loads((GOLD / "corpus_meta.json").read_text())
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 32500 + (os.getpid() % 1000)
    procs = [ctx.Process(target=_corpus_worker, args=(r, 2, port, names, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = q.get(timeout=380)
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    assert got == [meta["files"][n]["gsc_sha256"] for n in names]
