"""bench.py -- SoundChunks encode throughput on MI355X (driver contract).

Metric (BASELINE.json): encoded Msamples/s @44.1 kHz stereo, ChunkSize=8,
ChunkCount=4096 (configs[1]), bit-exact .gsc, measured from the in-memory WAV
to the .gsc bytes.

One step = one whole encode job of a synthetic WAV (SURVEY.md §8d signal:
0.25 sin(440/660 Hz) + 0.05 N(0,1), PCG64(20250217)):
  Load + PrepareFrames of the whole file (rank 0: the sequential frame-cut
  scan, encoder.lpr:1294-1429, run by gsc_prepare), the frame boundaries
  broadcast to every rank, then each rank's frame range (contiguous, balanced
  by chunk count -- SURVEY.md §8e LPT): sample staging, device DSP, yakmo +
  KNNScanReduce, KNNFit, bit packing; rank 0 gathers the frame-ordered .gsc
  bytes (torch.distributed over RCCL/xGMI).
The job's PrepareFrames is a host pass; rank 0 runs the next job's while the
GPUs encode the current one (a streaming encoder's double buffering), so the
timed region holds every job's prepare and every job's encode, and only the
first job's prepare is exposed.  `job_latency_ms` is one job run alone.

Scaling: weak by default (each rank adds --seconds of audio to one longer
file); --strong keeps one --seconds file for any world size.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--seconds S]
                  [--config c1|c2|c3|c4|c4d|c5|c5cs4|br128] [--strong] [--no-cpu-baseline]
                  [--backend nccl|gloo]

After the timed loop the last step's output is checked frame by frame against
the oracle's SHA-256 digests of the same workload (tests/golden/
bench_digests.json; c4 / c4d: corpus_meta.json / corpus_default_meta.json):
"bit_exact" in the line, and a
mismatch exits with status 3.

--gpus N without a launcher's WORLD_SIZE spawns N worker processes (one per
GPU, RANK/LOCAL_RANK/WORLD_SIZE, rendezvous at 127.0.0.1) before any GPU call.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

CONFIGS = {
    # name: (argv, channels, rate, chunk size, description)
    "c2": (["-cs8", "-cpf4096", "-cbd8"], 2, 44100, 8, "44.1 kHz stereo, ChunkSize=8 ChunkCount=4096 8-bit"),
    "c3": (["-cs16", "-cpf4096", "-cbd12"], 2, 44100, 16, "44.1 kHz stereo, ChunkSize=16 ChunkCount=4096 12-bit"),
    "c1": (["-cs8", "-cpf256"], 1, 44100, 8, "mono, ChunkSize=8 ChunkCount=256 8-bit"),
    # configs[4]'s signal (48 kHz stereo, ChunkCount=4096) at both ChunkSizes SURVEY.md §8 names
    "c5": (["-cs8", "-cpf4096"], 2, 48000, 8, "48 kHz stereo, ChunkSize=8 ChunkCount=4096"),
    "c5cs4": (["-cs4", "-cpf4096"], 2, 48000, 4, "48 kHz stereo, ChunkSize=4 ChunkCount=4096"),
    # the reference's own -br invocation (encoder/encoder.lps:270-279): ChunksPerFrame from the
    # bit-rate cost loop (encoder.lpr:1337-1351), not a power of two (485 at 44.1 kHz stereo)
    "br128": (["-br128", "-vfr0.5", "-cs8"], 2, 44100, 8, "44.1 kHz stereo, -br128 -vfr0.5 ChunkSize=8"),
    # configs[3]: the reference's lame_test corpus (22 mono 44.1 kHz files) as one batch, default flags
    "c4": (["-cs8", "-cpf4096"], 1, 44100, 8, "lame_test corpus (22 mono 44.1 kHz files), ChunkSize=8 ChunkCount=4096"),
    # configs[3] at the flags SURVEY.md §8d gives it ("all other flags default"): the encoder
    # defaults -cs4 -cpf4096 (encoder.lpr:1486-1509; encoder.lps:260 `mstest.wav -v`)
    "c4d": ([], 1, 44100, 4, "lame_test corpus (22 mono 44.1 kHz files), encoder defaults (ChunkSize=4 ChunkCount=4096)"),
}
CORPUS_CONFIGS = ("c4", "c4d")
CORPUS = ROOT / "tests" / "golden" / "lame_test"

VALU_F32_PEAK_TOPS = 78.6  # non-fused f32 VALU ops/s: half the 157.3 TFLOPS FMA-counted peak
HBM_PEAK_GBS = 8000.0      # MI355X_MICROARCH.md (spec)
PMC_SUMMARY = ROOT / "profiles" / "r06" / "pmc_summary.json"  # rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes
SQ_SUMMARY = ROOT / "profiles" / "r06" / "pmc_sq_summary.json"  # rocprofv3 --pmc SQ_* pass (tools/sq_summary.py)
DIGESTS = ROOT / "tests" / "golden" / "bench_digests.json"  # oracle per-frame .gsc digests (make_bench_digests.py)
# oracle .gsc digests of the lame_test files (tests/golden/make_corpus.py)
CORPUS_META = {"c4": ROOT / "tests" / "golden" / "corpus_meta.json",
               "c4d": ROOT / "tests" / "golden" / "corpus_default_meta.json"}


def _dist_env():
    return (int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("RANK", "0")),
            int(os.environ.get("LOCAL_RANK", "0")))


def _cpu_model() -> str:
    try:
        for line in Path("/proc/cpuinfo").read_text().splitlines():
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def _cpu_share() -> tuple[int, int, int | None]:
    """(threads to use, CPUs in the affinity mask, CPUs of the cgroup quota or
    None).  The GPU box's affinity mask lists every CPU of the host, but its
    cgroup (cpu.max) grants this job a quota (16 CPUs per GPU): more threads
    than the quota only time-slice the same CPU share."""
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:
        aff = os.cpu_count() or 1
    quota = None
    try:
        q, per = Path("/sys/fs/cgroup/cpu.max").read_text().split()[:2]
        if q != "max":
            quota = max(1, -(-int(q) // int(per)))
    except (OSError, ValueError):
        pass
    return (min(aff, quota) if quota else aff), aff, quota


def cpu_baseline(cfg: str, argv, rate: int, channels: int, frame_seconds: float, threads: int,
                 runs: int = 3) -> dict:
    """SURVEY.md §8d CPU baseline: the oracle (C restatement of the reference
    encoder, oracle/), frame-parallel like the reference's MTProcs pool
    (encoder.lpr:1449).  Single thread: `runs` independent 1-thread encodes of
    one full frame side by side on separate cores (ctypes releases the GIL),
    median.  All-core: `threads` threads on `threads` full frames of the same
    signal and flags (c4 / c4d: the corpus files in order until `threads`
    frames), median of `runs` runs."""
    import statistics
    import threading

    sys.path.insert(0, str(ROOT / "tests"))
    import oracle_ffi  # the checker / CPU baseline, never the product path
    from soundchunks_amd.synth import synth_wav

    oracle_ffi.load()
    if cfg in CORPUS_CONFIGS:
        wavs = [(CORPUS / n).read_bytes() for n in sorted(os.listdir(CORPUS)) if n.endswith(".wav")]
        nfr = [len(oracle_ffi.frame_bounds(w, argv)[0]) for w in wavs]
        one_wav = wavs[int(max(range(len(wavs)), key=lambda i: len(wavs[i]) / max(1, nfr[i])))]
        one_wav = oracle_ffi_first_frame_wav(one_wav, argv)
        sample, acc = [], 0
        for w, f in zip(wavs, nfr):
            if acc >= threads:
                break
            sample.append(w)
            acc += f
    else:
        one_wav = synth_wav(frame_seconds, rate, channels)
        sample = [synth_wav(frame_seconds * threads, rate, channels)]
    one_samples = (len(one_wav) - 44) // 2
    walls = [0.0] * runs
    stop = threading.Event()
    t_cpu = time.perf_counter()

    def heartbeat():  # minutes of CPU work print nothing else: a progress line every 30 s
        while not stop.wait(30.0):
            print(f"bench.py: cpu_baseline running, {time.perf_counter() - t_cpu:.0f} s", file=sys.stderr, flush=True)

    hb = threading.Thread(target=heartbeat, daemon=True)
    hb.start()

    def run(i):
        t = time.perf_counter()
        oracle_ffi.encode(one_wav, argv, threads=1)
        walls[i] = time.perf_counter() - t

    ths = [threading.Thread(target=run, args=(i,)) for i in range(runs)]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    w1 = statistics.median(walls)
    wns = []
    for _ in range(runs):
        t = time.perf_counter()
        if len(sample) == 1:
            oracle_ffi.encode(sample[0], argv, threads=threads)
        else:  # corpus files side by side, one encode per thread slot
            from concurrent.futures import ThreadPoolExecutor as TP

            with TP(threads) as pool:
                list(pool.map(lambda w: oracle_ffi.encode(w, argv, threads=1), sample))
        wns.append(time.perf_counter() - t)
    stop.set()
    hb.join()
    wn = statistics.median(wns)
    nsamp = sum((len(w) - 44) // 2 for w in sample)
    allv = nsamp / wn / 1e6
    _, share, quota = _cpu_share()
    what = (f"{len(sample)} corpus files ({nsamp / rate:.1f} s)" if cfg in CORPUS_CONFIGS
            else f"{threads} full {frame_seconds:g}-s frames ({frame_seconds * threads:g} s) of the same synthetic "
                 f"{rate} Hz {channels}-ch signal and flags")
    return {"value": round(allv, 6), "unit": "Msamples/s", "cores": threads, "kind": "port",
            "sample": f"all-core: {what}, oracle/ C restatement frame-parallel on {threads} threads, median of "
                      f"{runs} runs ({', '.join(f'{w:.1f}' for w in wns)} s); single-thread: one full frame, median "
                      f"of {runs} side-by-side runs",
            "single_thread": {"value": round(one_samples / w1 / 1e6, 6), "cores": 1, "wall_s": round(w1, 2),
                              "runs_s": [round(w, 2) for w in walls]},
            "all_core": {"value": round(allv, 6), "cores": threads, "wall_s": round(wn, 2),
                         "runs_s": [round(w, 2) for w in wns]},
            "cpu_model": _cpu_model(), "nproc": os.cpu_count(), "affinity_cpus": share, "cgroup_cpus": quota,
            "cores_note": "threads = the CPUs this job may use: the cgroup cpu.max quota when one is set (the GPU "
                          "box grants 16 CPUs per GPU while its affinity mask lists every host CPU), else the "
                          "affinity mask"}


def frame_digest_check(key: str, frame_begin: int, blob: bytes, sizes, frames_total: int) -> tuple[int, int, int]:
    """This rank's frames against the oracle's per-frame SHA-256 digests of the
    same workload (tests/golden/bench_digests.json; data only -- the oracle
    itself is not run here): (frames checked, frames differing, frames with a
    digest).  A .gsc is its frames' SaveStream bytes in order
    (encoder.lpr:1181-1215), so the per-frame split of the encoder's own
    output is exact."""
    import hashlib

    if not DIGESTS.exists():
        return 0, 0, 0
    ent = json.loads(DIGESTS.read_text()).get(key)
    if ent is None:
        return 0, 0, 0
    if int(ent["frames"]) != frames_total:
        return 1, 1, len(ent["per_frame"])  # a different frame cut is a mismatch
    want = ent["per_frame"]
    checked = bad = 0
    o = 0
    for i, n in enumerate(sizes):
        h = want.get(str(frame_begin + i))
        if h is not None:
            checked += 1
            if hashlib.sha256(blob[o:o + n]).hexdigest() != h:
                bad += 1
                print(f"bench.py: frame {frame_begin + i} differs from the oracle digest", file=sys.stderr)
        o += n
    if o != len(blob):
        bad += 1
    return checked, bad, len(want)


def oracle_ffi_first_frame_wav(wav: bytes, argv) -> bytes:
    """The first frame of a corpus file as its own WAV (the single-thread leg)."""
    import oracle_ffi
    import struct

    st, en = oracle_ffi.frame_bounds(wav, argv)
    ch = struct.unpack_from("<H", wav, 22)[0]
    n = int(en[0]) + 1
    body = wav[44: 44 + n * ch * 2]
    return wav[:40] + struct.pack("<I", len(body)) + body


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--seconds", type=float, default=1024.0,
                    help="audio seconds per GPU (weak) or in total (--strong); 1024 s = 256 frames of 4 s")
    ap.add_argument("--config", default="c2", choices=sorted(CONFIGS))
    ap.add_argument("--strong", action="store_true", help="one fixed-length file for any world size")
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="all-core CPU baseline threads (default: the job's CPU share, cgroup quota or affinity)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--share", default=None, metavar="R/N",
                    help="--strong on one GPU: encode only rank R of N's frame range of the whole file (the "
                         "PrepareFrames cut of the whole file, the range an N-GPU run gives rank R)")
    ap.add_argument("--dist", action="store_true",
                    help="run the torch.distributed path (bounds broadcast, all-gather) even at --gpus 1")
    ap.add_argument("--backend", default="nccl", choices=("nccl", "gloo"),
                    help="torch.distributed backend for N > 1 (nccl = RCCL over xGMI; gloo rehearses the "
                         "multi-rank path on host tensors, e.g. 2 ranks on a one-GPU box)")
    args = ap.parse_args()
    if args.cpu_threads <= 0:
        args.cpu_threads = _cpu_share()[0]

    ws, rank, local = _dist_env()
    share = None
    if args.share:
        share = tuple(int(v) for v in args.share.split("/"))
        if not (args.strong and args.gpus == 1 and len(share) == 2 and 0 <= share[0] < share[1]):
            print("bench.py: --share R/N needs --strong, --gpus 1 and 0 <= R < N", file=sys.stderr)
            sys.exit(2)
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        from soundchunks_amd.shard import spawn_workers

        sys.exit(spawn_workers(args.gpus, [sys.executable, str(Path(__file__).resolve())] + sys.argv[1:]))
    if ws != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={ws}", file=sys.stderr)
        sys.exit(2)

    import numpy as np
    import torch

    dist = None
    # one process per GPU; with more ranks than visible GPUs (the gloo rehearsal
    # on a one-GPU box) ranks share devices round-robin
    gpu = local % max(1, torch.cuda.device_count())
    dev = torch.device("cuda", gpu)
    cdev = dev if args.backend == "nccl" else torch.device("cpu")  # where the collectives' tensors live
    # the collective path runs for N > 1, and at N = 1 under a launcher
    # (WORLD_SIZE in the environment) or with --dist: a one-rank RCCL group
    # executes the same broadcast / all-gather code an N-GPU run takes
    use_dist = ws > 1 or "WORLD_SIZE" in os.environ or args.dist
    if use_dist:
        import torch.distributed as dist

        if "WORLD_SIZE" not in os.environ:  # --dist alone: a one-rank group at 127.0.0.1
            from soundchunks_amd.shard import free_port

            os.environ.update(RANK="0", LOCAL_RANK="0", WORLD_SIZE="1", MASTER_ADDR="127.0.0.1",
                              MASTER_PORT=str(free_port()))
        torch.cuda.set_device(gpu)
        dist.init_process_group(args.backend)
    import soundchunks_amd as sc
    from soundchunks_amd.shard import bounds_range, broadcast_bounds, gather_streams
    from soundchunks_amd.synth import synth_wav

    if use_dist:
        sc.set_device(gpu)

    argv, ch, rate, cs, desc = CONFIGS[args.config]
    enc = sc.Encoder(argv)
    if args.config in CORPUS_CONFIGS:
        return bench_corpus(args, enc, argv, desc, ws, rank, cdev, dist, cs)
    total_seconds = args.seconds if args.strong else args.seconds * ws
    wav = synth_wav(total_seconds, rate, ch)  # the job's input, in host memory on every rank

    pool = ThreadPoolExecutor(1) if rank == 0 else None

    def prepare_job():  # rank 0: Load + PrepareFrames of the whole file (encoder.lpr:1111-1152, 1294-1429)
        t = time.perf_counter()
        p = enc.prepare(wav)
        st, en = p.frame_bounds()
        return p, st, en, (time.perf_counter() - t) * 1e3

    info = {}

    def step(fut, prefetch: bool):
        """One job: consume this job's prepare (rank 0), start the next one's,
        broadcast the frame bounds, encode this rank's frames, gather."""
        p = st = en = None
        nxt = None
        if rank == 0:
            p, st, en, info["prepare_ms"] = fut.result()
            if prefetch:
                nxt = pool.submit(prepare_job)
        if dist is not None:  # rank 0's PrepareFrames boundaries to every rank
            st, en = broadcast_bounds(st, en, device=cdev)
        b, e = bounds_range(st, en, cs, ch, *(share or (rank, ws)))
        info["frames"], info["range"] = len(st), (b, e)
        info["range_samples"] = int(sum(int(en[f]) - int(st[f]) + 1 for f in range(b, e))) * ch
        t_enc = time.perf_counter()
        if rank == 0:
            out, sizes = p.encode_frames(b, e)
        else:
            out, sizes = enc.prepare_frames(wav, st, en, b, e).encode_frames(b, e)
        info["own"] = (b, out, sizes)
        if os.environ.get("BENCH_STEP_TIMING"):  # diagnostic: the encode call inside the step
            print(f"step: encode call {(time.perf_counter() - t_enc) * 1e3:.1f} ms", file=sys.stderr, flush=True)
        if dist is not None:
            out = gather_streams(out, device=cdev)
        return out, nxt

    # warmup (untimed): the first one, run alone, is the single-job latency
    lat = None
    for w in range(args.warmup):
        t = time.perf_counter()
        step(pool.submit(prepare_job) if rank == 0 else None, False)
        torch.cuda.synchronize()
        if w == 0:
            lat = (time.perf_counter() - t) * 1e3
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    fut = pool.submit(prepare_job) if rank == 0 else None
    timings = []
    whole = None
    for k in range(args.steps):
        t_step = time.perf_counter()
        whole, fut = step(fut, k + 1 < args.steps)
        timings.append(sc.Encoder.last_timing())
        if os.environ.get("BENCH_STEP_TIMING"):
            print(f"step: {(time.perf_counter() - t_step) * 1e3:.1f} ms", file=sys.stderr, flush=True)
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    dt = time.perf_counter() - t0
    if dist is not None:
        t = torch.tensor([dt], device=cdev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    # bit-exactness of the last timed step's output (after the clock stopped):
    # every rank checks its own frames against the oracle digests, rank 0 also
    # the length of the gathered file when every frame has a digest
    key = f"{args.config}:{total_seconds:g}"
    fb, blob, sizes = info["own"]
    if os.environ.get("BENCH_DUMP"):  # diagnostic: this rank's bytes and per-frame sizes of the last step
        Path(os.environ["BENCH_DUMP"] + f".r{rank}.gsc").write_bytes(blob)
        Path(os.environ["BENCH_DUMP"] + f".r{rank}.json").write_text(json.dumps({"first": fb, "sizes": sizes}))
    checked, bad, listed = frame_digest_check(key, fb, blob, sizes, info["frames"])
    if dist is not None:
        t = torch.tensor([checked, bad], dtype=torch.int64, device=cdev)
        dist.all_reduce(t)
        checked, bad = (int(v) for v in t.tolist())
    if rank != 0:
        dist.destroy_process_group()
        if bad:
            sys.exit(3)
        return
    if share is None and listed == info["frames"] and checked == listed:
        want_len = json.loads(DIGESTS.read_text())[key].get("total_bytes")
        if want_len is not None and len(whole) != int(want_len):
            bad += 1
    n_samples = int(round(total_seconds * rate)) * ch
    if share is not None:  # one rank's share: the samples of its frames
        n_samples = info["range_samples"]
    value = n_samples * args.steps / dt / 1e6
    result = base_result(args, ws, dt, value, desc, enc, timings[-1], cs, argv, rate, ch)
    result["config"] = {"workload": f"{desc}, {total_seconds:g} s synthetic", "frames": info["frames"],
                        "argv": argv, "parallelism": f"frame-sharded x{ws}", "rank0_frames": list(info["range"]),
                        "collectives": args.backend if dist is not None else None}
    if share is not None:
        result["config"]["share"] = {"rank": share[0], "of": share[1], "frames": list(info["range"]),
                                     "samples": n_samples,
                                     "note": "rank R of N's frame range of the whole file's PrepareFrames cut, "
                                             "encoded alone on one GPU (prepare of the whole file included)"}
    result["data"] = (f"synthetic (SURVEY.md §8d tone+noise, PCG64 20250217), "
                      f"{total_seconds:g} s {'in total' if args.strong else f'= {args.seconds:g} s per GPU'}")
    result["prepare_ms"] = round(info["prepare_ms"], 1)
    result["job_latency_ms"] = None if lat is None else round(lat, 1)
    result["realtime_x"] = round(value / (rate * ch / 1e6), 2)
    result["bit_exact"] = (bad == 0) if checked else None
    result["bit_exact_check"] = {
        "digests": f"tests/golden/bench_digests.json[{key}] (oracle SaveStream bytes per frame)",
        "frames_checked": checked, "frames_differing": bad, "frames_total": info["frames"],
        "whole_file": checked == info["frames"],
        "range_checked": checked == info["range"][1] - info["range"][0],
        "note": None if checked else "no oracle digests for this workload: not checked"}
    if not args.no_cpu_baseline:
        result["cpu_baseline"] = cpu_baseline(args.config, argv, rate, ch, enc.frame_length / 1000.0,
                                              args.cpu_threads)
    print(json.dumps(result))
    if dist is not None:
        dist.destroy_process_group()
    if bad:
        print(f"bench.py: {bad} frame(s) differ from the oracle digests", file=sys.stderr)
        sys.exit(3)


def base_result(args, ws, dt, value, desc, enc, tm, cs, argv, rate, ch) -> dict:
    # dominant kernel: KNNScanReduce passes; algorithmic ops = searches x K x 2CS x 3
    # (sub + mul + add per feature, SURVEY.md §8d: 6K ops per input sample per pass)
    K = enc.options.chunks_per_frame
    ops = tm["scan_point_passes"] * K * (2 * cs) * 3
    scan_s = tm["gpu_scan_ms"] / 1e3
    launches = max(1, tm["scan_launches"])
    achieved = (ops / scan_s / 1e12) if scan_s > 0 else 0.0
    avg_launch_s = scan_s / launches
    # HBM traffic of the scan kernel per launch: PMC bytes per frame (committed
    # rocprofv3 summary, gfx950-corrected) x frames in this launch
    traffic = None
    if PMC_SUMMARY.exists():
        ks = json.loads(PMC_SUMMARY.read_text())["kernels"]
        kern = next((v for k, v in ks.items()
                     if k.startswith("gsc::scan_batch_kernel") and (f"<{2 * cs}, 12," in k or f"<{2 * cs}, 12>" in k)),
                    None)
        if kern and K == 4096:
            traffic = kern["hbm_bytes_per_frame_per_launch"] * tm["reduce_frames"]
    # VALU issue fraction of the scan kernel from the committed SQ pass (VALU
    # wave-instructions x 2 cycles / (4 SIMDs x CUs x launch cycles)) -- a profile
    # of the C2 shape, so it is attached to the C2 line only, with its source
    issue = sq = None
    if SQ_SUMMARY.exists() and args.config == "c2":
        sq = json.loads(SQ_SUMMARY.read_text())
        issue = sq.get("scan_valu_issue_frac")
    metric = "encoded Msamples/s @44.1kHz stereo ChunkSize=8 ChunkCount=4096; bit-exact .gsc"  # BASELINE.json
    if args.config != "c2":
        metric = f"encoded Msamples/s ({desc}); bit-exact .gsc"
    return {
        "metric": metric,
        "value": round(value, 4),
        "unit": "Msamples/s",
        "n_gpus": ws,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(dt * 1e3 / args.steps, 2),
        "higher_is_better": True,
        "scaling": "strong" if args.strong else "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "roofline": {"bound": "valu", "kernel": "scan_batch_kernel", "achieved": round(achieved, 4),
                     "peak": VALU_F32_PEAK_TOPS,
                     "unit": "Tops/s (algorithmic: the reference's sub+mul+add per leaf coordinate, 6K ops per "
                             "sample per pass; peak = non-fused f32 VALU issue rate; the kernel itself bounds "
                             "distances with one fma per coordinate and recomputes exactly only what it commits)",
                     "frac": round(achieved / VALU_F32_PEAK_TOPS, 5),
                     "traffic": None if traffic is None else round(traffic),
                     "hbm_gbs": None if traffic is None or avg_launch_s <= 0 else round(traffic / avg_launch_s / 1e9, 2),
                     "hbm_frac": None if traffic is None or avg_launch_s <= 0 else
                     round(traffic / avg_launch_s / 1e9 / HBM_PEAK_GBS, 6),
                     "avg_launch_ms": round(avg_launch_s * 1e3, 3), "ops_per_launch": ops / launches,
                     "profiled_c2_valu_issue_frac": None if issue is None else round(issue, 4),
                     "valu_issue_note": None if issue is None else
                     f"from the committed SQ pass {SQ_SUMMARY.relative_to(ROOT)} (C2 shape, build "
                     f"{sq.get('source_commit', 'unrecorded')}), not this run: SQ_INSTS_VALU x 2 cycles / (4 SIMDs x "
                     f"frames x launch cycles at 2.4 GHz); frac above counts the reference's brute-force ops, which "
                     f"the kernel does not execute"},
        # host_post_ms: what the KNNFit / prune / packing pipeline adds after the
        # scan; post_overlap_ms: the part of it that ran in the scan tail
        "stages_ms": {k: round(tm[k], 1) for k in ("host_frames_ms", "gpu_dsp_ms", "gpu_yakmo_ms", "gpu_scan_ms",
                                                    "gpu_knnfit_ms", "host_post_ms", "post_overlap_ms", "total_ms")},
        "post_groups": tm["post_groups"],
        "stages_note": ("stages of rank 0's last encode: host_frames, gpu_dsp, gpu_yakmo, gpu_scan and host_post run "
                        "in series; gpu_knnfit_ms is submit-to-done of the KNNFit groups, which run on the CUs of "
                        "finished frames during the scan tail (post_overlap_ms), so it is not additive; PrepareFrames "
                        "(prepare_ms) overlaps the previous job's encode"),
        "scan": {"passes": tm["scan_passes"], "searches": tm["scan_point_passes"], "exact_dfs": tm["scan_slow"],
                 "solo_resolutions": tm["scan_restarts"]},
    }


def bench_corpus(args, enc, argv, desc, ws, rank, cdev, dist, cs):
    """configs[3]: the 22-file lame_test corpus as ONE batch -- every frame of
    every file in one device launch per stage (gsc_encode_many), frames of the
    batch sharded across ranks by chunk count, one .gsc per file on rank 0."""
    import torch

    import soundchunks_amd as sc

    names = sorted(n for n in os.listdir(CORPUS) if n.endswith(".wav"))
    wavs = [(CORPUS / n).read_bytes() for n in names]

    def step():
        return sc.encode_many(wavs, argv, rank=rank, world_size=ws, device=cdev if dist is not None else None)

    lat = None
    for w in range(args.warmup):
        t = time.perf_counter()
        step()
        torch.cuda.synchronize()
        if w == 0:
            lat = (time.perf_counter() - t) * 1e3
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        outs = step()
    tm = sc.Encoder.last_timing()
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    dt = time.perf_counter() - t0
    if dist is not None:
        t = torch.tensor([dt], device=cdev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    if rank != 0:
        dist.destroy_process_group()
        return
    n_samples = sum((len(w) - 44) // 2 for w in wavs)
    value = n_samples * args.steps / dt / 1e6
    result = base_result(args, ws, dt, value, desc, enc, tm, cs, argv, 44100, 1)
    result["config"] = {"workload": f"{desc}, {n_samples / 44100:.1f} s of audio in {len(wavs)} files",
                        "files": len(wavs), "frames": tm["frames"], "argv": argv,
                        "parallelism": f"frame-sharded x{ws}", "collectives": args.backend if dist is not None else None}
    result["data"] = "the reference's lame_test corpus WAVs (tests/golden/lame_test), encoded as one batch"
    result["job_latency_ms"] = None if lat is None else round(lat, 1)
    result["realtime_x"] = round(value / (44100 / 1e6), 2)
    result["outputs_bytes"] = sum(len(o) for o in outs)
    # every file's .gsc of the last timed step against the oracle's digest
    import hashlib

    meta_path = CORPUS_META[args.config]
    meta = json.loads(meta_path.read_text())
    bad = sum(hashlib.sha256(o).hexdigest() != meta["files"][n]["gsc_sha256"] for n, o in zip(names, outs))
    if meta["argv"] != list(argv):
        bad = len(names)
    result["bit_exact"] = bad == 0
    result["bit_exact_check"] = {"digests": f"tests/golden/{meta_path.name} (oracle .gsc per file)",
                                 "files_checked": len(names), "files_differing": bad, "whole_file": True}
    if not args.no_cpu_baseline:
        result["cpu_baseline"] = cpu_baseline(args.config, argv, 44100, 1, enc.frame_length / 1000.0, args.cpu_threads)
    print(json.dumps(result))
    if dist is not None:
        dist.destroy_process_group()
    if bad:
        print(f"bench.py: {bad} corpus file(s) differ from the oracle digests", file=sys.stderr)
        sys.exit(3)


if __name__ == "__main__":
    main()
