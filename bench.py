"""bench.py -- SoundChunks encode throughput on MI355X (driver contract).

Metric (BASELINE.json): encoded Msamples/s @44.1 kHz stereo, ChunkSize=8,
ChunkCount=4096 (configs[1]), bit-exact .gsc.  The job's one-off host pass
(Load + PrepareFrames: the sequential frame-boundary scan of the whole file,
encoder.lpr:1294-1429) runs once before timing and is reported as prepare_ms.
One step = one encode of this rank's frames of a synthetic 44.1 kHz stereo
signal (0.25 sin(440/660 Hz) + 0.05 N(0,1), PCG64(20250217)):
per-frame sample staging and DSP, GPU Reduce (yakmo + KNNScanReduce) and
KNNFit, bit packing.  Frames are independent: with N GPUs each rank encodes a
contiguous frame range (balanced by chunk count) of an N-times longer signal
(weak scaling) and rank 0 gathers the per-frame .gsc bytes (torch.distributed
over RCCL/xGMI).

python bench.py [--gpus N] [--steps K] [--warmup W] [--seconds S] [--config c2|c3|c1|c5|c5cs4]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
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
}

VALU_F32_PEAK_TOPS = 78.6  # non-fused f32 VALU ops/s: half the 157.3 TFLOPS FMA-counted peak
HBM_PEAK_GBS = 8000.0      # MI355X_MICROARCH.md (spec)
PMC_SUMMARY = ROOT / "profiles" / "r02" / "pmc_summary.json"  # rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes


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


def cpu_baseline(argv, rate: int, channels: int, frame_seconds: float, threads: int, runs: int = 3) -> dict:
    """SURVEY.md §8d CPU baseline: the oracle (C restatement of the reference
    encoder, oracle/), frame-parallel like the reference's MTProcs pool
    (encoder.lpr:1449).  Single thread: `runs` independent 1-thread encodes of
    one full frame, run side by side on separate cores (ctypes releases the
    GIL), median.  All-core: `threads` threads on `threads` full frames of the
    same signal and flags, one run (a full frame takes ~1.5 min on one core, so
    three all-core runs would triple the bench's wall time)."""
    import statistics
    import threading

    sys.path.insert(0, str(ROOT / "tests"))
    import oracle_ffi  # the checker / CPU baseline, never the product path
    from soundchunks_amd.synth import synth_wav

    oracle_ffi.load()
    one_wav = synth_wav(frame_seconds, rate, channels)
    one_samples = int(round(frame_seconds * rate)) * channels
    walls = [0.0] * runs

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
    many = frame_seconds * threads
    wav = synth_wav(many, rate, channels)
    t = time.perf_counter()
    oracle_ffi.encode(wav, argv, threads=threads)
    wn = time.perf_counter() - t
    allv = int(round(many * rate)) * channels / wn / 1e6
    try:
        share = len(os.sched_getaffinity(0))
    except AttributeError:
        share = os.cpu_count()
    return {"value": round(allv, 6), "unit": "Msamples/s", "cores": threads, "kind": "port",
            "sample": f"all-core: {threads} full {frame_seconds:g}-s frames ({many:g} s) of the same synthetic "
                      f"{rate} Hz {channels}-ch signal and flags, oracle/ C restatement frame-parallel on {threads} "
                      f"threads, 1 run ({wn:.1f} s); single-thread: one full frame, median of {runs} side-by-side runs",
            "single_thread": {"value": round(one_samples / w1 / 1e6, 6), "cores": 1, "wall_s": round(w1, 2),
                              "runs_s": [round(w, 2) for w in walls], "seconds_of_audio": frame_seconds},
            "all_core": {"value": round(allv, 6), "cores": threads, "wall_s": round(wn, 2), "seconds_of_audio": many},
            "cpu_model": _cpu_model(), "nproc": os.cpu_count(), "affinity_cpus": share}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--seconds", type=float, default=1024.0,
                    help="audio seconds per GPU (1024 s = 256 frames of 4 s: one frame per CU)")
    ap.add_argument("--config", default="c2", choices=sorted(CONFIGS))
    ap.add_argument("--cpu-threads", type=int, default=16,
                    help="all-core CPU baseline threads (the GPU box's CPU share is 16 per GPU)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    args = ap.parse_args()

    ws, rank, local = _dist_env()
    import torch

    dist = None
    if ws > 1:
        import torch.distributed as dist

        torch.cuda.set_device(local)
        dist.init_process_group("nccl")
    import soundchunks_amd as sc
    from soundchunks_amd.shard import frame_range_weighted, gather_streams
    from soundchunks_amd.synth import synth_wav

    if ws > 1:
        sc.set_device(local)

    argv, ch, rate, cs, desc = CONFIGS[args.config]
    total_seconds = args.seconds * ws
    wav = synth_wav(total_seconds, rate, ch)
    enc = sc.Encoder(argv)
    # Load + PrepareFrames once per job (the sequential frame-boundary scan of
    # the whole file, encoder.lpr:1294-1429); each step encodes this rank's
    # frame range, balanced by chunk count (SURVEY.md §8e LPT)
    prep = enc.prepare(wav)
    nframes = prep.frame_count
    b, e = frame_range_weighted(prep.frame_chunks().tolist(), rank, ws)

    def step():
        out = prep.encode(b, e)
        if dist is not None:  # frame-ordered .gsc on rank 0: one padded all-gather (RCCL over xGMI)
            out = gather_streams(out, device=torch.device("cuda", local))
        return out

    for _ in range(args.warmup):
        step()
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    timings = []
    for _ in range(args.steps):
        step()
        timings.append(sc.Encoder.last_timing())
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    dt = time.perf_counter() - t0
    if dist is not None:
        t = torch.tensor([dt], device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    if rank != 0:
        dist.destroy_process_group()
        return

    n_samples = int(round(total_seconds * rate)) * ch
    value = n_samples * args.steps / dt / 1e6
    tm = timings[-1]
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
        # the scan kernel's instance at this D and K = 4096 (ScanCfg<D, 12, slots, CUs>)
        kern = next((v for k, v in ks.items()
                     if k.startswith("gsc::scan_batch_kernel") and (f"<{2 * cs}, 12," in k or f"<{2 * cs}, 12>" in k)),
                    None)
        if kern:
            traffic = kern["hbm_bytes_per_frame_per_launch"] * tm["reduce_frames"]
    metric = "encoded Msamples/s @44.1kHz stereo ChunkSize=8 ChunkCount=4096; bit-exact .gsc"  # BASELINE.json
    if args.config != "c2":
        metric = f"encoded Msamples/s ({desc}); bit-exact .gsc"
    result = {
        "metric": metric,
        "value": round(value, 4),
        "unit": "Msamples/s",
        "n_gpus": ws,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(dt * 1e3 / args.steps, 2),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": f"synthetic (SURVEY.md §8d tone+noise, PCG64 20250217), {args.seconds:g} s per GPU",
        "config": {"workload": f"{desc}, {total_seconds:g} s synthetic", "frames": nframes, "argv": argv,
                   "parallelism": f"frame-sharded x{ws}", "rank0_frames": [b, e]},
        "prepare_ms": round(prep.prepare_ms, 1),
        "realtime_x": round(value / (rate * ch / 1e6), 2),
        "roofline": {"bound": "valu", "kernel": "scan_batch_kernel", "achieved": round(achieved, 4),
                     "peak": VALU_F32_PEAK_TOPS, "unit": "Tops/s (algorithmic: the reference's sub+mul+add per leaf coordinate, 6K ops per sample per "
                             "pass; peak = non-fused f32 VALU issue rate; the kernel itself bounds distances with one "
                             "fma per coordinate and recomputes exactly only what it commits)",
                     "frac": round(achieved / VALU_F32_PEAK_TOPS, 5),
                     "traffic": None if traffic is None else round(traffic),
                     "hbm_gbs": None if traffic is None else round(traffic / avg_launch_s / 1e9, 2),
                     "hbm_frac": None if traffic is None else round(traffic / avg_launch_s / 1e9 / HBM_PEAK_GBS, 6),
                     "avg_launch_ms": round(avg_launch_s * 1e3, 3), "ops_per_launch": ops / launches},
        # host_post_ms: what the KNNFit / prune / packing pipeline adds after the
        # scan; post_overlap_ms: the part of it that ran in the scan tail
        "stages_ms": {k: round(tm[k], 1) for k in ("host_prepare_ms", "host_frames_ms", "gpu_dsp_ms", "gpu_yakmo_ms",
                                                    "gpu_scan_ms", "gpu_knnfit_ms", "host_post_ms", "post_overlap_ms",
                                                    "total_ms")},
        "post_groups": tm["post_groups"],
        "stages_note": ("host_frames, gpu_dsp, gpu_yakmo, gpu_scan and host_post run in series; gpu_knnfit_ms is "
                        "submit-to-done of the KNNFit groups, which run on the CUs of finished frames during the "
                        "scan tail (post_overlap_ms), so it is not additive"),
        "scan": {"passes": tm["scan_passes"], "searches": tm["scan_point_passes"], "exact_dfs": tm["scan_slow"],
                 "solo_resolutions": tm["scan_restarts"]},
    }
    if not args.no_cpu_baseline:
        result["cpu_baseline"] = cpu_baseline(argv, rate, ch, enc.frame_length / 1000.0, args.cpu_threads)
    print(json.dumps(result))
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
