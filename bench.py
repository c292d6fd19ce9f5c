"""bench.py -- SoundChunks encode throughput on MI355X (driver contract).

Metric (BASELINE.json): encoded Msamples/s @44.1 kHz stereo, ChunkSize=8,
ChunkCount=4096 (configs[1]), bit-exact .gsc.  One step = one full encode of
this rank's share of a synthetic 44.1 kHz stereo signal (SURVEY.md §8d:
0.25 sin(440/660 Hz) + 0.05 N(0,1), PCG64(20250217)): host pre-pass, per-frame
DSP, GPU Reduce (yakmo + KNNScanReduce) and KNNFit, bit packing.  Frames are
independent: with N GPUs each rank encodes a contiguous frame range of an
N-times longer signal (weak scaling) and rank 0 gathers the per-frame .gsc
bytes (torch.distributed over RCCL/xGMI).

python bench.py [--gpus N] [--steps K] [--warmup W] [--seconds S] [--config c2|c3|c1]
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
}

VALU_F32_PEAK_TOPS = 78.6  # non-fused f32 VALU ops/s: half the 157.3 TFLOPS FMA-counted peak
HBM_PEAK_GBS = 8000.0      # MI355X_MICROARCH.md (spec)
PMC_SUMMARY = ROOT / "profiles" / "r01" / "pmc_summary.json"  # rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes


def _dist_env():
    return (int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("RANK", "0")),
            int(os.environ.get("LOCAL_RANK", "0")))


def cpu_baseline(argv, seconds: float, rate: int, channels: int) -> dict:
    """Oracle (C restatement, 1 thread) on a bounded sample of the same signal."""
    sys.path.insert(0, str(ROOT / "tests"))
    import oracle_ffi  # the checker / CPU baseline, never the product path
    from soundchunks_amd.synth import synth_wav

    wav = synth_wav(seconds, rate, channels)
    t = time.time()
    oracle_ffi.encode(wav, argv, threads=1)
    dt = time.time() - t
    samples = int(round(seconds * rate)) * channels
    return {"value": round(samples / dt / 1e6, 6), "unit": "Msamples/s", "cores": 1, "kind": "port",
            "sample": f"{seconds:g} s of the same synthetic {rate} Hz {channels}-ch signal and flags, "
                      f"oracle/ C restatement on 1 host thread, {dt:.1f} s wall"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--seconds", type=float, default=1024.0,
                    help="audio seconds per GPU (1024 s = 256 frames of 4 s: one frame per CU)")
    ap.add_argument("--config", default="c2", choices=sorted(CONFIGS))
    ap.add_argument("--cpu-seconds", type=float, default=1.5,
                    help="oracle baseline sample: 1.5 s = one 16.5k-chunk frame at the same flags, ~25 s of CPU")
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
    from soundchunks_amd.shard import frame_range, gather_streams
    from soundchunks_amd.synth import synth_wav

    if ws > 1:
        sc.set_device(local)

    argv, ch, rate, cs, desc = CONFIGS[args.config]
    total_seconds = args.seconds * ws
    wav = synth_wav(total_seconds, rate, ch)
    enc = sc.Encoder(argv)
    nframes = enc.frame_count(wav)
    b, e = frame_range(nframes, rank, ws)

    def step():
        out = enc.encode(wav, b, e)
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
        kern = json.loads(PMC_SUMMARY.read_text())["kernels"].get(f"gsc::scan_batch_kernel<{2 * cs}, 12>")
        if kern:
            traffic = kern["hbm_bytes_per_frame_per_launch"] * tm["reduce_frames"]
    result = {
        "metric": "encoded Msamples/s @44.1kHz stereo ChunkSize=8 ChunkCount=4096; bit-exact .gsc",
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
                   "parallelism": f"frame-sharded x{ws}"},
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
        "stages_ms": {k: round(tm[k], 1) for k in ("host_prepare_ms", "host_frames_ms", "gpu_dsp_ms", "gpu_yakmo_ms",
                                                    "gpu_scan_ms", "gpu_knnfit_ms", "host_post_ms", "total_ms")},
        "scan": {"passes": tm["scan_passes"], "searches": tm["scan_point_passes"], "exact_dfs": tm["scan_slow"],
                 "solo_resolutions": tm["scan_restarts"]},
    }
    if not args.no_cpu_baseline:
        result["cpu_baseline"] = cpu_baseline(argv, args.cpu_seconds, rate, ch)
    print(json.dumps(result))
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
