"""Bit-exactness diagnosis of single frames of a bench workload (GPU box or
build container).

    python tools/frame_probe.py diff DUMP_PREFIX [config seconds]     # which frames of a bench dump differ
    python tools/frame_probe.py probe FRAME [FRAME ...] [--config c2 --seconds 1024]   # GPU: stage by stage

`diff` compares a `BENCH_DUMP` (bench.py: the last step's bytes + per-frame
sizes) with tests/golden/bench_digests.json.  `probe` cuts frame i of the
bench's synthetic file into a WAV of its own (the frame's samples; -fl large
enough that PrepareFrames keeps one frame, checked with the oracle), then
compares the HIP path with the oracle (test infrastructure) stage by stage:
features, yakmo seeding means, KNNScanReduce (pass count, clusters,
centroids), and the whole-frame .gsc.
"""
from __future__ import annotations

import hashlib
import json
import struct
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "tests")]

CFG = {  # bench.py CONFIGS: argv, channels, rate
    "c2": (["-cs8", "-cpf4096", "-cbd8"], 2, 44100),
    "c3": (["-cs16", "-cpf4096", "-cbd12"], 2, 44100),
    "br128": (["-br128", "-vfr0.5", "-cs8"], 2, 44100),
    "c5": (["-cs8", "-cpf4096"], 2, 48000),
    "c5cs4": (["-cs4", "-cpf4096"], 2, 48000),
}


def diff(prefix: str, key: str) -> list[int]:
    blob = Path(prefix + ".r0.gsc").read_bytes()
    meta = json.loads(Path(prefix + ".r0.json").read_text())
    want = json.loads((ROOT / "tests/golden/bench_digests.json").read_text())[key]["per_frame"]
    bad, o = [], 0
    for i, n in enumerate(meta["sizes"]):
        f = meta["first"] + i
        h = want.get(str(f))
        if h is not None and hashlib.sha256(blob[o:o + n]).hexdigest() != h:
            bad.append(f)
        o += n
    return bad


def frame_wav(config: str, seconds: float, frame: int):
    """(single-frame WAV, argv) of frame `frame` of the bench workload."""
    import oracle_ffi
    from soundchunks_amd.synth import synth_wav, wav_header

    argv, ch, rate = CFG[config]
    wav = synth_wav(seconds, rate, ch)
    st, en = oracle_ffi.frame_bounds(wav, argv)
    a, b = int(st[frame]), int(en[frame]) + 1
    n = (len(wav) - 44) // (2 * ch)
    b = min(b, n)
    body = wav[44 + a * ch * 2: 44 + b * ch * 2]
    one = wav_header(ch, rate, b - a) + body
    for fl in (6000, 8000, 12000, 20000):
        av = argv + [f"-fl{fl}"]
        if len(oracle_ffi.frame_bounds(one, av)[0]) == 1:
            return one, av
    raise RuntimeError("could not keep the frame whole")


def probe(frames, config="c2", seconds=1024.0):
    import oracle_ffi
    import soundchunks_amd as sc

    for f in frames:
        wav, av = frame_wav(config, seconds, f)
        print(f"frame {f}: {(len(wav) - 44) // 4} samples, argv {av}", flush=True)
        g = sc.Encoder(av).encode(wav)
        o = oracle_ffi.encode(wav, av, threads=4)
        print(f"  whole frame .gsc: {'EQUAL' if g == o else 'DIFFERENT'} ({len(g)} vs {len(o)} bytes)", flush=True)
        tr = oracle_ffi.trace_frame(wav, av, 0)
        att, feat = sc.frame_dsp(wav, 0, av)
        print(f"  features equal: {att == tr['atten_div'] and np.array_equal(feat.view(np.uint32), tr['dataset'].view(np.uint32))}")
        y = sc.yakmo_seed_means(tr["dataset"], tr["K"])
        yeq = np.array_equal(y.view(np.uint32), tr["yakmo"].view(np.uint32))
        print(f"  yakmo equal: {yeq}")
        c, cl, it = sc.scan_reduce(tr["dataset"], tr["yakmo"], 3)
        print(f"  scan: passes {it} vs oracle {tr['scan_iters']}; clusters differ at "
              f"{int((cl != tr['clusters']).sum())} points; centroids differ in "
              f"{int((c.view(np.uint32) != tr['scan'].view(np.uint32)).any(axis=1).sum())} rows", flush=True)
        if it != tr["scan_iters"] or (cl != tr["clusters"]).any():
            # first pass where the chains part: re-run both with a pass limit
            lo, hi = 1, max(it, tr["scan_iters"])
            while lo < hi:
                mid = (lo + hi) // 2
                import os

                os.environ["GSC_SCAN_MAX_PASSES"] = str(mid)
                c1, cl1, _ = sc.scan_reduce(tr["dataset"], tr["yakmo"], 3)
                oc1, ocl1, _ = oracle_ffi.scan_reduce(tr["dataset"], tr["yakmo"], 3, mid)
                same = np.array_equal(c1.view(np.uint32), oc1.view(np.uint32)) and np.array_equal(cl1, ocl1)
                if same:
                    lo = mid + 1
                else:
                    hi = mid
                del os.environ["GSC_SCAN_MAX_PASSES"]
            print(f"  first differing pass: {lo}", flush=True)
            import os

            os.environ["GSC_SCAN_MAX_PASSES"] = str(lo)
            c1, cl1, _ = sc.scan_reduce(tr["dataset"], tr["yakmo"], 3)
            oc1, ocl1, _ = oracle_ffi.scan_reduce(tr["dataset"], tr["yakmo"], 3, lo)
            del os.environ["GSC_SCAN_MAX_PASSES"]
            idx = np.nonzero(cl1 != ocl1)[0]
            print(f"  pass {lo}: {len(idx)} points differ, first {idx[:8].tolist()}; "
                  f"gpu {cl1[idx[:8]].tolist()} oracle {ocl1[idx[:8]].tolist()}", flush=True)
            np.savez(ROOT / "gpurun_out" / f"probe_{config}_{f}.npz", dataset=tr["dataset"], yakmo=tr["yakmo"],
                     pass_=lo, gpu_cl=cl1, ora_cl=ocl1, gpu_c=c1, ora_c=oc1)


if __name__ == "__main__":
    if sys.argv[1] == "diff":
        key = f"{sys.argv[3]}:{float(sys.argv[4]):g}" if len(sys.argv) > 4 else "c2:1024"
        print(diff(sys.argv[2], key))
    else:
        args = sys.argv[2:]
        cfg, secs = "c2", 1024.0
        if "--config" in args:
            cfg = args[args.index("--config") + 1]
        if "--seconds" in args:
            secs = float(args[args.index("--seconds") + 1])
        fr = [int(a) for a in args if a.isdigit()]
        probe(fr, cfg, secs)
