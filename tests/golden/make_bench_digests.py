"""Oracle SHA-256 digests of the bench workloads' .gsc frames (bench.py's
`bit_exact` check).  Build container only: the oracle (oracle/, a C
restatement of the reference encoder, encoder.lpr:1433-1447 DoFrame and
:980-1107 SaveStream) encodes each listed frame of the exact synthetic file
bench.py encodes (soundchunks_amd.synth), and the per-frame
digests go to tests/golden/bench_digests.json, keyed "<config>:<seconds>".
A .gsc is the concatenation of its frames' SaveStream bytes
(encoder.lpr:1181-1215), so when every frame is listed the whole-file digest
is pinned too (total_bytes + every frame's digest).

    python tests/golden/make_bench_digests.py [--threads 6] [key ...]

Keys (default: all, in this order): c2 at 1024 s (every frame); the
weak-scaling c2 files of 2 / 4 / 8 ranks (1024 s per rank: every frame of the
2-rank file, the first and last frame of every rank's range of the others);
C5 at 3600 s, -cs8 and -cs4 (every frame: the whole 1-hour file); c2 at 600 s
(every frame) and 3600 s (every frame);
br128 and c3 at 1024 s (every frame); c2 at 16 s and 32 s (every frame: the
GPU tests run bench.py on them).  Resumable: finished frames are kept.
"""
from __future__ import annotations

import argparse
import hashlib
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))

import oracle_ffi  # noqa: E402
from soundchunks_amd.shard import bounds_range  # noqa: E402
from soundchunks_amd.synth import synth_wav  # noqa: E402

OUT = Path(__file__).resolve().parent / "bench_digests.json"
# bench.py CONFIGS (argv, channels, rate, chunk size)
CFG = {
    "c2": (["-cs8", "-cpf4096", "-cbd8"], 2, 44100, 8),
    "c3": (["-cs16", "-cpf4096", "-cbd12"], 2, 44100, 16),
    "br128": (["-br128", "-vfr0.5", "-cs8"], 2, 44100, 8),
    "c5": (["-cs8", "-cpf4096"], 2, 48000, 8),
    "c5cs4": (["-cs4", "-cpf4096"], 2, 48000, 4),
}
# key -> (config, seconds, frame selection): "all", ("range", b, e) or ("ranks", world_size)
WORKLOADS = {
    "c2:1024": ("c2", 1024.0, "all"),
    "c2:2048": ("c2", 2048.0, "all"),
    "c2:4096": ("c2", 4096.0, ("ranks", 4)),
    "c2:8192": ("c2", 8192.0, ("ranks", 8)),
    "c5:3600": ("c5", 3600.0, "all"),
    "c5cs4:3600": ("c5cs4", 3600.0, "all"),
    # SURVEY.md §8d's C2 throughput lengths (600 s = 150 frames, 3600 s = 900)
    "c2:600": ("c2", 600.0, "all"),
    "c2:3600": ("c2", 3600.0, "all"),
    "br128:1024": ("br128", 1024.0, "all"),
    "c3:1024": ("c3", 1024.0, "all"),
    # short files for the tests (bench.py --seconds 16, and 2 ranks x 16 s weak)
    "c2:16": ("c2", 16.0, "all"),
    "c2:32": ("c2", 32.0, "all"),
}
BATCH = 12  # frames per oracle call (progress is saved after each)


def load() -> dict:
    return json.loads(OUT.read_text()) if OUT.exists() else {}


def save(db: dict) -> None:
    OUT.write_text(json.dumps(db, indent=1, sort_keys=True) + "\n")


def run(key: str, threads: int) -> None:
    cfg, seconds, sel = WORKLOADS[key]
    argv, ch, rate, cs = CFG[cfg]
    wav = synth_wav(seconds, rate, ch)
    st, en = oracle_ffi.frame_bounds(wav, argv)
    nfr = len(st)
    if sel == "all":
        frames = list(range(nfr))
    elif sel[0] == "range":
        frames = list(range(sel[1], min(sel[2], nfr)))
    else:  # the first and last frame of every rank's range (bench.py's bounds_range)
        frames = sorted({f for r in range(sel[1]) for f in (bounds_range(st, en, cs, ch, r, sel[1])[0],
                                                             bounds_range(st, en, cs, ch, r, sel[1])[1] - 1)})
    fresh = {"config": cfg, "argv": argv, "seconds": seconds, "rate": rate, "channels": ch, "frames": nfr,
             "per_frame": {}}
    db = load()
    ent = db.setdefault(key, fresh)
    ent["frames"] = nfr
    save(db)
    todo = [f for f in frames if str(f) not in ent["per_frame"]]
    print(f"{key}: {nfr} frames, {len(frames)} listed, {len(todo)} to encode", flush=True)
    for i in range(0, len(todo), BATCH):
        part = todo[i:i + BATCH]
        t = time.time()
        blobs, fc = oracle_ffi.encode_frame_list(wav, argv, part, threads=threads)
        assert fc == nfr
        db = load()  # re-read: another key's run may have saved meanwhile
        ent = db.setdefault(key, fresh)
        for f, b in zip(part, blobs):
            ent["per_frame"][str(f)] = hashlib.sha256(b).hexdigest()
            ent.setdefault("frame_bytes", {})[str(f)] = len(b)
        save(db)
        print(f"  frames {part[0]}..{part[-1]} in {time.time() - t:.0f} s", flush=True)
    if sel == "all":
        # every frame listed: the whole file is the frames' bytes in order, so
        # len(file) == total_bytes and every frame digest equal <=> the file is equal
        db = load()
        db[key]["total_bytes"] = sum(db[key]["frame_bytes"].values())
        save(db)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", type=int, default=6)
    ap.add_argument("keys", nargs="*")
    a = ap.parse_args()
    for k in a.keys or list(WORKLOADS):
        run(k, a.threads)


if __name__ == "__main__":
    main()
