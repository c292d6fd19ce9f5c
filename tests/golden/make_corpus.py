"""C4 corpus fixtures: the reference's lame_test/*.wav inputs (data files the
reference's test corpus holds, copied verbatim into tests/golden/lame_test/)
and the oracle's .gsc digests at the C4 flags.

    python tests/golden/make_corpus.py        (build container: reads /root/reference)

Expected outputs are stored as sha256 + byte count (corpus_meta.json); the
GPU test encodes every file through the HIP path and compares digests.
"""
from __future__ import annotations

import hashlib
import json
import shutil
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))

import oracle_ffi  # noqa: E402

SRC = Path("/root/reference/lame_test")
DST = Path(__file__).resolve().parent / "lame_test"
ARGV = ["-cs8", "-cpf4096"]


def main():
    DST.mkdir(exist_ok=True)
    meta = {"argv": ARGV, "files": {}}
    for src in sorted(SRC.glob("*.wav")):
        dst = DST / src.name
        if not dst.exists():
            shutil.copyfile(src, dst)
        wav = dst.read_bytes()
        t = time.time()
        gsc = oracle_ffi.encode(wav, ARGV, threads=8)
        st = oracle_ffi.stats()
        meta["files"][src.name] = {"wav_sha256": hashlib.sha256(wav).hexdigest(),
                                   "gsc_sha256": hashlib.sha256(gsc).hexdigest(), "gsc_bytes": len(gsc),
                                   "frames": st["frame_count"], "scan_iterations": st["scan_iterations"],
                                   "oracle_seconds": round(time.time() - t, 2)}
        print(src.name, meta["files"][src.name], flush=True)
    (Path(__file__).resolve().parent / "corpus_meta.json").write_text(json.dumps(meta, indent=1, sort_keys=True) + "\n")


if __name__ == "__main__":
    main()
