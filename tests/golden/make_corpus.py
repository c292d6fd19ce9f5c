"""C4 corpus fixtures: the reference's lame_test/*.wav inputs (data files the
reference's test corpus holds, copied verbatim into tests/golden/lame_test/)
and the oracle's .gsc digests at two flag sets:

- corpus_meta.json: `-cs8 -cpf4096` (the C4 bench shape, ChunkSize 8 like C2);
- corpus_default_meta.json: no flags, i.e. the encoder defaults `-cs4
  -cpf4096` (encoder.lpr:1486-1509), which is what SURVEY.md §8d specifies for
  C4 ("all other flags default") and the reference's own first invocation
  `mstest.wav -v` (encoder/encoder.lps:260; -v changes nothing in the .gsc).

    python tests/golden/make_corpus.py [--set cs8|default] [--threads 8]
    (build container: reads /root/reference)

Expected outputs are stored as sha256 + byte count; the GPU tests encode every
file through the HIP path and compare digests.
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
SETS = {"cs8": (["-cs8", "-cpf4096"], "corpus_meta.json"), "default": ([], "corpus_default_meta.json")}


def main():
    import argparse

    ap = argparse.ArgumentParser()
    ap.add_argument("--set", choices=sorted(SETS), default="cs8")
    ap.add_argument("--threads", type=int, default=8)
    a = ap.parse_args()
    argv, out = SETS[a.set]
    DST.mkdir(exist_ok=True)
    meta = {"argv": argv, "files": {}}
    for src in sorted(SRC.glob("*.wav")):
        dst = DST / src.name
        if not dst.exists():
            shutil.copyfile(src, dst)
        wav = dst.read_bytes()
        t = time.time()
        gsc = oracle_ffi.encode(wav, argv, threads=a.threads)
        st = oracle_ffi.stats()
        meta["files"][src.name] = {"wav_sha256": hashlib.sha256(wav).hexdigest(),
                                   "gsc_sha256": hashlib.sha256(gsc).hexdigest(), "gsc_bytes": len(gsc),
                                   "frames": st["frame_count"], "scan_iterations": st["scan_iterations"],
                                   "oracle_seconds": round(time.time() - t, 2)}
        print(src.name, meta["files"][src.name], flush=True)
        # saved after every file (a long run can be watched and resumed by hand)
        (Path(__file__).resolve().parent / out).write_text(json.dumps(meta, indent=1, sort_keys=True) + "\n")


if __name__ == "__main__":
    main()
