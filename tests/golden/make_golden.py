"""Regenerate the committed golden .gsc fixtures with the C oracle.

    python tests/golden/make_golden.py [case ...]

The oracle is the CPU restatement of the reference encoder (oracle/); its
pinning status is documented in DESIGN.md.  Fixtures are data only.
"""
from __future__ import annotations

import hashlib
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))

import oracle_ffi  # noqa: E402
from golden.cases import CASES, golden_path  # noqa: E402


def main(names):
    meta_path = Path(__file__).with_name("golden_meta.json")
    meta = json.loads(meta_path.read_text()) if meta_path.exists() else {}
    for name in names or CASES:
        make, argv = CASES[name]
        wav = make()
        t = time.time()
        gsc = oracle_ffi.encode(wav, argv, threads=8)
        st = oracle_ffi.stats()
        golden_path(name).write_bytes(gsc)
        meta[name] = {"argv": argv, "wav_sha256": hashlib.sha256(wav).hexdigest(),
                      "gsc_sha256": hashlib.sha256(gsc).hexdigest(), "gsc_bytes": len(gsc),
                      "oracle_seconds": round(time.time() - t, 2), "frames": st["frame_count"],
                      "scan_iterations": st["scan_iterations"]}
        print(name, meta[name], flush=True)
    meta_path.write_text(json.dumps(meta, indent=1, sort_keys=True) + "\n")


if __name__ == "__main__":
    main(sys.argv[1:])
