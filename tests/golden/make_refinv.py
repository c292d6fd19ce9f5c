"""Oracle goldens for the reference's own invocations and test files.

    python tests/golden/make_refinv.py [--threads 4] [name ...]   (build container)

The command lines come from the reference's Lazarus session history
(encoder/encoder.lps:260-279, the CommandLineParameters list) and its test
inputs: opus_test/mo_b_44_2.wav (48 kHz stereo real audio), opus_test/
mo_10_44.wav (44.1 kHz mono), lame_test/mstest.wav, and one file per odd
sample rate of my_test/ (tone26.wav 26,390 Hz, testxn32.wav 32 kHz,
testn.wav 48 kHz).  The WAVs are input data, copied once into
tests/golden/ref_inputs/ (the GPU box has no /root/reference).

The oracle (oracle/, the C restatement of encoder.lpr) encodes each case; the
.gsc SHA-256 and size (or the SaveStream assertion failure, encoder.lpr:986,
that -pr0 passthrough frames of real audio hit) go to
tests/golden/refinv_meta.json.  "-v" (verbose output) is dropped: it changes
nothing in the .gsc.
"""
from __future__ import annotations

import argparse
import hashlib
import json
import shutil
import sys
import time
from pathlib import Path

HERE = Path(__file__).resolve().parent
sys.path[:0] = [str(HERE.parents[1]), str(HERE.parent)]

import oracle_ffi  # noqa: E402

REF = Path("/root/reference")
INPUTS = HERE / "ref_inputs"
OUT = HERE / "refinv_meta.json"
FILES = {
    "mo_b_44_2.wav": REF / "opus_test" / "mo_b_44_2.wav",
    "mo_10_44.wav": REF / "opus_test" / "mo_10_44.wav",
    "tone26.wav": REF / "my_test" / "tone26.wav",
    "testxn32.wav": REF / "my_test" / "testxn32.wav",
    "testn.wav": REF / "my_test" / "testn.wav",
    # the rest of the reference's opus_test/ and my_test/ inputs (round 5)
    "mo_10_32.wav": REF / "opus_test" / "mo_10_32.wav",
    "mo_62_32.wav": REF / "opus_test" / "mo_62_32.wav",
    "mo_10_44_new.wav": REF / "opus_test" / "mo_10_44_new.wav",
    "mo_10_48_new.wav": REF / "opus_test" / "mo_10_48_new.wav",
    "test2.wav": REF / "my_test" / "test2.wav",
    "testenv.wav": REF / "my_test" / "testenv.wav",
    "testn26.wav": REF / "my_test" / "testn26.wav",
    "testxn.wav": REF / "my_test" / "testxn.wav",
    "testn44.wav": REF / "my_test" / "testn44.wav",
}
# name -> (input, argv); encoder.lps:260-279 item numbers in the comments
CASES = {
    "mo_b_44_2_default": ("mo_b_44_2.wav", []),                   # item 3
    "mo_b_44_2_fl1000": ("mo_b_44_2.wav", ["-fl1000"]),            # item 6
    "mo_b_44_2_pr0": ("mo_b_44_2.wav", ["-pr0"]),                  # item 9
    "mo_b_44_2_cs16": ("mo_b_44_2.wav", ["-cs16"]),                # item 10
    "mo_b_44_2_br150": ("mo_b_44_2.wav", ["-br150"]),              # item 11
    "mo_b_44_2_br128": ("mo_b_44_2.wav", ["-br128"]),              # item 12
    "mo_b_44_2_br999": ("mo_b_44_2.wav", ["-br999"]),              # item 13
    "mo_10_44_default": ("mo_10_44.wav", []),                      # item 14
    "mo_10_44_pr0": ("mo_10_44.wav", ["-pr0"]),                    # item 15
    "mo_10_44_br64_vfr05_cs16_pr0": ("mo_10_44.wav", ["-br64", "-vfr0.5", "-cs16", "-pr0"]),  # item 20
    "tone26_default": ("tone26.wav", []),
    "testxn32_default": ("testxn32.wav", []),
    "testn_default": ("testn.wav", []),
    "mo_10_32_default": ("mo_10_32.wav", []),
    "mo_62_32_default": ("mo_62_32.wav", []),
    "mo_10_44_new_default": ("mo_10_44_new.wav", []),
    "mo_10_48_new_default": ("mo_10_48_new.wav", []),
    "test2_default": ("test2.wav", []),
    "testenv_default": ("testenv.wav", []),
    "testn26_default": ("testn26.wav", []),
    "testxn_default": ("testxn.wav", []),
    "testn44_default": ("testn44.wav", []),
}


def wav_path(name: str) -> Path:
    return INPUTS / name


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", type=int, default=4)
    ap.add_argument("names", nargs="*")
    a = ap.parse_args()
    INPUTS.mkdir(exist_ok=True)
    for n, src in FILES.items():
        if not wav_path(n).exists():
            shutil.copyfile(src, wav_path(n))
    for name in a.names or CASES:
        inp, argv = CASES[name]
        wav = wav_path(inp).read_bytes()
        t = time.time()
        ent = {"input": inp, "argv": argv, "wav_sha256": hashlib.sha256(wav).hexdigest()}
        st, _ = oracle_ffi.frame_bounds(wav, argv)
        ent["frames"] = len(st)
        try:
            gsc = oracle_ffi.encode(wav, argv, threads=a.threads)
            ent.update(gsc_sha256=hashlib.sha256(gsc).hexdigest(), gsc_bytes=len(gsc), error=None)
        except RuntimeError as e:
            if "-4" not in str(e):
                raise
            ent.update(gsc_sha256=None, gsc_bytes=None, error="SaveStream assertion (encoder.lpr:986)")
        ent["oracle_seconds"] = round(time.time() - t, 1)
        db = json.loads(OUT.read_text()) if OUT.exists() else {}
        db[name] = ent
        OUT.write_text(json.dumps(db, indent=1, sort_keys=True) + "\n")
        print(name, ent, flush=True)


if __name__ == "__main__":
    main()
