"""a9 fixtures: Birch labels from the reference's own encoder/cluster.py.

    python tests/golden/make_birch.py      (build container: runs /root/reference/encoder/cluster.py)

For each case, the frame's Reduce dataset (a1 staging, from the oracle trace)
is written the way DoExternalSKLearn does (extern.pas:363-369: "i v0 v1 ... "
per row; FloatToStr(Single) prints 10 significant digits -- encoder.exe's
str_real digit table, see soundchunks_amd/csrc/gsc_birch_host.cpp), cluster.py is run on
it exactly as extern.pas:389-393 invokes it (-i FILE -n K -t 10^(1-Precision)),
and the .membership labels are stored with the dataset (float32) in
tests/golden/birch_<case>.npz.  The GPU test feeds the same dataset to the
product's -py reducer and compares labels.
"""
from __future__ import annotations

import subprocess
import sys
import tempfile
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
sys.path[:0] = [str(HERE.parents[1]), str(HERE.parent)]

import oracle_ffi  # noqa: E402
from golden.cases import CASES  # noqa: E402

CLUSTER_PY = Path("/root/reference/encoder/cluster.py")

BIRCH_CASES = {
    # name: (wav factory, argv, frame)
    "mstest_fl500_f0": (lambda: (HERE / "lame_test" / "mstest.wav").read_bytes(), ["-fl500", "-cpf256"], 0),
    "mstest_fl500_f2": (lambda: (HERE / "lame_test" / "mstest.wav").read_bytes(), ["-fl500", "-cpf256"], 2),
    "hihat_cs8_cpf256_f0": (CASES["hihat_cs8_cpf256"][0], ["-cs8", "-cpf256"], 0),
    "silence_tone_cs8_cpf256_f0": (CASES["silence_tone_cs8_cpf256"][0], ["-cs8", "-cpf256"], 0),
    "c1_test_cs8_cpf256_f1": (CASES["c1_test_cs8_cpf256"][0], ["-cs8", "-cpf256"], 1),
}


def fpc_single_text(v: float) -> str:
    """FloatToStr(Single): 10 significant digits (the value numpy.loadtxt reads back)."""
    return "%.9E" % float(v)


def dataset_text(x: np.ndarray) -> str:
    return "".join(str(i) + " " + "".join(fpc_single_text(v) + " " for v in row) + "\n" for i, row in enumerate(x))


def main(names):
    for name in names or BIRCH_CASES:
        make, argv, frame = BIRCH_CASES[name]
        tr = oracle_ffi.trace_frame(make(), argv, frame)
        x, k = tr["dataset"], tr["K"]
        assert tr["N"] > k, "the -py reducer only runs on frames with more chunks than ChunksPerFrame"
        with tempfile.TemporaryDirectory() as td:
            fn = Path(td) / "dataset.txt"
            fn.write_text(dataset_text(x))
            r = subprocess.run([sys.executable, str(CLUSTER_PY), "-i", str(fn), "-n", str(k), "-t", "0.01"],
                               capture_output=True, text=True, cwd=td)
            assert r.returncode == 0, r.stderr
            labels = np.loadtxt(str(fn) + ".membership", dtype=np.int32)
        np.savez_compressed(HERE / f"birch_{name}.npz", dataset=x, k=np.int32(k), labels=labels,
                            argv=np.array(argv), frame=np.int32(frame))
        print(name, x.shape, "K", k, "distinct labels", len(np.unique(labels)), flush=True)


if __name__ == "__main__" and sys.argv[1:2] != ["--files"]:
    main(sys.argv[1:])


# whole-file -py golden: the reference's own -py invocation on a corpus file
# ("-fl500 -cpf256 -py"); cluster.py labels for every reduced
# frame, then the oracle encodes with them (oracle_ffi.set_py_labels)
PY_FILES = {
    "mstest_fl500_cpf256_py": ("lame_test/mstest.wav", ["-fl500", "-cpf256", "-py"]),
    # encoder/encoder.lps:261 `mstest.wav -v -py`: the defaults (-cs4 -cpf4096),
    # Birch at K = 4096 on N ~ 43,750 rows per frame
    "mstest_default_py": ("lame_test/mstest.wav", ["-py"]),
    # full-length frames: 4.5 s mono at ChunkSize 4 -> N ~ 44100 chunks per frame
    "tone_lsb45_cs4_cpf256_py": ("tone_lsb45", ["-cs4", "-cpf256", "-py"]),
}


def py_file_wav(rel: str) -> bytes:
    if rel == "tone_lsb45":
        from golden.cases import _tone_lsb

        return _tone_lsb(seconds=4.5)
    return (HERE / rel).read_bytes()


def make_py_file(name):
    import hashlib
    import json

    rel, argv = PY_FILES[name]
    wav = py_file_wav(rel)
    base = [a for a in argv if a != "-py"]
    _, nfr = oracle_ffi.encode_frames(wav, base, 0, 1)
    labels, offsets = [], []
    off = 0
    for f in range(nfr):
        tr = oracle_ffi.trace_frame(wav, base, f)
        offsets.append(off)
        if tr["N"] > tr["K"]:
            with tempfile.TemporaryDirectory() as td:
                fn = Path(td) / "dataset.txt"
                fn.write_text(dataset_text(tr["dataset"]))
                r = subprocess.run([sys.executable, str(CLUSTER_PY), "-i", str(fn), "-n", str(tr["K"]), "-t", "0.01"],
                                   capture_output=True, text=True, cwd=td)
                assert r.returncode == 0, r.stderr
                lab = np.loadtxt(str(fn) + ".membership", dtype=np.int32)
        else:
            lab = np.zeros(tr["N"], np.int32)
        labels.append(lab)
        off += len(lab)
    labels = np.concatenate(labels)
    oracle_ffi.set_py_labels(labels, offsets)
    gsc = oracle_ffi.encode(wav, argv, threads=8)
    oracle_ffi.set_py_labels(None)
    (HERE / f"{name}.gsc").write_bytes(gsc)
    np.savez_compressed(HERE / f"birch_file_{name}.npz", labels=labels, offsets=np.array(offsets, np.int64))
    meta_path = HERE / "golden_meta.json"
    meta = json.loads(meta_path.read_text())
    meta[name] = {"argv": argv, "wav_sha256": hashlib.sha256(wav).hexdigest(),
                  "gsc_sha256": hashlib.sha256(gsc).hexdigest(), "gsc_bytes": len(gsc), "frames": nfr,
                  "labels": "cluster.py (reference encoder/cluster.py, sklearn 1.7.2) via tests/golden/make_birch.py"}
    meta_path.write_text(json.dumps(meta, indent=1, sort_keys=True) + "\n")
    print(name, "frames", nfr, "gsc bytes", len(gsc), flush=True)


if __name__ == "__main__" and len(sys.argv) > 1 and sys.argv[1] == "--files":
    for n in sys.argv[2:] or PY_FILES:
        make_py_file(n)
