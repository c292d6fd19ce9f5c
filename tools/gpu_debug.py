"""Quick stage-level GPU vs oracle diff for one golden case (debug helper)."""
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))

import oracle_ffi  # noqa: E402
import soundchunks_amd as sc  # noqa: E402
from golden.cases import CASES, golden_path  # noqa: E402


def bits(a):
    return np.ascontiguousarray(a).view(np.uint32)


def main(name):
    make, argv = CASES[name]
    wav = make()
    tr = oracle_ffi.trace_frame(wav, argv, 0)
    print(name, "N", tr["N"], "K", tr["K"], "D", tr["D"], "iters", tr["scan_iters"], flush=True)
    if tr["N"] > tr["K"]:
        t = time.time()
        c = sc.yakmo_seed_means(tr["dataset"], tr["K"])
        print(" yakmo", time.time() - t, "mismatch", int((bits(c) != bits(tr["yakmo"])).sum()), flush=True)
        t = time.time()
        c2, cl, it = sc.scan_reduce(tr["dataset"], tr["yakmo"], 3)
        print(" scan", time.time() - t, "passes", it, "cl mismatch", int((cl != tr["clusters"]).sum()),
              "c mismatch", int((bits(c2) != bits(tr["scan"])).sum()), flush=True)
    fwd = tr["knn_cand"][0::4]
    t = time.time()
    b = sc.knnfit_assign(fwd, tr["knn_query"], tr["knn_eps"])
    print(" knnfit", time.time() - t, "mismatch", int((b != tr["knn_best"]).sum()), flush=True)
    t = time.time()
    g = sc.Encoder(argv).encode(wav)
    exp = golden_path(name).read_bytes()
    print(" encode", time.time() - t, len(g), len(exp), "equal", g == exp, sc.Encoder.last_timing(), flush=True)


if __name__ == "__main__":
    for n in sys.argv[1:] or ["c1_test_cs8_cpf256"]:
        main(n)
