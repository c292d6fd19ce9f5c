"""Stage-by-stage HIP vs oracle diff of one frame of a golden case (GPU box):
    python tools/diag_stages.py CASE [FRAME]"""
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "tests")]

import numpy as np  # noqa: E402

import oracle_ffi  # noqa: E402
import soundchunks_amd as sc  # noqa: E402
from golden.cases import CASES  # noqa: E402


def diff(name, a, b):
    a = np.ascontiguousarray(a)
    b = np.ascontiguousarray(b)
    if a.dtype == np.float32:
        a, b = a.view(np.uint32), b.view(np.uint32)
    bad = np.flatnonzero((a != b).reshape(a.shape[0], -1).any(axis=1)) if a.ndim > 1 else np.flatnonzero(a != b)
    print(f"  {name}: {len(bad)} rows differ of {a.shape[0]}" + (f", first {bad[:8].tolist()}" if len(bad) else ""),
          flush=True)
    return len(bad)


def main():
    case = sys.argv[1]
    frame = int(sys.argv[2]) if len(sys.argv) > 2 else 0
    make, argv = CASES[case]
    wav = make()
    tr = oracle_ffi.trace_frame(wav, argv, frame)
    print(case, argv, "frame", frame, "N", tr["N"], "K", tr["K"], "D", tr["D"], "iters", tr["scan_iters"], flush=True)
    att, feat = sc.frame_dsp(wav, frame, argv)
    print("  atten", att, tr["atten_div"])
    diff("features", feat, tr["dataset"])
    if tr["N"] > tr["K"]:
        t = time.time()
        y = sc.yakmo_seed_means(tr["dataset"], tr["K"])
        print(f"  yakmo {time.time() - t:.2f}s, NaN rows {int(np.isnan(tr['yakmo']).any(axis=1).sum())}")
        diff("yakmo", y, tr["yakmo"])
        t = time.time()
        c, cl, it = sc.scan_reduce(tr["dataset"], tr["yakmo"], 3)
        print(f"  scan {time.time() - t:.2f}s passes {it} vs {tr['scan_iters']}")
        diff("clusters", cl, tr["clusters"])
        diff("centroids", c, tr["scan"])
        for p in (1, 2, 3):
            import os
            os.environ["GSC_SCAN_MAX_PASSES"] = str(p)
            c, cl, it = sc.scan_reduce(tr["dataset"], tr["yakmo"], 3)
            oc, ocl, on = oracle_ffi.scan_reduce(tr["dataset"], tr["yakmo"], 3, p)
            del os.environ["GSC_SCAN_MAX_PASSES"]
            print(f"  after {p} passes:")
            if diff("clusters", cl, ocl) + diff("centroids", c, oc) == 0 and p == 3:
                break
    best = sc.knnfit_assign(tr["knn_cand"][0::4], tr["knn_query"], tr["knn_eps"])
    diff("knnfit", best, tr["knn_best"])


if __name__ == "__main__":
    main()
