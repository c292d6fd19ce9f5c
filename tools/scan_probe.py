"""Stage probe: batched KNNScanReduce on GPU vs the oracle for the first P
passes of an oracle-traced frame (debug helper, GPU box)."""
import os
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))

import oracle_ffi  # noqa: E402
import soundchunks_amd as sc  # noqa: E402
from golden.cases import CASES  # noqa: E402


def main(name, passes):
    make, argv = CASES[name]
    tr = oracle_ffi.trace_frame(make(), argv, 0)
    os.environ["GSC_SCAN_MAX_PASSES"] = str(passes)
    os.environ["GSC_SCAN_DEBUG"] = "1"
    t = time.time()
    oc, ocl, on = oracle_ffi.scan_reduce(tr["dataset"], tr["yakmo"], 3, passes)
    to = time.time() - t
    t = time.time()
    gc, gcl, gn = sc.scan_reduce(tr["dataset"], tr["yakmo"], 3)
    tg = time.time() - t
    bad = np.nonzero(gcl != ocl)[0]
    print(f"{name} N={tr['N']} K={tr['K']} D={tr['D']} passes o={on} g={gn} t_oracle={to:.2f}s t_gpu={tg:.2f}s "
          f"cluster mismatches={len(bad)} first={bad[:5]} centroid bit mismatches="
          f"{int((gc.view(np.uint32) != oc.view(np.uint32)).sum())}", flush=True)


if __name__ == "__main__":
    p = int(sys.argv[1])
    for n in sys.argv[2:]:
        main(n, p)
