"""GPU debug: batched KNNScanReduce vs the oracle on a frame with NaN centroids,
pass by pass (GSC_SCAN_MAX_PASSES), first differing query and its ANN context.
    python tools/nan_debug.py [case] [frame] [passes]"""
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT)); sys.path.insert(0, str(ROOT / "tests"))
import numpy as np  # noqa: E402

import oracle_ffi  # noqa: E402  (checker)
import soundchunks_amd as sc  # noqa: E402
from golden.cases import CASES  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "quiet_tone_cs4_cpf1024"
frame = int(sys.argv[2]) if len(sys.argv) > 2 else 0
npass = int(sys.argv[3]) if len(sys.argv) > 3 else 3
mk, argv = CASES[name]
wav = mk()
t = oracle_ffi.trace_frame(wav, argv, frame)
X = np.ascontiguousarray(t["dataset"], np.float32)
Y = np.ascontiguousarray(t["yakmo"], np.float32)
print(name, frame, "N", X.shape[0], "K", Y.shape[0], "nan rows", int(np.isnan(Y).any(1).sum()), flush=True)
for p in range(1, npass + 1):
    os.environ["GSC_SCAN_MAX_PASSES"] = str(p)
    cg, clg, itg = sc.scan_reduce(X, Y, 3)
    co, clo, ito = oracle_ffi.scan_reduce(X, Y, 3, max_passes=p)
    dif = np.nonzero(clg != clo)[0]
    cm = ~(np.isnan(cg) & np.isnan(co)) & (cg.view(np.uint32) != co.view(np.uint32))
    print(f"passes {p}: gpu iters {itg} oracle iters {ito}; cluster diffs {len(dif)} first {dif[:5].tolist()}; "
          f"centroid rows differing {int(cm.any(1).sum())}", flush=True)
    if len(dif):
        i = int(dif[0])
        print(f"  query {i}: gpu -> {clg[i]} (nan row {bool(np.isnan(co[clg[i]]).any())}), oracle -> {clo[i]} "
              f"(nan row {bool(np.isnan(co[clo[i]]).any())})", flush=True)
        break
