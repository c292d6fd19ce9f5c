"""Stamps of the batched scan on tests/test_gpu_scan.py's integer-grid tie
dataset (how many queries took the in-batch DFS path):
    GSC_LIB=soundchunks_amd/lib/stamps/libsoundchunks_amd.so GSC_SCAN_DEBUG=1 \
        GSC_SCAN_MAX_PASSES=3 python tools/grid_ties_stamps.py D K"""
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import soundchunks_amd as sc  # noqa: E402

d, k = int(sys.argv[1]), int(sys.argv[2])
rng = np.random.default_rng(7 + d + k)
n = 24000
x = rng.integers(-6, 7, size=(n, d)).astype(np.float32)
x[::5] = x[1::5][: len(x[::5])]
c0 = x[rng.choice(n, k, replace=False)] + rng.integers(-1, 2, size=(k, d)).astype(np.float32) * 0.5
c, cl, it = sc.scan_reduce(x, c0, precision=3)
print(f"D={d} K={k} passes={it}", flush=True)
