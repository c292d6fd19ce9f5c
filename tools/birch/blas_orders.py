"""Derivation check of the BLAS summation orders pinned in
soundchunks_amd/csrc/gsc_npblas.h (the -py reducer).

    python tools/birch/blas_orders.py [--trials 2000]

sklearn's Birch (cluster.py:21) reaches numpy / scipy BLAS through np.dot,
np.einsum, X @ X.T and scipy's dgemm / ddot.  Which summation order each call
uses depends on the BLAS build and on the CPU core its DYNAMIC_ARCH dispatch
selects, so this script

1. records the pin: numpy / scipy / OpenBLAS versions and the OpenBLAS core
   (threadpoolctl), the environment the cluster.py label fixtures were made in
   (tests/golden/make_birch.py);
2. checks every restated order of gsc_npblas.h element for element against
   the live library on random rows at the feature widths 8 / 16 / 32 (random
   scales, `--trials` draws);
3. shows that the check discriminates: plain sequential sums (unfused and
   fused) disagree with the library on a large share of the same draws, so
   agreement is not an accident of benign inputs.

On a host whose OpenBLAS selects another core (Zen, Haswell) step 2 fails
where the orders differ -- the labels of cluster.py on such a host are not
what the committed fixtures hold (-py).
"""
from __future__ import annotations

import argparse
import ctypes
import subprocess
import sys
import tempfile
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
HDR = ROOT / "soundchunks_amd" / "csrc" / "gsc_npblas.h"

SHIM = """#include "%s"
#include <cmath>
using namespace gsc::npblas;
extern "C" double f_ddot(const double* a, const double* b, int n) { return np_ddot(a, b, n); }
extern "C" double f_gemv(const double* r, const double* v, int n, int m, int i) { return np_gemv_row(r, v, n, m, i); }
extern "C" double f_ein(const double* a, int n) { return np_einsum_sq(a, n); }
extern "C" double f_syrk(const double* c, int n, int i, int j) { return np_syrk51(c, n, i, j); }
extern "C" double f_seq(const double* a, const double* b, int n) { double s = 0; for (int i = 0; i < n; ++i) s = s + a[i] * b[i]; return s; }
extern "C" double f_seqfma(const double* a, const double* b, int n) { double s = 0; for (int i = 0; i < n; ++i) s = std::fma(a[i], b[i], s); return s; }
"""


def build():
    td = Path(tempfile.mkdtemp())
    (td / "npb.cpp").write_text(SHIM % HDR)
    so = td / "npb.so"
    subprocess.run(["g++", "-O2", "-ffp-contract=off", "-shared", "-fPIC", "-o", str(so), str(td / "npb.cpp")],
                   check=True)
    L = ctypes.CDLL(str(so))
    for f in (L.f_ddot, L.f_gemv, L.f_ein, L.f_syrk, L.f_seq, L.f_seqfma):
        f.restype = ctypes.c_double
    return L


def pin() -> dict:
    import scipy

    info = {"numpy": np.__version__, "scipy": scipy.__version__}
    try:
        from threadpoolctl import threadpool_info

        for lib in threadpool_info():
            if lib.get("internal_api") == "openblas":
                info.setdefault("openblas", []).append({k: lib.get(k) for k in ("version", "architecture",
                                                                                  "prefix", "filepath")})
    except ImportError:
        info["openblas"] = "threadpoolctl not importable"
    return info


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--trials", type=int, default=2000)
    a = ap.parse_args()
    print("pin:", pin())
    L = build()
    P = lambda x: np.ascontiguousarray(x).ctypes.data_as(ctypes.c_void_p)  # noqa: E731
    rng = np.random.default_rng(20250217)
    bad = {"ddot": 0, "gemv": 0, "einsum": 0, "syrk": 0}
    seq_diff = seqfma_diff = total = 0
    for t in range(a.trials):
        d = (8, 16, 32)[t % 3]
        C = rng.standard_normal((51, d)) * rng.uniform(1e-3, 3.0) + rng.uniform(-1, 1) * rng.uniform(0, 2)
        v = rng.standard_normal(d) * rng.uniform(1e-3, 3.0)
        dots = np.array([np.dot(C[i], v) for i in range(51)])
        for i in range(51):
            got = L.f_ddot(P(C[i]), P(v), d)
            bad["ddot"] += got != dots[i]
            seq_diff += L.f_seq(P(C[i]), P(v), d) != dots[i]
            seqfma_diff += L.f_seqfma(P(C[i]), P(v), d) != dots[i]
            total += 1
        m = int(rng.choice([1, 2, 3, 5, 6, 7, 50, 51]))
        g = np.dot(C[:m], v)
        bad["gemv"] += sum(L.f_gemv(P(C[i]), P(v), d, m, i) != g[i] for i in range(m))
        e = np.einsum("ij,ij->i", C, C)
        bad["einsum"] += sum(L.f_ein(P(C[i]), d) != e[i] for i in range(51))
        if t % 10 == 0:
            G = C @ C.T
            bad["syrk"] += sum(L.f_syrk(P(C), d, i, j) != G[i, j] for i in range(51) for j in range(51))
    print("restated orders that differ from the live library:", bad)
    print(f"discrimination: plain sequential dot differs on {seq_diff}/{total}, sequential fma on "
          f"{seqfma_diff}/{total} of the same ddot draws")
    ok = not any(bad.values())
    print("pinned orders hold on this host" if ok else "orders differ on this host: -py labels are not pinned here")
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
