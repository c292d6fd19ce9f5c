"""a9 (-py reducer) on the CPU: the product's Birch host code
(soundchunks_amd/csrc/gsc_birch_host.cpp, with its BLAS summation orders in
gsc_npblas.h) built with tools/birch/host_check.cpp, which restates the two
device steps (Ward linkage, predict) on the host.  Labels must equal the
reference's own encoder/cluster.py (sklearn 1.7.2) on every committed fixture
(tests/golden/make_birch.py), bit for bit."""
from __future__ import annotations

import ctypes
import subprocess
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parents[1]
GOLD = ROOT / "tests" / "golden"
DATASETS = ["mstest_fl500_f0", "mstest_fl500_f2", "hihat_cs8_cpf256_f0", "silence_tone_cs8_cpf256_f0",
            "c1_test_cs8_cpf256_f1"]


@pytest.fixture(scope="module")
def birch_host(tmp_path_factory):
    so = tmp_path_factory.mktemp("birch") / "birch_host.so"
    subprocess.run(["g++", "-O2", "-ffp-contract=off", "-shared", "-fPIC", "-o", str(so),
                    str(ROOT / "tools" / "birch" / "host_check.cpp"),
                    str(ROOT / "soundchunks_amd" / "csrc" / "gsc_birch_host.cpp")], check=True)
    lib = ctypes.CDLL(str(so))
    lib.birch_host_labels.restype = ctypes.c_int
    return lib


def _labels(lib, x, k):
    x = np.ascontiguousarray(x, dtype=np.float32)
    out = np.zeros(x.shape[0], np.int32)
    rc = lib.birch_host_labels(x.shape[0], x.shape[1], x.ctypes.data_as(ctypes.c_void_p), int(k),
                               out.ctypes.data_as(ctypes.c_void_p))
    assert rc == 0
    return out


@pytest.mark.parametrize("name", DATASETS)
def test_birch_host_labels_equal_cluster_py(birch_host, name):
    z = np.load(GOLD / f"birch_{name}.npz")
    got = _labels(birch_host, z["dataset"], z["k"])
    assert int((got != z["labels"]).sum()) == 0


def test_npblas_orders_match_numpy(tmp_path):
    """gsc_npblas.h against the numpy / scipy calls sklearn makes (the pin of
    the summation orders), on random rows at the three feature widths."""
    src = tmp_path / "npb.cpp"
    src.write_text('#include "%s"\n' % (ROOT / "soundchunks_amd" / "csrc" / "gsc_npblas.h") + """
using namespace gsc::npblas;
extern "C" double f_ddot(const double* a, const double* b, int n) { return np_ddot(a, b, n); }
extern "C" double f_gemv(const double* r, const double* v, int n, int m, int i) { return np_gemv_row(r, v, n, m, i); }
extern "C" double f_ein(const double* a, int n) { return np_einsum_sq(a, n); }
extern "C" double f_syrk(const double* c, int n, int i, int j) { return np_syrk51(c, n, i, j); }
""")
    so = tmp_path / "npb.so"
    subprocess.run(["g++", "-O2", "-ffp-contract=off", "-shared", "-fPIC", "-o", str(so), str(src)], check=True)
    L = ctypes.CDLL(str(so))
    for f in (L.f_ddot, L.f_gemv, L.f_ein, L.f_syrk):
        f.restype = ctypes.c_double
    P = lambda a: np.ascontiguousarray(a).ctypes.data_as(ctypes.c_void_p)  # noqa: E731
    rng = np.random.default_rng(2026)
    for d in (8, 16, 32):
        C = rng.standard_normal((51, d)) * rng.uniform(1e-3, 3.0)
        v = rng.standard_normal(d)
        assert all(L.f_ddot(P(C[i]), P(v), d) == np.dot(C[i], v) for i in range(51))
        for m in (1, 2, 3, 5, 6, 7, 50, 51):
            g = np.dot(C[:m], v)
            assert all(L.f_gemv(P(C[i]), P(v), d, m, i) == g[i] for i in range(m))
        e = np.einsum("ij,ij->i", C, C)
        assert all(L.f_ein(P(C[i]), d) == e[i] for i in range(51))
        G = C @ C.T
        assert all(L.f_syrk(P(C), d, i, j) == G[i, j] for i in range(51) for j in range(51))


@pytest.mark.parametrize("name", ["tone_lsb45_cs4_cpf256_py", "mstest_fl500_cpf256_py"])
def test_birch_host_whole_file_labels(birch_host, oracle, name):
    """Every reduced frame of the whole-file -py goldens (frames of N ~ 25k
    chunks in tone_lsb45): the host restatement's labels equal cluster.py's."""
    import sys

    sys.path.insert(0, str(GOLD.parent))
    from golden.make_birch import PY_FILES, py_file_wav

    rel, argv = PY_FILES[name]
    wav = py_file_wav(rel)
    base = [a for a in argv if a != "-py"]
    z = np.load(GOLD / f"birch_file_{name}.npz")
    labels, offsets = z["labels"], z["offsets"]
    _, nfr = oracle.encode_frames(wav, base, 0, 1)
    big = 0
    for f in range(nfr):
        tr = oracle.trace_frame(wav, base, f)
        if tr["N"] <= tr["K"]:
            continue
        big = max(big, tr["N"])
        got = _labels(birch_host, tr["dataset"], tr["K"])
        want = labels[offsets[f]: offsets[f] + tr["N"]]
        assert int((got != want).sum()) == 0, f
    if name.startswith("tone_lsb45"):
        assert big >= 20000
