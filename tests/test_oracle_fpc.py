"""FPC 3.2.2 RTL numerics restated in oracle/fpc_rtl.c:
Cephes-style sin/cos with FPC's own argument reduction, fdlibm ln, log10 =
ln * 0.43429448190325182765.  Checked against mpmath (correctly rounded) on
the finite argument sets the encoder actually uses: the DCT table
((pi/CS)*(n+0.5))*k and the cepstrum DFT table ((-2*pi*k)*i)/N, including
the multiples of pi/2 that take FPC's precise reduction path."""
from __future__ import annotations

import ctypes
import math

import mpmath
import numpy as np
import pytest

import oracle_ffi

mpmath.mp.prec = 200


def _ulps(a: float, b: float) -> float:
    if a == b:
        return 0.0
    return abs(a - b) / math.ulp(max(abs(a), abs(b), 1e-300))


def _args():
    xs = []
    for cs in (4, 8, 16):
        for k in range(cs):
            for n in range(cs):
                xs.append(((math.pi / cs) * (n + 0.5)) * k)
        for k in range(cs):
            for i in range(cs):
                xs.append(((-2 * math.pi) * k * i) / cs)
    xs += [0.0, 1e-9, -1e-9, math.pi / 4, math.pi / 2, math.pi, 3 * math.pi / 2, 100.0, -1000.5, 2.0 ** 31]
    return xs


@pytest.mark.parametrize("fn,ref", [("fpc_sin", mpmath.sin), ("fpc_cos", mpmath.cos)])
def test_trig_within_one_ulp(fn, ref):
    f = getattr(oracle_ffi.load(), fn)
    for x in _args():
        got = f(x)
        want = float(ref(mpmath.mpf(x)))
        if abs(want) < 1e-15:  # exact zeros of the true function: absolute check
            assert abs(got - want) < 1e-15, (fn, x, got, want)
        else:
            assert _ulps(got, want) <= 1.0, (fn, x, got, want)


def test_ln_log10():
    lib = oracle_ffi.load()
    rng = np.random.default_rng(7)
    for x in list(rng.uniform(1e-12, 1e3, 2000)) + [1.0, 2.0, 10.0, 1e-12, 1e300, 5e-324]:
        x = float(x)
        assert _ulps(lib.fpc_ln(x), float(mpmath.log(x))) <= 1.0, x
        assert lib.fpc_log10(x) == lib.fpc_ln(x) * 0.43429448190325182765


def test_ceil_iszero():
    lib = oracle_ffi.load()
    lib.fpc_ceil.argtypes = [ctypes.c_double]
    lib.fpc_ceil.restype = ctypes.c_longlong
    lib.fpc_iszero.argtypes = [ctypes.c_double]
    lib.fpc_iszero.restype = ctypes.c_int
    assert [lib.fpc_ceil(x) for x in (1.0, 1.2, -1.2, 0.0, 32766.5)] == [1, 2, -1, 0, 32767]
    assert lib.fpc_iszero(1e-12) and not lib.fpc_iszero(1.1e-12)
