"""The arithmetic behind yakmo's integer prefix chain (gsc_yakmo.hip chain_fast),
checked against the sequential f32 chain it replaces (the DLL's cum[] prefix,
yakmo_single.dll @0x180001e74).

While the running total stays in one binade every partial is m*u, and
fl(m*u + d) = (m + n)*u with n = rint(d/u) unless d/u is a tie.  chain_fast
resolves ties in place: a tie rounds to the even neighbour of the exact partial
before it, and the parity of the adjustments made up to tie i equals the parity
of the unadjusted (rint) partial at tie i, so the adjustment at tie i is nonzero
exactly when that parity differs from the previous tie's.  Negative totals run
on the negated values.  This emulates one lane's walk (lanes only split the
same recurrence) and compares every accepted partial with the f32 chain.
"""
import numpy as np

F32 = np.float32
LO, HI = (1 << 23) + 1, (1 << 24) - 2


def _integer_chain(run, d):
    """Partials accepted by the integer path (stops at the first point it cannot take)."""
    sgn = -1.0 if run < 0 else 1.0
    fe = np.frexp(abs(float(run)))[1]
    scale = sgn * 2.0 ** (24 - fe)
    t = d.astype(np.float64) * scale
    r = np.rint(t)
    dl = t - r
    q = int(abs(float(run)) * 2.0 ** (24 - fe))
    p, bprev, out = q, 0, []
    for i in range(len(d)):
        if not abs(dl[i]) <= 0.5:
            break
        q += int(r[i])
        c = 0
        if abs(dl[i]) == 0.5:
            b = q & 1
            if b != bprev:
                c = -1 if dl[i] < 0 else 1
            bprev = b
        p += int(r[i]) + c
        if not LO <= p <= HI:
            break
        out.append(p / scale)
    return np.array(out, np.float64)


def _f32_chain(run, d):
    out = np.empty(len(d), F32)
    r = F32(run)
    for i, x in enumerate(d):
        r = F32(r + x)
        out[i] = r
    return out


def test_tie_parity_chain_matches_sequential_f32():
    rng = np.random.default_rng(20250217)
    accepted = ties = 0
    for _ in range(3000):
        sgn = rng.choice([-1.0, 1.0])
        e = int(rng.integers(-20, 20))
        u = 2.0 ** (e - 23)
        m0 = int(rng.integers(2 ** 23, 2 ** 24 - (2 ** 20 if rng.random() < 0.5 else 0)))
        run = F32(sgn * m0 * u)
        n = int(rng.integers(1, 160))
        kind = rng.random(n)
        frac = np.where(kind < 0.4, 0.5, np.where(kind < 0.6, 0.0, rng.random(n)))
        frac = np.where(rng.random(n) < 0.5, frac, -frac)
        base = rng.integers(-50, 200, n).astype(np.float64)
        d = (sgn * (base + frac) * u).astype(F32)
        got = _integer_chain(run, d)
        want = _f32_chain(run, d)[: len(got)]
        assert np.array_equal(got.astype(F32), want)
        accepted += len(got)
        ties += int(np.sum(np.abs(frac[: len(got)]) == 0.5))
    assert accepted > 100000 and ties > 30000  # the ties were exercised, not skipped
