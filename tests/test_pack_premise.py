"""The device index packer's premise (gsc_pack.hip), on the CPU.

TFrame.SaveStream (encoder.lpr:1050-1106) packs each chunk's variable-length
code into a 32-bit `bits` register and flushes one 16-bit word whenever
bitCnt >= 16.  The device packer instead writes the plain LSB-first
concatenation of the codes (a prefix sum of the code sizes).  The two agree
only if the register never drops a bit, which needs bitCnt + codeSize <= 32
for every code.  With CMaxChunksPerFrame = 4096 (encoder.lpr:15) every index
is < 4096.  Here the reference's loop is restated literally, with Cardinal
wrap-around, and compared with the concatenation on random, adversarial and
exhaustive-transition index sequences.
"""
from __future__ import annotations

import itertools

import numpy as np
import pytest

M32 = 0xFFFFFFFF


def vcbs(idx: int) -> int:
    """vcbsCnt (encoder.lpr:1054): 0 for index 0, else BsrWord(index) div 3."""
    return 0 if idx == 0 else (idx.bit_length() - 1) // 3


def code_of(idx: int, neg: int, rev: int, prev_vc: int) -> tuple[int, int]:
    """One chunk's code and size (encoder.lpr:1062-1088)."""
    vc = vcbs(idx)
    code, size = neg, 1
    code |= rev << size
    size += 1
    if vc == prev_vc:
        size += 1
    else:
        code |= 1 << size
        size += 1
        code |= vc << size
        size += 2
    for k in range(vc, -1, -1):
        code |= ((idx >> (3 * k)) & 7) << size
        size += 3
    return code, size


def reference_stream(chunks) -> tuple[bytes, int]:
    """The reference's sequential packer with a 32-bit `bits` register; also
    returns the largest bitCnt + codeSize seen."""
    out = bytearray()
    bits, bit_cnt, prev_vc, worst = 0, 0, -1, 0
    for idx, neg, rev in chunks:
        code, size = code_of(idx, neg, rev, prev_vc)
        worst = max(worst, bit_cnt + size)
        bits = (bits | ((code << bit_cnt) & M32)) & M32
        bit_cnt += size
        if bit_cnt >= 16:
            bit_cnt -= 16
            out += (bits & 0xFFFF).to_bytes(2, "little")
            bits >>= 16
        prev_vc = vcbs(idx)
    if bit_cnt > 0:
        out += (bits & 0xFFFF).to_bytes(2, "little")
    return bytes(out), worst


def concat_stream(chunks) -> bytes:
    """What gsc_pack.hip writes: codes at prefix-sum bit offsets, 16-bit words."""
    acc, total, prev_vc = 0, 0, -1
    for idx, neg, rev in chunks:
        code, size = code_of(idx, neg, rev, prev_vc)
        acc |= code << total
        total += size
        prev_vc = vcbs(idx)
    nwords = (total + 15) // 16
    return acc.to_bytes(2 * nwords, "little") if nwords else b""


def _check(chunks):
    ref, worst = reference_stream(chunks)
    assert worst <= 32
    assert concat_stream(chunks) == ref


@pytest.mark.parametrize("seed", range(8))
def test_random_indices(seed):
    rng = np.random.default_rng(seed)
    n = 3000
    hi = [8, 64, 512, 4096][seed % 4]
    idx = rng.integers(0, hi, n)
    flags = rng.integers(0, 2, (n, 2))
    _check([(int(i), int(a), int(b)) for i, (a, b) in zip(idx, flags)])


def test_every_transition_pair():
    # one representative index per vcbsCnt class, with its largest member, in
    # every order pair, repeated so that bitCnt walks through all residues
    reps = [0, 7, 8, 63, 64, 511, 512, 4095]
    seq = []
    for a, b in itertools.product(reps, repeat=2):
        for _ in range(17):
            seq += [(a, 1, 1), (b, 1, 0)]
    _check(seq)


def test_longest_codes_back_to_back():
    # 17-bit codes need a vcbsCnt change to 3; alternate with every shorter class
    seq = []
    for other in (0, 7, 63, 511):
        for _ in range(40):
            seq += [(4095, 1, 1), (other, 1, 1)]
    seq += [(4095, 1, 1)] * 50  # same class: 15-bit codes
    _check(seq)


def test_index_4096_would_break_the_premise():
    # beyond CMaxChunksPerFrame the 2-bit vcbsCnt field overflows and the
    # register drops bits: the device packer is specified for r <= 4096 only
    seq = [(8191, 1, 1), (63, 1, 1), (8191, 1, 1)] * 20
    ref, worst = reference_stream(seq)
    assert worst > 32
    assert concat_stream(seq) != ref
