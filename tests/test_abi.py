"""The drop-in boundary without a GPU: the in-tree C-ABI library loads,
exports every symbol include/soundchunks.h declares, parses options exactly
like the oracle (encoder.lpr:201-227, 1985-1998 semantics), and fails loudly
(no CPU fallback) when no gfx950 device is present."""
from __future__ import annotations

import ctypes
import re
from pathlib import Path

import pytest

import oracle_ffi

ROOT = Path(__file__).resolve().parents[1]
HEADER = ROOT / "include" / "soundchunks.h"


def _declared():
    txt = re.sub(r"/\*.*?\*/", "", HEADER.read_text(), flags=re.S)
    names = re.findall(r"\b([a-z_][a-z0-9_]*)\s*\(", txt)
    return sorted({n for n in names if n.startswith(("yakmo_", "ann_", "gsc_"))})


def test_header_lists_reference_boundary():
    names = _declared()
    # exactly the extern.pas:112-123 numeric-library surface
    for n in ("yakmo_create", "yakmo_destroy", "yakmo_load_train_data", "yakmo_train_on_data", "yakmo_get_centroids",
              "ann_kdtree_create", "ann_kdtree_destroy", "ann_kdtree_search", "ann_kdtree_pri_search",
              "ann_kdtree_search_multi", "ann_kdtree_pri_search_multi"):
        assert n in names


def test_library_exports_every_declared_symbol():
    import soundchunks_amd

    lib = soundchunks_amd.load()
    missing = [n for n in _declared() if not hasattr(lib, n)]
    assert not missing, missing
    from soundchunks_amd._lib import SIGNATURES

    assert set(_declared()) == set(SIGNATURES)


ARGVS = [[], ["-cs8", "-cpf4096", "-cbd8"], ["-cs16", "-cpf4096", "-cbd12"], ["-cs8", "-cpf256"], ["-cpf100"],
         ["-cpf9999"], ["-cbd12", "-cb3", "-cs8"], ["-pr2", "-fl2500", "-vfr0.5"], ["-vfr3"], ["-pbb", "-v"],
         ["-cs8", "-cb"], ["-br128"], ["-cbdx"], ["-cs2"], ["-cs6", "-cbd12"], ["-cs12"], ["-cs17"], ["-cs0"]]


@pytest.mark.parametrize("argv", ARGVS)
def test_option_parsing_matches_oracle(argv):
    import soundchunks_amd as sc

    o = sc.parse_options(argv)
    p = oracle_ffi.params(argv)
    for f, _ in p._fields_:
        assert getattr(o, f) == getattr(p, f), (argv, f)


@pytest.mark.parametrize("cs,ok", [(1, True), (3, True), (12, True), (16, True), (0, False), (17, False),
                                   (32, False)])
def test_chunk_size_range(cs, ok):
    """-cs is unclamped in the reference (encoder.lpr:1992); the kernels take
    2*ChunkSize <= 32 features, so ChunkSize 1..16 prepares and anything else is
    refused up front (host code: no GPU needed)."""
    import soundchunks_amd as sc
    from soundchunks_amd.synth import synth_wav

    enc = sc.Encoder([f"-cs{cs}"])
    if ok:
        assert enc.frame_count(synth_wav(5.0)) >= 1
    else:
        with pytest.raises(sc.GscError, match="ChunkSize"):
            enc.frame_count(synth_wav(5.0))


def test_no_gpu_fails_loudly():
    import torch

    if torch.cuda.is_available():
        pytest.skip("GPU present")
    import soundchunks_amd as sc
    from soundchunks_amd.synth import synth_wav

    with pytest.raises(sc.GscError, match="no HIP device|gfx950"):
        sc.Encoder(["-cs8", "-cpf256"]).encode(synth_wav(0.3))
    lib = sc.load()
    assert lib.gsc_device_count() == 0
    # the reference-ABI shim has no CPU fallback either
    assert lib.ann_kdtree_create(None, 0, 0, 1, 0) is None
