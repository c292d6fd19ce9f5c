"""The reference's own invocations and test files (encoder/encoder.lps:260-279
session history; opus_test/, my_test/, lame_test/ inputs) through the HIP
encoder, against the oracle's digests (tests/golden/refinv_meta.json, made by
tests/golden/make_refinv.py).  -pr0 on real audio keeps more than 4096
passthrough chunks after KNNFit, so the reference stops at SaveStream's
Assert (encoder.lpr:986): the product must refuse those files the same way."""
from __future__ import annotations

import hashlib
import json
from pathlib import Path

import pytest

GOLD = Path(__file__).resolve().parent / "golden"
META = json.loads((GOLD / "refinv_meta.json").read_text())


@pytest.mark.parametrize("name", sorted(META))
def test_inputs_are_the_recorded_files(name):
    ent = META[name]
    wav = (GOLD / "ref_inputs" / ent["input"]).read_bytes()
    assert hashlib.sha256(wav).hexdigest() == ent["wav_sha256"]


@pytest.mark.gpu
@pytest.mark.timeout(300)
@pytest.mark.parametrize("name", sorted(META))
def test_reference_invocation_matches_oracle(name):
    import soundchunks_amd as sc
    from soundchunks_amd import _lib

    ent = META[name]
    wav = (GOLD / "ref_inputs" / ent["input"]).read_bytes()
    enc = sc.Encoder(ent["argv"])
    assert enc.frame_count(wav) == ent["frames"]
    if ent["error"]:
        with pytest.raises(_lib.GscError, match="SaveStream: Assert"):
            enc.encode(wav)
        return
    got = enc.encode(wav)
    assert len(got) == ent["gsc_bytes"]
    assert hashlib.sha256(got).hexdigest() == ent["gsc_sha256"]


@pytest.mark.gpu
def test_py_precision_reaches_only_cluster_py():
    """`-fl500 -cpf256 -py -pr7` (encoder.lps:263): Precision reaches only
    cluster.py's -t argument (extern.pas:390), which Birch ignores
    (cluster.py:21 hard-codes threshold 0.001), and -py runs no
    KNNScanReduce: the .gsc equals the -pr3 golden."""
    import soundchunks_amd as sc

    wav = (GOLD / "lame_test" / "mstest.wav").read_bytes()
    got = sc.Encoder(["-fl500", "-cpf256", "-py", "-pr7"]).encode(wav)
    assert got == (GOLD / "mstest_fl500_cpf256_py.gsc").read_bytes()


@pytest.mark.gpu
def test_pr0_noise_fails_like_the_reference():
    import soundchunks_amd as sc
    from soundchunks_amd import _lib
    from soundchunks_amd.synth import synth_wav

    with pytest.raises(_lib.GscError, match="SaveStream: Assert"):
        sc.Encoder(["-cs8", "-pr0"]).encode(synth_wav(1.0, 44100, 1))
