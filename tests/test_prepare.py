"""f3: TEncoder.Load + PrepareFrames (encoder.lpr:1111-1152, 1294-1429) on the
host.  The product evaluates the three sequential f64 power sums in parallel
(soundchunks_amd/csrc/gsc_seqsum.h) and speculates + verifies the frame cut;
the frame boundaries must equal the oracle's sequential loops exactly.  No GPU
needed (gsc_prepare is host code)."""
from __future__ import annotations

import numpy as np
import pytest

from soundchunks_amd.synth import synth_wav, wav_header


def _tone_noise(seconds, rate=44100, ch=1, amp=0.3, noise=0.02, seed=3):
    rng = np.random.default_rng(seed)
    n = int(seconds * rate)
    t = np.arange(n) / rate
    cols = [amp * np.sin(2 * np.pi * (220 + 110 * c) * t) + noise * rng.standard_normal(n) for c in range(ch)]
    x = np.clip(np.stack(cols, 1), -1, 1)
    return wav_header(ch, rate, n) + np.round(x * 32767).astype("<i2").tobytes()


def _bursts(seconds=30.0, rate=44100, seed=4):
    """Loud bursts in silence: very uneven power, cuts far from uniform."""
    rng = np.random.default_rng(seed)
    n = int(seconds * rate)
    x = np.zeros(n)
    for _ in range(12):
        a = int(rng.integers(0, n - rate))
        x[a:a + rate // 3] = rng.uniform(-0.9, 0.9, rate // 3)
    return wav_header(1, rate, n) + np.round(x * 32767).astype("<i2").tobytes()


CASES = [
    ("stereo64_c2", lambda: synth_wav(64.0), ["-cs8", "-cpf4096", "-cbd8"]),
    ("stereo64_vfr05", lambda: synth_wav(64.0), ["-cs8", "-vfr0.5"]),
    ("stereo64_vfr0", lambda: synth_wav(64.0), ["-cs16", "-vfr0"]),
    ("mono_fl500", lambda: _tone_noise(20.0), ["-fl500"]),
    ("mono_bursts", lambda: _bursts(), ["-cs8"]),
    ("mono_bursts_vfr03", lambda: _bursts(), ["-cs4", "-vfr0.3", "-fl1000"]),
    ("stereo48k_cs4", lambda: synth_wav(40.0, 48000), ["-cs4"]),
    ("short", lambda: synth_wav(0.3), ["-cs8"]),
    ("empty", lambda: wav_header(2, 44100, 0), ["-cs8"]),
    ("br128", lambda: synth_wav(30.0), ["-br128", "-vfr0.5", "-cs8"]),
]


@pytest.mark.parametrize("name,make,argv", CASES, ids=[c[0] for c in CASES])
def test_frame_bounds_match_oracle(oracle, name, make, argv):
    import soundchunks_amd as sc

    wav = make()
    want_s, want_e = oracle.frame_bounds(wav, argv)
    p = sc.Encoder(argv).prepare(wav)
    got_s, got_e = p.frame_bounds()
    np.testing.assert_array_equal(got_s, want_s)
    np.testing.assert_array_equal(got_e, want_e)


def test_prepare_frames_checks_bounds():
    import soundchunks_amd as sc
    from soundchunks_amd import _lib

    wav = synth_wav(20.0)
    enc = sc.Encoder(["-cs8"])
    st, en = enc.prepare(wav).frame_bounds()
    q = enc.prepare_frames(wav, st, en, 1, 3)  # a rank's share: only frames 1..2 loaded
    assert q.frame_count == len(st)
    np.testing.assert_array_equal(q.frame_bounds()[0], st)
    bad = en.copy()
    bad[0] += 1  # not contiguous
    with pytest.raises(_lib.GscError):
        enc.prepare_frames(wav, st, bad, 0, 1)


def test_every_prepared_entry_point_checks_the_loaded_range():
    """A gsc_prepare_frames handle holds only its frames' samples: encoding
    other frames through any entry point is an error, never an out-of-bounds
    read (the check runs before any device work, so no GPU is needed)."""
    import soundchunks_amd as sc
    from soundchunks_amd import _lib

    wav = synth_wav(20.0)
    enc = sc.Encoder(["-cs8"])
    st, en = enc.prepare(wav).frame_bounds()
    q = enc.prepare_frames(wav, st, en, 1, 3)
    for call in (lambda: q.encode(0, 2), lambda: q.encode(2, 4), lambda: q.encode(),
                 lambda: q.encode_files(0, 1), lambda: q.encode_files(3, -1),
                 lambda: q.encode_frames(0, 3)):
        with pytest.raises(_lib.GscError, match="outside the range"):
            call()


def test_single_file_handles_are_one_file():
    """gsc_prepare / gsc_prepare_frames handles report one file spanning every frame."""
    import soundchunks_amd as sc

    wav = synth_wav(20.0)
    enc = sc.Encoder(["-cs8"])
    p = enc.prepare(wav)
    np.testing.assert_array_equal(p.file_frames(), [0, p.frame_count])
    st, en = p.frame_bounds()
    q = enc.prepare_frames(wav, st, en, 0, 2)
    np.testing.assert_array_equal(q.file_frames(), [0, len(st)])


def test_prepare_frames_accepts_an_empty_first_frame():
    """The reference's cut can end frame 0 at i = 0 (encoder.lpr:1411-1417:
    curPower >= perFramePower at the first block), leaving frame 0 = (0, -1);
    broadcast bounds with that frame are valid."""
    import soundchunks_amd as sc
    from soundchunks_amd import _lib

    wav = synth_wav(20.0)
    enc = sc.Encoder(["-cs8"])
    st, en = enc.prepare(wav).frame_bounds()
    st2 = np.concatenate([[0], st]).astype(np.int32)
    en2 = np.concatenate([[-1], en]).astype(np.int32)
    q = enc.prepare_frames(wav, st2, en2, 1, 3)
    assert q.frame_count == len(st) + 1
    bad_s = np.concatenate([st[:1], [0], st[1:]]).astype(np.int32)  # an empty frame later on is still refused
    bad_e = np.concatenate([en[:1], [en[0]], en[1:]]).astype(np.int32)
    bad_e[1] = st[1] - 1
    bad_s[1] = st[1]
    with pytest.raises(_lib.GscError):
        enc.prepare_frames(wav, bad_s, bad_e, 0, 1)
