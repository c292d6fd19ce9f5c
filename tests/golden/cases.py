"""Golden parity cases: inputs and flags.  Expected .gsc bytes are produced by
the C oracle (oracle/) with tests/golden/make_golden.py and committed next to
this file; GPU tests compare the HIP path against them byte for byte.

Reference inputs (data files the reference's own test corpus holds):
  my_test_test.wav   = /root/reference/my_test/test.wav   (config C1)
  lame_test_hihat.wav = /root/reference/lame_test/hihat.wav (corpus C4 member)
Synthetic inputs are regenerated deterministically (soundchunks_amd.synth).
"""
from __future__ import annotations

from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent


def _synth(seconds, rate=44100, channels=2):
    from soundchunks_amd.synth import synth_wav

    return synth_wav(seconds, rate, channels)


def _silence_tone(seconds=2.0, rate=44100):
    """1/2 digital silence then a tone: exact ties / duplicate points (edge case)."""
    from soundchunks_amd.synth import wav_header

    n = int(seconds * rate)
    t = np.arange(n) / rate
    x = np.where(t < seconds / 2, 0.0, 0.3 * np.sin(2 * np.pi * 220 * t))
    pcm = np.round(x * 32767).astype("<i2")
    return wav_header(1, rate, n) + pcm.tobytes()


def _quiet_tone(seconds=3.0, frac=0.6, rate=44100, seed=5):
    """Mono: +-1 LSB noise for the first `frac`, then a tone.  Thousands of
    reduced chunks quantise to all zeros, so KNNFit queries in the quiet part
    tie with far more than 64 candidates: ANN's bucket order decides them
    (encoder.lpr:945-958)."""
    from soundchunks_amd.synth import wav_header

    rng = np.random.default_rng(seed)
    n = int(seconds * rate)
    t = np.arange(n) / rate
    x = np.round(0.3 * np.sin(2 * np.pi * 330 * t) * 32767).astype(np.int64)
    x = np.where(t < seconds * frac, rng.integers(-1, 2, size=n), x)
    return wav_header(1, rate, n) + x.astype("<i2").tobytes()


def _tone_lsb(seconds=4.5, rate=44100, seed=7):
    """Mono 220 Hz tone with +-1 LSB noise: full 4-s frames (N ~ 44100 chunks at
    ChunkSize 4) whose Birch subclusters stay in the thousands (the -py case)."""
    from soundchunks_amd.synth import wav_header

    rng = np.random.default_rng(seed)
    n = int(seconds * rate)
    t = np.arange(n) / rate
    x = np.round(0.3 * np.sin(2 * np.pi * 220 * t) * 32767).astype(np.int64) + rng.integers(-1, 2, size=n)
    return wav_header(1, rate, n) + x.astype("<i2").tobytes()


def _silence_burst(seconds=3.0, rate=44100):
    """Mono digital silence with one 0.1-s tone burst: with -pr0 every chunk is
    its own reduced chunk (passthrough, encoder.lpr:891-905), N ~ 16,500 > 4096,
    but KNNFit maps the silent chunks onto one zero entry, so the pruned list
    fits SaveStream's 4096 (encoder.lpr:986) and the reference encodes it."""
    from soundchunks_amd.synth import wav_header

    n = int(seconds * rate)
    t = np.arange(n) / rate
    x = np.where((t >= 1.0) & (t < 1.1), 0.25 * np.sin(2 * np.pi * 440 * t), 0.0)
    return wav_header(1, rate, n) + np.round(x * 32767).astype("<i2").tobytes()


def _square_empty_first(seconds=3.0, rate=44100):
    """Mono full-scale square wave whose first sample is 0: every later sample
    has power 1, so totalPower = 1 and at -cs4 (no padding) the cut loop ends
    frame 0 at its first sample (encoder.lpr:1411-1417: curPower >= perFramePower
    at i = 0), leaving frame 0 = (0, -1) -- one chunk (MakeChunks' ChunkCount =
    (-1) div ChunkSize + 1) -- before one frame with the rest."""
    from soundchunks_amd.synth import wav_header

    n = int(seconds * rate)
    t = np.arange(n) / rate
    x = np.where(np.sin(2 * np.pi * 220 * t + 0.1) >= 0, 32767, -32767).astype(np.int64)
    x[0] = 0
    return wav_header(1, rate, n) + x.astype("<i2").tobytes()


def _tiny():
    """0.02 s: fewer chunks than ChunksPerFrame -> passthrough mode (encoder.lpr:891-912)."""
    return _synth(0.02)


CASES = {
    # name: (input factory, argv)
    "c1_test_cs8_cpf256": (lambda: (HERE / "my_test_test.wav").read_bytes(), ["-cs8", "-cpf256"]),
    "hihat_cs8_cpf256": (lambda: (HERE / "lame_test_hihat.wav").read_bytes(), ["-cs8", "-cpf256"]),
    "hihat_cs4_default": (lambda: (HERE / "lame_test_hihat.wav").read_bytes(), ["-cpf512"]),
    "syn2s_c2_cs8_cpf4096": (lambda: _synth(2.0), ["-cs8", "-cpf4096", "-cbd8"]),
    "syn3s_cs8_cpf1000_cbd12": (lambda: _synth(3.0), ["-cs8", "-cpf1000", "-cbd12"]),
    "silence_tone_cs8_cpf256": (lambda: _silence_tone(), ["-cs8", "-cpf256"]),
    "tiny_passthrough_cs8": (lambda: _tiny(), ["-cs8", "-cpf256"]),
    # KNNFit tie sets beyond the 64-NN bucket (ANN priority-search order)
    "quiet_tone_cs8_cpf1024": (lambda: _quiet_tone(), ["-cs8", "-cpf1024"]),
    "quiet_tone_cs4_cpf1024": (lambda: _quiet_tone(frac=0.9), ["-cs4", "-cpf1024"]),
    # C2 at the benchmark's frame shape: two full 4-s frames (N = 44100 each) in one launch
    "syn8s_c2_cs8_cpf4096": (lambda: _synth(8.0), ["-cs8", "-cpf4096", "-cbd8"]),
    # C3: ChunkSize 16 (D = 32 features), 12-bit, two N = 22050 frames
    "syn8s_c3_cs16_cpf4096_cbd12": (lambda: _synth(8.0), ["-cs16", "-cpf4096", "-cbd12"]),
    # C5: 48 kHz stereo at ChunkCount 4096, the encoder default ChunkSize 4 and 8
    "syn8s_48k_cs4_cpf4096": (lambda: _synth(8.0, 48000), ["-cs4", "-cpf4096"]),
    "syn8s_48k_cs8_cpf4096": (lambda: _synth(8.0, 48000), ["-cs8", "-cpf4096"]),
    # the reference's own -br invocations (encoder/encoder.lps:270-279): ChunksPerFrame from the bit-rate
    # cost loop (encoder.lpr:1337-1351) -- K = 485 and 1852 here, not powers of two
    "syn8s_br128_vfr05_cs8": (lambda: _synth(8.0), ["-br128", "-vfr0.5", "-cs8"]),
    "syn8s_br128_vfr05_cs16": (lambda: _synth(8.0), ["-br128", "-vfr0.5", "-cs16"]),
    # -pr0 (Precision 0: passthrough, encoder.lpr:808) with more than 4096 chunks per frame:
    # KNNFit over 4N candidates; quiet input keeps <= 4096 entries after pruning
    "silence_burst_pr0_cs8": (lambda: _silence_burst(), ["-cs8", "-pr0"]),
    "quiet_tone_pr0_cs4": (lambda: _quiet_tone(seconds=2.0, frac=0.97), ["-cs4", "-pr0"]),
    # any ChunkSize (-cs is unclamped, encoder.lpr:1992; odd sizes, decoder.lpr:151-156): 2*CS features
    # padded with zeros to the 8 / 16 / 32-wide kernels (gsc_device.h feature_stride)
    "syn3s_cs2_cpf512": (lambda: _synth(3.0), ["-cs2", "-cpf512"]),
    "syn3s_cs3_mono_cbd12": (lambda: _synth(3.0, 44100, 1), ["-cs3", "-cpf1000", "-cbd12"]),
    "syn3s_cs6_cpf1024_cbd12": (lambda: _synth(3.0), ["-cs6", "-cpf1024", "-cbd12"]),
    "syn3s_cs12_cpf2048": (lambda: _synth(3.0), ["-cs12", "-cpf2048"]),
    # ChunkSize 1 (2 features in the 8-wide kernels) and odd sizes in the 16-wide (5, 7) and
    # 32-wide (9, 15) kernels: the odd-size sign / reverse split, the half-dimension tail box and
    # the non-power-of-two residual divisor
    "syn1s_cs1_cpf256": (lambda: _synth(1.0), ["-cs1", "-cpf256"]),
    "syn2s_cs5_cpf512": (lambda: _synth(2.0), ["-cs5", "-cpf512"]),
    "syn2s_cs7_mono_cbd12": (lambda: _synth(2.0, 44100, 1), ["-cs7", "-cpf1024", "-cbd12"]),
    "syn2s_cs9_cpf512": (lambda: _synth(2.0), ["-cs9", "-cpf512"]),
    "syn3s_cs15_cpf1024_cbd12": (lambda: _synth(3.0), ["-cs15", "-cpf1024", "-cbd12"]),
    # an empty frame 0 = (0, -1) from the reference's cut, encoded (one chunk)
    "square_empty_frame0_cs4": (lambda: _square_empty_first(), ["-cs4", "-cpf512"]),
    # a frame of more than 262,144 chunks (13-s frames at 48 kHz stereo -cs4: N ~ 312,000): yakmo's
    # chosen-point bitmap and prefix summaries live in HBM instead of LDS
    "syn13s_48k_cs4_cpf256_fl13000": (lambda: _synth(13.0, 48000), ["-cs4", "-cpf256", "-fl13000"]),
}


def golden_path(name: str) -> Path:
    return HERE / f"{name}.gsc"
