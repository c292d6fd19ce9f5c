"""Synthetic benchmark input: canonical 44-byte RIFF/WAVE PCM16.

L = 0.25*sin(2*pi*440*t) + 0.05*N(0,1); R = 0.25*sin(2*pi*660*t) + 0.05*N(0,1);
clip to [-1, 1]; int16 = round(x * 32767); numpy Generator(PCG64(20250217)).
The reference loader copies exactly 44 header bytes (encoder.lpr:1133) and
treats the rest as interleaved samples (encoder.lpr:1137-1145).
"""
from __future__ import annotations

import struct

import numpy as np

SEED = 20250217


def wav_header(channels: int, rate: int, n_frames: int) -> bytes:
    data_len = n_frames * channels * 2
    return struct.pack(
        "<4sI4s4sIHHIIHH4sI",
        b"RIFF", 36 + data_len, b"WAVE", b"fmt ", 16, 1, channels, rate,
        rate * channels * 2, channels * 2, 16, b"data", data_len,
    )


def synth_pcm(seconds: float, rate: int = 44100, channels: int = 2, seed: int = SEED,
              chunk: int = 1 << 22) -> np.ndarray:
    """Interleaved int16 samples, shape (n_frames, channels).  Generated in
    chunks (the normal stream of one Generator is the same whether drawn at
    once or in pieces), so a long signal never holds n float64 temporaries."""
    n = int(round(seconds * rate))
    rng = np.random.Generator(np.random.PCG64(seed))
    freqs = [440.0, 660.0]
    out = np.empty((n, channels), dtype=np.int16)
    for c in range(channels):  # channel 0's noise first, then channel 1's
        for a in range(0, n, chunk):
            b = min(n, a + chunk)
            t = np.arange(a, b, dtype=np.float64) / rate
            x = 0.25 * np.sin(2.0 * np.pi * freqs[c % 2] * t) + 0.05 * rng.standard_normal(b - a)
            x = np.clip(x, -1.0, 1.0)
            out[a:b, c] = np.round(x * 32767.0).astype(np.int16)
    return out


def synth_wav(seconds: float, rate: int = 44100, channels: int = 2, seed: int = SEED) -> bytes:
    pcm = synth_pcm(seconds, rate, channels, seed)
    return wav_header(channels, rate, pcm.shape[0]) + pcm.astype("<i2", copy=False).tobytes()


if __name__ == "__main__":  # pragma: no cover
    import sys

    secs = float(sys.argv[1]) if len(sys.argv) > 1 else 10.0
    rate = int(sys.argv[3]) if len(sys.argv) > 3 else 44100
    with open(sys.argv[2] if len(sys.argv) > 2 else "synth.wav", "wb") as f:
        f.write(synth_wav(secs, rate))
