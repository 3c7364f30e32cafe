"""Deterministic synthetic PCM for parity tests and the benchmark.

Per channel c: three sines (220*(c+1) Hz @ 0.25 FS, 1375.3 Hz @ 0.1 FS,
5512.5 Hz @ 0.03 FS) plus one-pole low-passed Gaussian noise (sigma 0.02 FS,
alpha 0.9); every odd channel is 0.9 * its left neighbour plus a little
independent noise, so L/S, S/R and M/S all get chosen.  Every 64th block
cycles through the special cases the encoder must handle: all-zero
(CONSTANT, waste = bps), DC constant, full-scale white noise (VERBATIM /
escape partitions), samples << 3 (wasted bits) and +/- full-scale
alternation (wide-overflow path at 32 bit).  Seed = 20260821 + stream id.

Returns interleaved little-endian PCM bytes exactly as a WAV data chunk holds
them (2/3/4 bytes per sample), which is what the encoder boundary consumes.
"""
from __future__ import annotations

import numpy as np

SEED = 20260821


def _lowpass(x: np.ndarray, alpha: float) -> np.ndarray:
    from scipy.signal import lfilter

    return lfilter([1.0 - alpha], [1.0, -alpha], x)


def synth_samples(n: int, channels: int, bits: int, rate: int, stream: int = 0,
                  block: int = 4096, specials: bool = True) -> np.ndarray:
    """Return int32/int64 samples shaped (n, channels), within the signed bit range."""
    rng = np.random.Generator(np.random.PCG64(SEED + stream))
    fs = float(1 << (bits - 1))
    t = np.arange(n, dtype=np.float64) / rate
    out = np.empty((n, channels), dtype=np.float64)
    for c in range(channels):
        x = (0.25 * np.sin(2 * np.pi * 220.0 * (c + 1) * t + 0.3 * c)
             + 0.10 * np.sin(2 * np.pi * 1375.3 * t + 1.1 * c)
             + 0.03 * np.sin(2 * np.pi * 5512.5 * t + 2.3 * c))
        noise = _lowpass(rng.standard_normal(n), 0.9)
        noise *= 0.02 / max(np.std(noise), 1e-12)
        x = x + noise
        if c % 2 == 1:
            x = 0.9 * out[:, c - 1] / fs + 0.002 * rng.standard_normal(n)
        out[:, c] = x * fs
    lo, hi = -(1 << (bits - 1)), (1 << (bits - 1)) - 1
    s = np.clip(np.rint(out), lo, hi).astype(np.int64)
    if specials:
        nblocks = (n + block - 1) // block
        for b in range(63, nblocks, 64):
            a, e = b * block, min(n, (b + 1) * block)
            kind = (b // 64) % 5
            if kind == 0:
                s[a:e] = 0
            elif kind == 1:
                s[a:e] = rng.integers(lo // 2, hi // 2, size=(1, channels))
            elif kind == 2:
                s[a:e] = rng.integers(lo, hi + 1, size=(e - a, channels))
            elif kind == 3:
                s[a:e] = np.clip(s[a:e] >> 3 << 3, lo, hi) & ~np.int64(7)
            else:
                alt = np.where(np.arange(e - a) % 2 == 0, hi, lo)
                s[a:e] = alt[:, None]
    return s


def to_pcm_bytes(samples: np.ndarray, bits: int) -> bytes:
    """Interleave to little-endian bytes of bits/8 per sample."""
    B = bits // 8
    s = samples.astype(np.int64).reshape(-1)
    u = (s & ((1 << (8 * B)) - 1)).astype(np.uint64)
    b = np.empty((u.size, B), dtype=np.uint8)
    for k in range(B):
        b[:, k] = ((u >> np.uint64(8 * k)) & np.uint64(0xFF)).astype(np.uint8)
    return b.tobytes()


def synth_pcm(n: int, channels: int, bits: int, rate: int, stream: int = 0,
              block: int = 4096, specials: bool = True) -> bytes:
    return to_pcm_bytes(synth_samples(n, channels, bits, rate, stream, block, specials), bits)


def from_pcm_bytes(pcm: bytes, channels: int, bits: int) -> np.ndarray:
    B = bits // 8
    a = np.frombuffer(pcm, dtype=np.uint8).reshape(-1, B).astype(np.int64)
    v = np.zeros(a.shape[0], dtype=np.int64)
    for k in range(B):
        v |= a[:, k] << (8 * k)
    sign = np.int64(1) << (8 * B - 1)
    v = (v ^ sign) - sign
    return v.reshape(-1, channels)
