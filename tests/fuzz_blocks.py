"""Adversarial block generator shared by the fuzz tests (test infrastructure).

Each block kind stresses one decision of the encode path: random walks of a
random step size (Rice parameters across their whole range), sparse spikes
(escape partitions, long unary runs), per-partition mixtures of silence and
noise (mixed escape / Rice partitions), full-scale extremes and alternation
(wide-overflow path, 33-bit sides), constant runs, wasted bits, and sums of
sinusoids (where LPC wins).
"""
import numpy as np

KINDS = ["walk", "spikes", "mixture", "extreme", "constant", "wasted", "sines", "noise"]


def block(rng, n, channels, bits, kind):
    lo, hi = -(1 << (bits - 1)), (1 << (bits - 1)) - 1
    span = hi - lo
    if kind == "walk":
        step = 1 << int(rng.integers(0, bits - 1))
        x = np.cumsum(rng.integers(-step, step + 1, size=(n, channels)), axis=0)
    elif kind == "spikes":
        x = rng.integers(-3, 4, size=(n, channels)).astype(np.int64)
        idx = rng.integers(0, n, size=max(1, n // 97))
        x[idx] = rng.integers(lo, hi + 1, size=(len(idx), channels))
    elif kind == "mixture":
        x = np.zeros((n, channels), dtype=np.int64)
        seg = max(1, n // 16)
        for a in range(0, n, seg):
            amp = 1 << int(rng.integers(0, bits))
            if rng.random() < 0.5:
                x[a:a + seg] = rng.integers(-amp, amp, size=(min(seg, n - a), channels))
    elif kind == "extreme":
        x = np.where(rng.random((n, channels)) < 0.5, lo, hi).astype(np.int64)
        if rng.random() < 0.5:
            x[::2] = lo
            x[1::2] = hi
    elif kind == "constant":
        x = np.full((n, channels), int(rng.integers(lo, hi + 1)), dtype=np.int64)
        if rng.random() < 0.3 and n > 1:
            x[int(rng.integers(0, n))] ^= 1
    elif kind == "wasted":
        w = int(rng.integers(1, bits))
        x = rng.integers(lo >> w, (hi >> w) + 1, size=(n, channels)).astype(np.int64) << w
    elif kind == "sines":
        t = np.arange(n)[:, None]
        f = rng.uniform(0.001, 3.0, size=(1, channels))
        x = (0.4 * np.sin(t * f) + 0.2 * np.sin(t * f * 2.7 + 1.0)) * hi
        x = x + rng.normal(0, 2 ** int(rng.integers(0, max(1, bits - 8))), size=(n, channels))
    else:
        x = rng.integers(lo, hi + 1, size=(n, channels))
    return np.clip(np.rint(x), lo, hi).astype(np.int64)


def stream(seed, channels, bits, n_frames_max=3):
    """PCM bytes of a short stream whose frames are each of a random kind; last frame ragged."""
    import synth

    rng = np.random.default_rng(seed)
    nf = int(rng.integers(1, n_frames_max + 1))
    tail = int(rng.integers(1, 4097))
    parts = [block(rng, 4096 if f < nf - 1 else tail, channels, bits, KINDS[int(rng.integers(0, len(KINDS)))])
             for f in range(nf)]
    s = np.concatenate(parts, axis=0)
    return synth.to_pcm_bytes(s, bits), len(s)
