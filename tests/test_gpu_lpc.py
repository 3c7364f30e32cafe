"""GPU LPC search (build-defined extension; the reference has no LPC,
readme.md:27) vs the CPU restatement of the same contract (oracle/flac_oracle.c
"LPC -- build-defined extension"): bit-exact streams, per-candidate decision
records (order, shift, quantised coefficients, Rice parameters) and lossless
round trips.  BASELINE configs 3 (96 kHz/24-bit stereo, LPC order 8) and 5
(192 kHz/32-bit stereo, LPC order 12) are covered at parity-test sizes.
"""
import numpy as np
import pytest

import oracle_ref
import synth
from test_gpu_parity import _records_match, check_stream, gpu_encoder

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("ch,bits,rate,q", [
    (2, 24, 96000, 8),    # config 3
    (2, 32, 192000, 12),  # config 5
    (2, 16, 44100, 8),
    (2, 16, 44100, 12),
    (1, 16, 44100, 1),
    (1, 24, 48000, 5),
    (8, 24, 96000, 8),    # config 4 channel layout
    (3, 16, 48000, 9),
    (2, 8, 8000, 4),
    (1, 32, 48000, 12),
    (7, 32, 96000, 12),   # the largest frame whose LPC tail kernel fits LDS
])
def test_lpc_stream_parity(ch, bits, rate, q):
    check_stream(ch, bits, rate, 4096 * 66 + 1000, lpc_order=q)


@pytest.mark.parametrize("tail", [1, 2, 3, 5, 8, 9, 12, 13, 16, 31, 100, 255, 256, 1000, 4095])
@pytest.mark.parametrize("q", [8, 12])
def test_lpc_tails(tail, q):
    check_stream(2, 24, 96000, 4096 + tail, stream=tail, lpc_order=q)


@pytest.mark.parametrize("ch,bits,rate,q", [(2, 24, 96000, 8), (2, 32, 192000, 12), (2, 16, 44100, 12),
                                            (8, 24, 96000, 8)])  # channel-split analysis
def test_lpc_decision_records(ch, bits, rate, q):
    _records_match(ch, bits, rate, 4096 * 66 + 333, lpc=q)


def test_lpc_is_chosen_and_lossless():
    # a strongly predictable signal (two sines, tiny noise): LPC must win most subframes
    n = 4096 * 20
    t = np.arange(n)
    rng = np.random.default_rng(5)
    x = (2 ** 21 * np.sin(t * 1.3) + 2 ** 20 * np.sin(t * 2.1) + rng.normal(0, 3, n)).astype(np.int64)
    s = np.stack([x, (x * 0.75).astype(np.int64)], axis=1).astype("<i4")
    pcm = b"".join(int(v).to_bytes(4, "little", signed=True)[:3] for v in s.reshape(-1))
    enc = gpu_encoder(2, 24, 96000, lpc_order=8)
    enc.set_records(True)
    try:
        got, sizes = enc.encode_frames(pcm)
        recs = enc.records()
    finally:
        enc.set_records(False)
    ref, ref_sizes, _ = oracle_ref.encode_stream(pcm, 2, 24, 96000, lpc=8)
    assert sizes == ref_sizes and got == ref
    lpc_written = sum(1 for r in recs for c in range(r.n_cand) if r.cand[c].written and r.cand[c].type == 3)
    assert lpc_written >= len(recs)  # at least one LPC subframe per frame on average
    dec, _ = oracle_ref.decode_frames(got, 2, 24, 96000, n)
    assert dec == pcm


def test_lpc_order_validation():
    import flacgpu

    with pytest.raises(flacgpu.FlacGpuError):
        flacgpu.Encoder(2, 16, 44100, lpc_order=13, max_frames=16)
    # 8 channels x 32 bit with LPC: the tail kernel's LDS would exceed 160 KiB -> InvalidConfig
    with pytest.raises(flacgpu.FlacGpuError):
        flacgpu.Encoder(8, 32, 96000, lpc_order=8, max_frames=16)
