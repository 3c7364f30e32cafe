"""Adversarial blocks (tests/fuzz_blocks.py) on the GPU vs the CPU restatement:
bit-exact streams and per-frame sizes for random kinds, channel counts, bit
depths, ragged tails and LPC settings."""
import pytest

import fuzz_blocks
import oracle_ref
from test_gpu_parity import _diff_msg, gpu_encoder

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("seed", range(64))
def test_gpu_fuzz_parity(seed):
    ch = [2, 1, 3, 8][seed % 4]
    bits = [16, 24, 32, 8][(seed // 4) % 4]
    lpc = [0, 8, 12, 0][(seed // 16) % 4]
    if ch == 8 and bits == 32:
        lpc = 0  # 8-channel 32-bit LPC exceeds the tail kernel's LDS: InvalidConfig (test_abi)
    pcm, n = fuzz_blocks.stream(1000 + seed, ch, bits)
    enc = gpu_encoder(ch, bits, 48000, **({"lpc_order": lpc} if lpc else {}))
    got, sizes = enc.encode_frames(pcm)
    ref, ref_sizes, _ = oracle_ref.encode_stream(pcm, ch, bits, 48000, lpc=lpc)
    assert sizes == ref_sizes, f"sizes differ (seed {seed})"
    assert got == ref, _diff_msg(got, ref)
