"""Adversarial blocks (tests/fuzz_blocks.py) through the CPU restatement: every
stream must decode losslessly through the independent verifier decoder, with
and without the build-defined LPC search."""
import pytest

import fuzz_blocks
import oracle_ref


@pytest.mark.parametrize("seed", range(40))
def test_fuzz_round_trip(seed):
    ch = [1, 2, 3, 8][seed % 4]
    bits = [16, 24, 32, 8][(seed // 4) % 4]
    lpc = [0, 8, 12, 3][(seed // 16) % 4]
    pcm, n = fuzz_blocks.stream(seed, ch, bits)
    out, sizes, _ = oracle_ref.encode_stream(pcm, ch, bits, 48000, lpc=lpc)
    dec, dsizes = oracle_ref.decode_frames(out, ch, bits, 48000, n)
    assert dec == pcm and dsizes == sizes
