"""Pin the CPU restatement's third-party primitives to published known answers.

The reference ships no tests or fixtures; CRC-8/SMBUS,
CRC-16/UMTS, MD5 and the UTF-8 frame-number coder come from Zig std /
OpenSSL, whose published check values pin them.
"""
import ctypes
import hashlib

import numpy as np
import pytest

import oracle_ref


def test_crc8_smbus_check():
    # CRC-8/SMBUS catalogue check value (std.hash.crc.Crc8Smbus, frame_writer.zig:138)
    assert oracle_ref.lib().oracle_crc8(b"123456789", 9) == 0xF4


def test_crc16_umts_check():
    # CRC-16/UMTS (a.k.a. BUYPASS) catalogue check value (crc16.zig, std Crc16Umts)
    assert oracle_ref.lib().oracle_crc16(0, b"123456789", 9) == 0xFEE8


def test_crc16_incremental():
    L = oracle_ref.lib()
    data = bytes(range(256)) * 7
    c = 0
    for i in range(0, len(data), 37):
        c = L.oracle_crc16(c, data[i:i + 37], len(data[i:i + 37]))
    assert c == L.oracle_crc16(0, data, len(data))



def test_crc16_sliced_equals_bitwise():
    """oracle_crc16 (slicing-by-8 tables) equals the one-bit-per-step definition for every
    start value class, length 0..70 (both the 8-byte body and the byte tail) and random data."""
    import random

    L = oracle_ref.lib()
    assert L.oracle_crc16_bitwise(0, b"123456789", 9) == 0xFEE8
    rnd = random.Random(7)
    for n in list(range(71)) + [4096, 10357]:
        data = bytes(rnd.randrange(256) for _ in range(n))
        for crc in (0, 0xFFFF, rnd.randrange(65536)):
            assert L.oracle_crc16(crc, data, n) == L.oracle_crc16_bitwise(crc, data, n), (n, crc)

RFC1321 = [
    (b"", "d41d8cd98f00b204e9800998ecf8427e"),
    (b"a", "0cc175b9c0f1b6a831c399e269772661"),
    (b"abc", "900150983cd24fb0d6963f7d28e17f72"),
    (b"message digest", "f96b697d7cb7938d525a2f31aaf161d0"),
    (b"abcdefghijklmnopqrstuvwxyz", "c3fcd3d76192e4007dfb496cca67e13b"),
    (b"ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789", "d174ab98d277d9f5a5611c2c9f419d9f"),
    (b"1234567890" * 8, "57edf4a22be3c955ac49da2e2107b67a"),
]


@pytest.mark.parametrize("msg,hexd", RFC1321)
def test_md5_rfc1321(msg, hexd):
    out = ctypes.create_string_buffer(16)
    oracle_ref.lib().oracle_md5(msg, len(msg), out)
    assert out.raw.hex() == hexd


def test_md5_lengths_vs_hashlib():
    L = oracle_ref.lib()
    rng = np.random.default_rng(5)
    out = ctypes.create_string_buffer(16)
    for n in list(range(0, 200)) + [4095, 4096, 4097, 100003]:
        m = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        L.oracle_md5(m, n, out)
        assert out.raw == hashlib.md5(m).digest(), n


def _flac_utf8(v: int) -> bytes:
    """FLAC 'UTF-8' coded number (RFC 9639 9.1.5), up to 36 bits, independent of the oracle."""
    if v < 0x80:
        return bytes([v])
    for nbytes, lead, cap in [(2, 0xC0, 11), (3, 0xE0, 16), (4, 0xF0, 21), (5, 0xF8, 26), (6, 0xFC, 31),
                              (7, 0xFE, 36)]:
        if v < (1 << cap):
            out = []
            for _ in range(nbytes - 1):
                out.append(0x80 | (v & 0x3F))
                v >>= 6
            out.append(lead | v)
            return bytes(reversed(out))
    raise ValueError(v)


def test_utf8_frame_number_matches_utf8():
    L = oracle_ref.lib()
    buf = ctypes.create_string_buffer(8)
    # standard UTF-8 for the code-point range (surrogates encoded as plain 3-byte sequences)
    for v in list(range(0, 70000)) + list(range(0x10FFF0, 0x110000)):
        k = L.oracle_utf8_number(v, buf)
        assert buf.raw[:k] == chr(v).encode("utf-8", "surrogatepass"), v


def test_utf8_frame_number_36bit():
    L = oracle_ref.lib()
    buf = ctypes.create_string_buffer(8)
    rng = np.random.default_rng(1)
    vals = [(1 << b) - 1 for b in range(1, 37)] + [1 << b for b in range(0, 36)]
    vals += [int(x) for x in rng.integers(0, 1 << 36, 2000, dtype=np.int64)]
    for v in vals:
        k = L.oracle_utf8_number(v, buf)
        assert buf.raw[:k] == _flac_utf8(v), v
