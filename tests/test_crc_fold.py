"""The table-free CRC-16 fold of the pack kernels (fg_device.hpp: q_fold, q_word, q_mul, crc_from_q,
crc_lane_q, crc_byte_v, crc_mulmod_v), restated operation for operation in Python and checked against
the oracle's CRC-16/UMTS (crc16.zig:15-57 via oracle/flac_oracle.c oracle_crc16).

P = z^16 + z^15 + z^2 + 1 = (z + 1)(z^15 + z + 1): each lane folds its words mod Q = z^15 + z + 1 with
shifts and XORs (z^15 = z + 1), keeps the parity of its words (the residue mod z + 1), scales by a
host-computed power z^(16 + 32 * words after it) mod Q (fg_api.cpp q_zpow), and the workgroup's XOR of
both recombines by CRT.  The GPU parity tests check the same kernels' bytes end to end; this test pins
the algebra, the fold bounds and the front-zero-padded lane geometry on the CPU."""
import random

import oracle_ref

Q = 0x8003


def q_fold(t):
    h = t >> 15
    return (t & 0x7FFF) ^ h ^ (h << 1)


def q_word(s, w):
    return q_fold(w ^ (s << 4) ^ (s << 2))


def q_mul(a, e):
    r = 0
    for i in range(15):
        if (a >> i) & 1:
            r ^= e << i
    return q_fold(r)


def crc_from_q(qp):
    A = qp & 0x7FFF
    return A ^ (Q if (bin(A).count("1") ^ (qp >> 16)) & 1 else 0)


def crc_byte_v(crc, b):
    t = ((crc >> 8) ^ b) & 255
    return ((crc << 8) ^ (t << 1) ^ (t << 2) ^ (Q if bin(t).count("1") & 1 else 0)) & 0xFFFF


def crc_mulmod_host(a, b):  # fg_api.cpp crc_mulmod_host
    r = 0
    for i in range(15, -1, -1):
        r <<= 1
        if r & 0x10000:
            r ^= 0x18005
        if (a >> i) & 1:
            r ^= b
    return r & 0xFFFF


def crc_zpow(e):
    r, b = 1, 2
    while e:
        if e & 1:
            r = crc_mulmod_host(r, b)
        b = crc_mulmod_host(b, b)
        e >>= 1
    return r


def q_zpow(e):  # fg_api.cpp q_zpow
    r = crc_zpow(e)
    return r ^ Q if r & 0x8000 else r


def crc_mulmod_v(a, b):
    t = 0
    for i in range(16):
        if (a >> i) & 1:
            t ^= b << i
    return crc_from_q(q_fold(q_fold(t)) | ((bin(t).count("1") & 1) << 16))


def frame_crc(data, NT, two_chains=False):
    """One frame as the kernels fold it: NT threads, 2H words each, front-padded with zeros."""
    W4 = len(data) // 4
    words = [int.from_bytes(data[4 * i:4 * i + 4], "big") for i in range(W4)]
    H = max((W4 + 2 * NT - 1) // (2 * NT), 1)
    if two_chains:  # k_pack: H odd, two interleaved halves joined by z^(32H)
        H |= 1
    Z = NT * 2 * H - W4

    def word(r):
        return words[r] if r >= 0 else 0

    qp = 0
    for t in range(NT):
        va = t * 2 * H - Z
        e = q_zpow(16 + 64 * H * (NT - 1 - t))
        if two_chains:
            sa = sb = px = 0
            for i in range(H):
                wa, wb = word(va + i), word(va + H + i)
                sa, sb = q_word(sa, wa), q_word(sb, wb)
                assert sa < 1 << 18 and sb < 1 << 18
                px ^= wa ^ wb
            ct = q_fold(q_mul(q_fold(sa), q_zpow(32 * H)) ^ sb)
            contrib = q_mul(ct, e)
        else:
            s = px = 0
            for i in range(2 * H):
                w = word(va + i)
                s = q_word(s, w)
                assert s < 1 << 18
                px ^= w
            assert q_fold(s) < 1 << 15
            contrib = q_mul(q_fold(s), e)
        assert contrib < 1 << 15
        qp ^= contrib | ((bin(px).count("1") & 1) << 16)
    crc = crc_from_q(qp)
    for b in data[4 * W4:]:
        crc = crc_byte_v(crc, b)
    return crc


def test_byte_step_matches_table_crc():
    L = oracle_ref.lib()
    for crc in (0, 1, 0x8000, 0xFFFF, 0x1234):
        for b in range(256):
            assert crc_byte_v(crc, b) == L.oracle_crc16(crc, bytes([b]), 1)


def test_q_power_table_and_mulmod():
    rng = random.Random(5)
    for _ in range(2000):
        a, b = rng.randrange(1 << 16), rng.randrange(1 << 16)
        assert crc_mulmod_v(a, b) == crc_mulmod_host(a, b)
    for e in (0, 1, 15, 16, 32, 1000, 64 * 3 * 511 + 16):
        assert q_zpow(e) < 1 << 15


def test_frame_fold_matches_oracle():
    L = oracle_ref.lib()
    rng = random.Random(7)
    for trial in range(120):
        n = rng.choice([0, 1, 3, 4, 5, 63, 64, 255, 1000, 4099]) + rng.randrange(4)
        data = bytes(rng.randrange(256) for _ in range(n))
        want = L.oracle_crc16(0, data, n)
        NT = rng.choice([1, 2, 64, 128, 512])
        assert frame_crc(data, NT) == want, (n, NT)
        assert frame_crc(data, NT, two_chains=True) == want, (n, NT)
