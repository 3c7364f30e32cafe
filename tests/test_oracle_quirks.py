"""Hand-derived known answers for the decision rules of SURVEY.md Appendix A.

Each case builds a tiny input whose correct outcome follows directly from the
cited reference lines, and checks the CPU restatement produces it.  These pin
the restatement's reading of the reference where no reference output exists.
"""
import numpy as np
import pytest

import oracle_ref

L = oracle_ref.lib()


def frame(planes, bits=16, rate=44100, number=0, **kw):
    planes = [np.asarray(p, dtype=np.int32) for p in planes]
    return oracle_ref.encode_frame(planes, len(planes[0]), number, len(planes), bits, rate, **kw)


def best_order(s, wide=False):
    import ctypes

    a = np.ascontiguousarray(np.asarray(s, dtype=np.int64))
    tot = (ctypes.c_uint64 * 5)()
    k = L.oracle_best_order(a.ctypes.data_as(ctypes.c_void_p), len(a), 1 if wide else 0, tot)
    return k, list(tot)


# ---- fixed.zig:85-167 -------------------------------------------------------------
def test_best_order_lowest_k_on_ties():
    # ramp: |d1| = 1, d2 = d3 = d4 = 0 -> T2 == T3 == T4 == 0, first minimum is k = 2
    k, tot = best_order(np.arange(100))
    assert tot[2] == tot[3] == tot[4] == 0 and k == 2


def test_best_order_excludes_warmup():
    # T_k sums i >= k only (warm-up loop sets e_k[i<k] = 0)
    s = np.array([1000, 0, 0, 0, 0, 0, 0, 0])
    k, tot = best_order(s)
    assert tot[0] == 1000
    assert tot[1] == 1000          # |0 - 1000| at i = 1 only
    assert tot[4] == 1000          # e4[4] = s4 - 4s3 + 6s2 - 4s1 + s0 = 1000


def test_best_order_wide_invalid():
    # wide mode: order invalid if any |e_k| > 2^31 - 1 (warm-up terms included, fixed.zig:160)
    big = 1 << 30
    s = np.array([big, -big] * 4, dtype=np.int64)  # |e0| = 2^30 valid, |e1| = 2^31 invalid
    k, tot = best_order(s, wide=True)
    assert tot[1] == 2**64 - 1 and tot[0] != 2**64 - 1 and k == 0


# ---- rice.zig:343-405 ---------------------------------------------------------------
def test_part_size_no_half_len_at_p0():
    assert L.oracle_rice_part_size(16, 0, 100) == 16 + 200
    assert L.oracle_rice_part_size(16, 1, 100) == 2 * 16 + 100 - 8
    assert L.oracle_rice_part_size(16, 3, 100) == 4 * 16 + (100 >> 2) - 8


def rice_closed_form(S, n, maxp):
    """The GPU kernel's closed-form parameter choice (zig-flac_amd/csrc/fg_device.hpp rice_choose)."""
    if S <= (n + 1) >> 1:
        p = 0
    else:
        two = 2 * n
        m = 0
        if S > two:
            m = S.bit_length() - two.bit_length()
            if (S >> m) > two:
                m += 1
        p = m + 1
    return min(p, maxp - 1)


def rice_scan(S, n, maxp):
    """rice.zig:368-381: strict '<', lowest parameter wins ties."""
    best, bp = None, None
    for p in range(maxp):
        c = L.oracle_rice_part_size(n, p, S)
        if best is None or c < best:
            best, bp = c, p
    return bp, best


def test_rice_closed_form_exhaustive_small():
    for n in range(0, 70):
        for S in range(0, 40 * max(n, 1) + 50):
            for maxp in (1, 2, 5, 14, 30):
                p, c = rice_scan(S, n, maxp)
                q = rice_closed_form(S, n, maxp)
                assert q == p, (S, n, maxp, p, q)


def test_rice_closed_form_random_large():
    rng = np.random.default_rng(3)
    for _ in range(20000):
        n = int(rng.choice([16 - 4, 16, 32, 64, 128, 256, 512, 1024, 2048, 4092, 4096]))
        S = int(rng.integers(0, n * (1 << int(rng.integers(0, 33))) + 1))
        maxp = int(rng.choice([14, 30]))
        p, _ = rice_scan(S, n, maxp)
        assert rice_closed_form(S, n, maxp) == p, (S, n, maxp)


def test_escape_wins_ties():
    # All 16 residuals = 0 except a few: escape cost 5 + w*len must beat equal rice cost.
    # Construct S/len with f(p*) == 5 + w*len: len 16, w = 1 -> esc = 21.  f(0) = 16 + 2S -> S = 2.5 (no).
    # len 16, w = 2: esc 37; f(1) = 32 + S - 8 = 24 + S -> S = 13 with zigzag width 2 means |r| <= 1 -> S <= 16.
    # residual block of the frame partitions cannot be set directly; check the rule on the restatement's
    # primitive: the chosen cost is min(esc, f(p*)) with esc preferred on equality.
    esc = 5 + 2 * 16
    assert L.oracle_rice_part_size(16, 1, 13) == esc  # a tie exists; rice.zig:372 keeps the escape (strict <)


# ---- encoder.zig decisions ------------------------------------------------------------
def test_constant_all_zero_and_flag():
    z = np.zeros(4096, dtype=np.int32)
    data, rec = frame([z, z])
    c = rec.cand
    assert all(c[i].type == 0 and c[i].estimate == 0 for i in range(4))
    assert c[0].waste == 16 and c[3].waste == 17   # waste = bps when all zero (encoder.zig:561)
    # first minimum of [L+R, L+S, S+R, M+S] = all 0 -> independent (code 1)
    assert rec.channel_code == 1
    # header 6 bytes for frame 0 at 44.1k/16/4096: FF F8 C9 18 00 crc; then CONSTANT subframes:
    # 0x00 + 16 zero bits each, never the wasted flag (frame_writer.zig:269-279)
    assert data[:4] == bytes([0xFF, 0xF8, 0xC9, 0x18])
    body = data[6:-2]
    assert body == bytes(6)


def test_constant_dc_value_written_shifted_back():
    v = np.full(4096, 12288, dtype=np.int32)  # 12288 = 3 << 12 -> waste 12
    data, rec = frame([v, v])
    L0 = rec.cand[0]
    assert L0.type == 0 and L0.waste == 12 and L0.constant == 3 and L0.estimate == 4
    # written as (3 << 12) in 16 bits after a 0x00 header
    assert rec.channel_code in (1, 8, 9, 10)


def test_mid_side_from_unshifted_samples():
    rng = np.random.default_rng(0)
    Lr = (rng.integers(-1000, 1000, 4096) * 4).astype(np.int32)   # waste 2 on L
    Rr = (rng.integers(-1000, 1000, 4096) * 4 + 2).astype(np.int32)  # waste 1 on R
    _, rec = frame([Lr, Rr])
    assert rec.cand[0].waste == 2 and rec.cand[1].waste == 1
    # side = L - R computed before any shift: odd values -> waste 1... L-R = 4a - 4b - 2 -> ctz 1
    assert rec.cand[3].waste == 1 and rec.cand[3].bits == 17


def test_stereo_first_minimum():
    # identical channels: side == 0 (constant, est 0), so L+S and S+R and M+S tie at est(L);
    # L+S comes first among them and beats L+R (2*est(L)) -> code 8
    rng = np.random.default_rng(1)
    x = np.cumsum(rng.integers(-50, 50, 4096)).astype(np.int32)
    _, rec = frame([x, x])
    assert rec.cand[3].type == 0 and rec.cand[3].estimate == 0
    assert rec.channel_code == 8


def test_verbatim_for_short_block():
    _, rec = frame([np.array([1, 2, 3, 4], dtype=np.int32)], bits=16)
    assert rec.cand[0].type == 1 and rec.cand[0].estimate == 4 * 16  # n <= 4 -> verbatim (encoder.zig:514)


def test_fixed_needs_strict_improvement():
    # white noise at full scale: fixed estimate >= verbatim -> VERBATIM
    rng = np.random.default_rng(2)
    x = rng.integers(-32768, 32768, 4096).astype(np.int32)
    y = rng.integers(-32768, 32768, 4096).astype(np.int32)
    _, rec = frame([x, y])
    assert rec.cand[0].type == 1


# ---- frame header (frame_writer.zig:151-265) -------------------------------------------
@pytest.mark.parametrize("n,code,extra", [(4096, 12, 0), (256, 8, 0), (192, 1, 0), (576, 7, 2), (1152, 7, 2),
                                          (100, 6, 1), (255, 6, 1), (4095, 7, 2), (128, 6, 1)])
def test_block_size_codes(n, code, extra):
    rng = np.random.default_rng(n)
    x = rng.integers(-100, 100, n).astype(np.int32)
    data, _ = frame([x], bits=16)
    assert data[2] >> 4 == code
    # header length = 4 + 1 (frame 0) + extra + 1 (crc8); its CRC-8 covers the bytes before it
    hl = 4 + 1 + extra
    assert data[hl] == L.oracle_crc8(data[:hl], hl)
    if extra:
        assert int.from_bytes(data[5:5 + extra], "big") == n - 1


@pytest.mark.parametrize("bits,code", [(8, 2), (16, 8), (24, 12), (32, 14)])
def test_bps_codes(bits, code):
    x = np.arange(4096, dtype=np.int32) % 100
    data, _ = frame([x], bits=bits)
    assert data[3] & 0x0F == code


def test_streaminfo_min_max_quirk():
    # one-frame file: the first frame raises max, so min keeps 0xFFFFFF (metadata.zig:35-40)
    import synth

    pcm = synth.synth_pcm(1000, 2, 16, 44100)
    f = oracle_ref.encode_file(pcm, 2, 16, 44100)
    assert f[:4] == b"fLaC" and f[4] == 0x00 and f[5:8] == b"\x00\x00\x22"
    si = f[8:42]
    assert si[4:7] == b"\xff\xff\xff"
    assert int.from_bytes(si[0:2], "big") == 4096 == int.from_bytes(si[2:4], "big")
    # VORBIS_COMMENT (last) with the reference vendor string, no tags: 73-byte header in total
    assert f[42] == 0x84 and f[46:50] == (19).to_bytes(4, "little") and f[50:69] == b"toastori FLAC 0.0.0"
    assert f[69:73] == b"\x00\x00\x00\x00" and f[73:75] == b"\xff\xf8"


def test_unsupported_bits_rejected():
    x = np.zeros(16, dtype=np.int32)
    with pytest.raises(RuntimeError):
        frame([x], bits=12)
