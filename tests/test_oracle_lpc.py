"""CPU checks of the LPC contract (build-defined extension; the reference has
no LPC: readme.md:27, encoder.zig:629-640,694-699).  The restatement in
oracle/flac_oracle.c is pinned here by (1) an independent Python statement of
each step with exact integer / IEEE-double arithmetic, (2) hand-derived
known answers, and (3) lossless round trips through the verifier decoder.
Parity with any external encoder is not claimed (none exists for this contract).
"""
import ctypes
import math

import numpy as np
import pytest

import oracle_ref
import synth


def _lib():
    L = oracle_ref.lib()
    L.oracle_lpc_autocorr.restype = ctypes.c_int
    L.oracle_lpc_levinson.restype = ctypes.c_int
    L.oracle_lpc_quantize.restype = ctypes.c_int
    return L


def _autocorr(x, max_lag):
    L = _lib()
    xa = np.ascontiguousarray(np.asarray(x, dtype=np.int64))
    R = (ctypes.c_int64 * (max_lag + 1))()
    sh = L.oracle_lpc_autocorr(xa.ctypes.data_as(ctypes.c_void_p), len(xa), max_lag, R)
    return sh, list(R)


def _py_autocorr(x, max_lag):
    n = len(x)
    m = max(abs(int(v)) for v in x)
    wmax = (n + 1) * (n + 1) // 4
    sh = max(0, m.bit_length() + wmax.bit_length() - 25)
    xw = [(int(x[i]) * (i + 1) * (n - i)) >> sh for i in range(n)]
    assert all(abs(v) <= 1 << 25 for v in xw)
    return sh, [sum(xw[i] * xw[i - g] for i in range(g, n)) for g in range(max_lag + 1)]


def _py_levinson(R, Q):
    r = [float(v) for v in R]
    out = []
    if not r[0] > 0.0:
        return out
    err, a = r[0], []
    for m in range(Q):
        acc = r[m + 1]
        for t in range(m):
            acc = acc - a[t] * r[m - t]
        k = acc / err
        a = [a[t] - k * a[m - 1 - t] for t in range(m)] + [k]
        out.append(list(a))
        err = err * (1.0 - k * k)
        if not err > 0.0:
            break
    return out


def _py_quantize(a, prec=15):
    cmax = max(abs(v) for v in a)
    if not cmax > 0.0:
        return None
    _, e = math.frexp(cmax)
    sh = min(prec - 1 - e, 15)
    if sh < 0:
        return None
    qmax, qmin = (1 << (prec - 1)) - 1, -(1 << (prec - 1))
    carry, q = 0.0, []
    for v in a:
        v = v * float(1 << sh)
        v = v + carry
        qi = math.floor(v + 0.5) if v >= 0.0 else -math.floor(-v + 0.5)
        qi = max(qmin, min(qmax, qi))
        carry = v - float(qi)
        q.append(qi)
    return q, sh


@pytest.mark.parametrize("n,bits,seed", [(4096, 16, 0), (4096, 24, 1), (4096, 33, 2), (1000, 16, 3), (13, 24, 4),
                                         (2, 8, 5)])
def test_autocorr_matches_exact_python(n, bits, seed):
    rng = np.random.default_rng(seed)
    x = rng.integers(-(1 << (bits - 1)), 1 << (bits - 1), size=n, dtype=np.int64)
    assert _autocorr(x, 12) == _py_autocorr(x, min(12, n - 1) if n > 12 else 12) or n <= 12
    if n > 12:
        assert _autocorr(x, 12) == _py_autocorr(x, 12)


def test_levinson_ar1_known_answer():
    # R = [1e6, 5e5, 2.5e5]: order 1 = [0.5]; order 2 = [0.5, 0.0] exactly
    L = _lib()
    R = (ctypes.c_int64 * 3)(1000000, 500000, 250000)
    C = (ctypes.c_double * (32 * 32))()
    assert L.oracle_lpc_levinson(R, 2, C) == 2
    assert C[0] == 0.5 and C[32] == 0.5 and C[33] == 0.0
    q = (ctypes.c_int32 * 32)()
    sh = ctypes.c_int()
    assert L.oracle_lpc_quantize(C, 1, 15, q, ctypes.byref(sh)) == 0
    assert (q[0], sh.value) == (8192, 14)  # 0.5 = 0.5 * 2^0 -> shift 14 - 0


def test_levinson_and_quantize_match_python():
    L = _lib()
    for stream in range(6):
        x = synth.synth_samples(4096, 1, 24, 96000, stream=stream)[:, 0].astype(np.int64)
        _, R = _autocorr(x, 12)
        Ra = (ctypes.c_int64 * 13)(*R)
        C = (ctypes.c_double * (32 * 32))()
        valid = L.oracle_lpc_levinson(Ra, 12, C)
        ref = _py_levinson(R, 12)
        assert valid == len(ref)
        for q in range(1, valid + 1):
            got = [C[(q - 1) * 32 + t] for t in range(q)]
            assert got == ref[q - 1]  # bit-identical doubles
            qc = (ctypes.c_int32 * 32)()
            sh = ctypes.c_int()
            rc = L.oracle_lpc_quantize(C[(q - 1) * 32:(q - 1) * 32 + 32] and (ctypes.c_double * 32)(*got), q, 15, qc,
                                       ctypes.byref(sh))
            pq = _py_quantize(got)
            if pq is None:
                assert rc == -1
            else:
                assert rc == 0 and (list(qc)[:q], sh.value) == pq


def test_quantize_edge_cases():
    L = _lib()
    qc = (ctypes.c_int32 * 32)()
    sh = ctypes.c_int()
    # all-zero coefficients: unusable
    assert L.oracle_lpc_quantize((ctypes.c_double * 2)(0.0, 0.0), 2, 15, qc, ctypes.byref(sh)) == -1
    # |a| >= 2^14 needs a negative shift: unusable
    assert L.oracle_lpc_quantize((ctypes.c_double * 1)(20000.0,), 1, 15, qc, ctypes.byref(sh)) == -1
    # tiny coefficients clamp the shift to 15
    assert L.oracle_lpc_quantize((ctypes.c_double * 1)(1e-6,), 1, 15, qc, ctypes.byref(sh)) == 0
    assert sh.value == 15 and qc[0] == 0
    # error feedback: 3 x 1/3 at shift 15 -> 10923, 10922, 10923 (sum preserved)
    assert L.oracle_lpc_quantize((ctypes.c_double * 3)(1 / 3, 1 / 3, 1 / 3), 3, 15, qc, ctypes.byref(sh)) == 0
    assert sh.value == 15 and list(qc)[:3] == _py_quantize([1 / 3] * 3)[0]


@pytest.mark.parametrize("ch,bits,rate,q", [(2, 16, 44100, 8), (2, 24, 96000, 8), (2, 32, 192000, 12),
                                            (1, 16, 44100, 32), (8, 24, 96000, 8), (2, 8, 8000, 3)])
def test_lpc_round_trip(ch, bits, rate, q):
    n = 4096 * 9 + 123
    pcm = synth.synth_pcm(n, ch, bits, rate, stream=q)
    out, sizes, md5 = oracle_ref.encode_stream(pcm, ch, bits, rate, lpc=q)
    dec, dsizes = oracle_ref.decode_frames(out, ch, bits, rate, n)
    assert dec == pcm and dsizes == sizes


def test_lpc_wins_on_predictable_signal():
    n = 4096 * 4
    t = np.arange(n)
    # high-frequency sines: fixed differences amplify them, order-4 LPC predicts them
    x = (2 ** 20 * np.sin(t * 1.3) + 2 ** 19 * np.sin(t * 2.1)).astype(np.int64)
    pcm = np.stack([x, x // 2], axis=1).astype("<i4").tobytes()
    fixed, _, _ = oracle_ref.encode_stream(pcm, 2, 32, 48000)
    lpc, _, _ = oracle_ref.encode_stream(pcm, 2, 32, 48000, lpc=8)
    assert len(lpc) < 0.5 * len(fixed)
    planes = [np.ascontiguousarray(np.stack([x, x // 2], axis=1)[:4096, c]).astype(np.int32) for c in range(2)]
    _, rec = oracle_ref.encode_frame(planes, 4096, 0, 2, 32, 48000, lpc=8)
    assert any(rec.written[i].type == 3 for i in range(rec.n_sub))


def test_prediction_zero_is_the_reference_path():
    # LPC off must reproduce the fixed-only stream byte for byte (golden vectors pin it too)
    pcm = synth.synth_pcm(4096 * 3 + 9, 2, 16, 44100)
    a, _, _ = oracle_ref.encode_stream(pcm, 2, 16, 44100)
    b, _, _ = oracle_ref.encode_stream(pcm, 2, 16, 44100, lpc=0)
    assert a == b


def _py_levinson_err(R, Q):
    r = [float(v) for v in R]
    errs = []
    if not r[0] > 0.0:
        return errs
    err, a = r[0], []
    for m in range(Q):
        acc = r[m + 1]
        for t in range(m):
            acc = acc - a[t] * r[m - t]
        k = acc / err
        a = [a[t] - k * a[m - 1 - t] for t in range(m)] + [k]
        err = err * (1.0 - k * k)
        errs.append(err)
        if not err > 0.0:
            break
    return errs


def _py_key(err, q, n, bps):
    # contract step 7: l2(x) = (e - 1) + (2f - 1) for x = f 2^e, f in [0.5, 1)
    if not err > 0.0:
        return -1e300
    f, e = math.frexp(err)
    l2 = float(e - 1) + (2.0 * f - 1.0)
    return l2 * (0.5 * float(n)) + float(q * (bps + 15))


def test_levinson_errors_and_order_key_match_python():
    L = _lib()
    L.oracle_lpc_levinson_err.restype = ctypes.c_int
    L.oracle_lpc_order_key.restype = ctypes.c_double
    L.oracle_lpc_order_key.argtypes = [ctypes.c_double, ctypes.c_uint, ctypes.c_uint32, ctypes.c_uint]
    for stream in range(6):
        x = synth.synth_samples(4096, 1, 24, 96000, stream=stream)[:, 0].astype(np.int64)
        _, R = _autocorr(x, 12)
        Ra = (ctypes.c_int64 * 13)(*R)
        C = (ctypes.c_double * (32 * 32))()
        E = (ctypes.c_double * 32)()
        valid = L.oracle_lpc_levinson_err(Ra, 12, C, E)
        ref = _py_levinson_err(R, 12)
        assert valid == len(ref) and list(E)[:valid] == ref  # bit-identical doubles
        for q in range(1, valid + 1):
            for n, bps in [(4096, 24), (1000, 17), (13, 32)]:
                assert L.oracle_lpc_order_key(ref[q - 1], q, n, bps) == _py_key(ref[q - 1], q, n, bps)
    assert L.oracle_lpc_order_key(0.0, 3, 4096, 16) == -1e300
    # the piecewise-linear log2 is exact at powers of two: key(2^10) = 10 n/2 + q (bps + 15)
    assert L.oracle_lpc_order_key(1024.0, 2, 4096, 16) == 10 * 2048 + 2 * 31


def test_lpc_selects_the_order_of_the_smallest_key():
    # the written LPC subframe of a predictable signal carries the key-selected order
    n = 4096
    t = np.arange(n)
    x = (2 ** 20 * np.sin(t * 1.3) + 2 ** 19 * np.sin(t * 2.1) + 3 * np.sin(t * 0.37)).astype(np.int64)
    planes = [np.ascontiguousarray(x).astype(np.int32)]
    _, rec = oracle_ref.encode_frame(planes, n, 0, 1, 24, 48000, lpc=8)
    sub = rec.written[0]
    assert sub.type == 3
    _, R = _py_autocorr(x, 8)
    errs = _py_levinson_err(R, 8)
    coefs = _py_levinson(R, 8)
    bps = 24 - sub.waste
    keys = [(_py_key(errs[q - 1], q, n, bps), q) for q in range(1, len(errs) + 1)
            if _py_quantize(coefs[q - 1]) is not None]
    assert sub.order == min(keys)[1]


def test_exhaustive_order_search_analysis_mode():
    """tools/lpc_ratio.py's analysis mode (oracle_set_lpc_exhaustive; NOT the contract the GPU
    implements): every order's Rice search, smallest total kept -- lossless, never larger than the
    contract's single order, and switched off again the default encode is the contract's."""
    import oracle_ref
    import synth

    L = oracle_ref.lib()
    pcm = synth.synth_pcm(4096 * 6 + 77, 2, 24, 96000, stream=9)
    base, _, _ = oracle_ref.encode_stream(pcm, 2, 24, 96000, lpc=8)
    L.oracle_set_lpc_exhaustive(1)
    try:
        exh, _, _ = oracle_ref.encode_stream(pcm, 2, 24, 96000, lpc=8)
    finally:
        L.oracle_set_lpc_exhaustive(0)
    assert len(exh) <= len(base)
    dec, _ = oracle_ref.decode_frames(exh, 2, 24, 96000, len(pcm) // 6)
    assert dec == pcm
    assert oracle_ref.encode_stream(pcm, 2, 24, 96000, lpc=8)[0] == base
