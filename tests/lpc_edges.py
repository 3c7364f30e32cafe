"""Frames that sit on the GPU LPC fast path's bound (fg_device.hpp k_analyze step 8b).

The kernel takes the 32-bit-only residual pass when
    xmax + ((csum * xmax) >> shift) + 1 < 3 * 2^30                       (*)
where xmax = max |x| over the wave's 64 lanes (wave_max32), csum = sum |c_t| of the selected
order's quantised coefficients.  (*) bounds |e| = |x - P| below 3 * 2^30, so the low word of e
identifies it.  A wrong xmax (the round-5 FG_MAX bug returned a partial maximum: only the row
heads 0/16/32/48 survived) lets a residual of |e| >= 3 * 2^30 wrap into [-2^30, 2^30) and the
frame is encoded wrongly.  These fixtures (test infrastructure; the order selection below is the
restatement's lpc_search, oracle/flac_oracle.c:606-633, through its exported steps):

  hot_lane_frame -- mono, i32 samples: a 0.9*pi sinusoid everywhere, small except in the 64
                    samples of ONE lane (full scale), one of them sign-flipped.  The true xmax
                    fails (*) (slow path; the flipped residual is unusable, no LPC); a maximum
                    that misses the hot lane passes (*), and the flipped residual wraps into
                    range: a kernel with that bug writes a different (wrong) subframe.
  threshold_frame -- the same sinusoid, no flip, scaled so that (*)'s left side is exactly
                    3 * 2^30 - 1 (fast path) or 3 * 2^30 (slow path): the boundary itself.
"""
from __future__ import annotations

import ctypes

import numpy as np

import oracle_ref

LPC_MAX = 32  # ORACLE_LPC_MAX_ORDER
LPC_PREC = 15  # ORACLE_LPC_PRECISION
LIMIT = 3 << 30


def lpc_select(x: np.ndarray, Q: int, bps: int):
    """The restatement's order selection (contract steps 1-7) for plane x -> (q, coefs, shift) or None."""
    L = oracle_ref.lib()
    L.oracle_lpc_order_key.restype = ctypes.c_double
    L.oracle_lpc_order_key.argtypes = [ctypes.c_double, ctypes.c_uint, ctypes.c_uint32, ctypes.c_uint]
    x = np.ascontiguousarray(x, dtype=np.int64)
    n = len(x)
    R = (ctypes.c_int64 * (Q + 1))()
    L.oracle_lpc_autocorr(x.ctypes.data_as(ctypes.c_void_p), n, Q, R)
    coefs = (ctypes.c_double * (LPC_MAX * LPC_MAX))()
    errs = (ctypes.c_double * LPC_MAX)()
    valid = L.oracle_lpc_levinson_err(R, Q, coefs, errs)
    best = None
    for q in range(1, valid + 1):
        c = (ctypes.c_int32 * LPC_MAX)()
        sh = ctypes.c_int(0)
        a = ctypes.cast(ctypes.byref(coefs, (q - 1) * LPC_MAX * 8), ctypes.POINTER(ctypes.c_double))
        if L.oracle_lpc_quantize(a, q, LPC_PREC, c, ctypes.byref(sh)):
            continue
        key = L.oracle_lpc_order_key(errs[q - 1], q, n, bps)
        if best is None or key < best[0]:
            best = (key, q, list(c)[:q], sh.value)
    return None if best is None else best[1:]


def bound(xmax: int, coefs, shift: int) -> int:
    csum = sum(abs(int(v)) for v in coefs)
    return xmax + ((csum * xmax) >> shift) + 1


def _sinusoid(n: int, amp: float, seed: int) -> np.ndarray:
    rng = np.random.default_rng(seed)
    t = np.arange(n)
    x = np.round(amp * np.cos(0.9 * np.pi * t)).astype(np.int64)
    return x + rng.integers(-1, 2, n)  # +-1 noise: odd samples, so no wasted bits


def hot_lane_frame(Q: int = 12, start_lane: int = 49, n: int = 4096, small: float = 2 ** 10, seed: int = 7):
    """(samples int64[n], info): a 0.9*pi sinusoid whose envelope rises smoothly (log-linear)
    from `small` at lane `start_lane` to full 32-bit scale at the frame's LAST sample, which is
    then sign-flipped.  The maximum |x| sits in lane 63 (never a row head); lanes 0/16/32/48 hold
    only small samples.  The flip is the last sample, so no later residual uses it: its residual
    (about 2 x 2^31) is the only large one."""
    t = np.arange(n)
    s0 = 64 * start_lane
    env = np.full(n, small)
    u = np.clip((t - s0) / (n - 1 - s0), 0.0, 1.0)
    peak = 2 ** 31 - 2
    env = np.where(t >= s0, small * (peak / small) ** u, env)
    rng = np.random.default_rng(seed)
    x = np.round(env * np.cos(0.9 * np.pi * (t - (n - 1)))).astype(np.int64)
    x[t < s0] += rng.integers(-1, 2, int((t < s0).sum()))  # odd samples: no wasted bits
    x = np.clip(x, -(2 ** 31) + 1, 2 ** 31 - 1)
    x[n - 1] = -x[n - 1]
    return x, {"flip": n - 1, "hot_lanes": list(range(start_lane, 64))}


def hot_lane_properties(x: np.ndarray, Q: int, bits: int = 32):
    """What makes the fixture bite: the true bound fails (*), the bound over the row-head lanes
    0/16/32/48 alone (what the pre-fix wave_max32 returned) passes it, and every residual of the
    selected order lies in [-2^30, 2^30) after wrapping to 32 bits, while the flipped one does not
    before wrapping -> dict."""
    sel = lpc_select(x, Q, bits)
    assert sel is not None
    q, c, sh = sel
    lanes = np.abs(x).reshape(64, -1)
    xmax = int(lanes.max())
    heads = int(lanes[[0, 16, 32, 48]].max())
    e = []
    for i in range(q, len(x)):
        acc = sum(int(c[t]) * int(x[i - 1 - t]) for t in range(q))
        e.append(int(x[i]) - (acc >> sh))
    big = [v for v in e if not -(1 << 30) <= v < (1 << 30)]
    wrapped = [((v + (1 << 31)) % (1 << 32)) - (1 << 31) for v in e]
    return {"q": q, "shift": sh, "true_bound": bound(xmax, c, sh), "head_bound": bound(heads, c, sh),
            "big_residuals": big, "all_wrapped_in_range": all(-(1 << 30) <= w < (1 << 30) for w in wrapped),
            "max_lane": int(np.argmax(lanes.max(axis=1)))}


def threshold_frame(side: str, Q: int, n: int = 4096, bits: int = 32):
    """(samples, info) on either side of (*) for the order the restatement selects: "fast" = the
    largest peak whose bound is < 3 * 2^30 (fixed-point iteration: the quantised coefficients stop
    moving with the amplitude); "slow" = the same frame with its peak sample raised until the bound
    of the coefficients selected for THAT frame reaches 3 * 2^30 (in practice +1)."""
    t = np.arange(n)
    amp = LIMIT / 4.0
    x = None
    for _ in range(12):
        peak = int(round(amp))
        x = np.round(peak * np.cos(0.9 * np.pi * t)).astype(np.int64)
        x[1::7] += np.sign(x[1::7])  # odd samples: no wasted bits
        x = np.clip(x, -peak, peak)
        x[0] = peak  # |x| max exactly at sample 0 (cos 0 = 1)
        q, c, sh = lpc_select(x, Q, bits)
        lo, hi = 1, 2 ** 31 - 1  # the largest xmax with bound(xmax) < LIMIT
        while lo < hi:
            mid = (lo + hi + 1) // 2
            if bound(mid, c, sh) < LIMIT:
                lo = mid
            else:
                hi = mid - 1
        if lo == peak:
            break
        amp = float(lo)
    else:
        raise RuntimeError("threshold fixture did not converge")
    if side == "slow":
        for _ in range(64):
            x = x.copy()
            x[0] += 1
            q, c, sh = lpc_select(x, Q, bits)
            if bound(int(x[0]), c, sh) >= LIMIT:
                break
        else:
            raise RuntimeError("slow-side fixture not found")
    xm = int(np.abs(x).max())
    return x, {"q": q, "coefs": c, "shift": sh, "xmax": xm, "bound": bound(xm, c, sh)}
