"""The product's wave64 cross-lane reductions (zig-flac_amd/csrc/fg_device.hpp row_* / wave_* /
wave_incl_scan32) against numpy, lane by lane, on adversarial lane patterns: one hot lane at each
of the 64 positions (not only the row heads 0/16/32/48 that the reductions read), all-equal,
alternating, ramps, INT_MAX / 0x80000000 / 0xFFFFFFFF edges and random words.

VERDICT r5 item 3: the FG_MAX ternary made wave_max32 return partial maxima (it re-read a DPP
source under a partial exec mask), which fed the LPC fast path's xmax bound while the parity suite
stayed green.  tests/hip/wave_ops.hip runs these helpers in a test-only module (never linked into
libflacgpu.so); its ternary build (libwaveops_ternary.so, the pre-fix macro) must FAIL here --
the proof that this test catches that bug."""
import ctypes
import os
import subprocess

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
HIPDIR = os.path.join(HERE, "hip")
M32, M64 = (1 << 32) - 1, (1 << 64) - 1


def patterns():
    """(n, 64) uint32 and uint64 lane patterns and their names."""
    rng = np.random.default_rng(20260821)
    p32, p64, names = [], [], []

    def add(name, a32, a64=None):
        a32 = np.asarray(a32, dtype=np.uint64) & M32
        if a64 is None:
            a64 = (a32.astype(np.uint64) << np.uint64(29)) | a32.astype(np.uint64)
        p32.append(a32.astype(np.uint32))
        p64.append(np.asarray(a64, dtype=np.uint64))
        names.append(name)

    for hot in range(64):
        for val, base in ((0xFFFFFFFF, 0), (1000, 0), (0x80000000, 0x7FFFFFFF), (7, 3), (0x7FFFFFFF, 0)):
            a = np.full(64, base, dtype=np.uint64)
            a[hot] = val
            a64 = np.full(64, base, dtype=np.uint64)
            a64[hot] = (val << 32) | val
            add(f"hot{hot}_{val:#x}_on_{base:#x}", a, a64)
        # one cold lane (the min idiom ~max(~x))
        a = np.full(64, 0xFFFFFFF0, dtype=np.uint64)
        a[hot] = 5
        add(f"cold{hot}", a)
    for v in (0, 1, 0x7FFFFFFF, 0x80000000, 0xFFFFFFFF):
        add(f"equal_{v:#x}", np.full(64, v, dtype=np.uint64), np.full(64, (v << 32) | v, dtype=np.uint64))
    add("alt_aa55", np.array([0xAAAAAAAA if i % 2 else 0x55555555 for i in range(64)], dtype=np.uint64))
    add("ramp", np.arange(64, dtype=np.uint64))
    add("ramp_down", np.arange(64, 0, -1, dtype=np.uint64))
    add("ramp_big", np.arange(64, dtype=np.uint64) * 0x04000001)
    for k in range(16):
        add(f"random{k}", rng.integers(0, 1 << 32, 64, dtype=np.uint64),
            rng.integers(0, 1 << 63, 64, dtype=np.uint64) * 2 + rng.integers(0, 2, 64, dtype=np.uint64))
    return np.stack(p32), np.stack(p64), names


def _build():
    subprocess.check_call(["make", "-s", "-C", HIPDIR])


def run(lib_name):
    _build()
    L = ctypes.CDLL(os.path.join(HIPDIR, "build", lib_name))
    p32, p64, names = patterns()
    n = len(names)
    U = L.wave_ops_uniform_words()
    uni = np.zeros((n, U), dtype=np.uint32)
    outs = [np.zeros((n, 64), dtype=np.uint32) for _ in range(4)]
    ptr = lambda a: a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
    rc = L.wave_ops_run(ptr(np.ascontiguousarray(p32)), ptr(np.ascontiguousarray(p64)), n, ptr(uni),
                        *[ptr(o) for o in outs])
    assert rc == 0, f"HIP error {rc}"
    return p32, p64, names, uni, outs


def mismatches(p32, p64, names, uni, outs):
    scan, rowmax, rowsum, maxfl = outs
    bad = []
    for i, name in enumerate(names):
        a = [int(x) for x in p32[i]]
        b = [int(x) for x in p64[i]]
        exp = {"sum32": sum(a) & M32, "sum64": sum(b) & M64, "or32": np.bitwise_or.reduce(p32[i]).item(),
               "or64": np.bitwise_or.reduce(p64[i]).item(), "max32": max(a), "min32": min(a),
               "xor32": np.bitwise_xor.reduce(p32[i]).item()}
        u = [int(x) for x in uni[i]]
        got = {"sum32": u[0], "sum64": u[1] | (u[2] << 32), "or32": u[3], "or64": u[4] | (u[5] << 32),
               "max32": u[6], "min32": u[7], "xor32": u[8]}
        for k in exp:
            if exp[k] != got[k]:
                bad.append(f"{name}: {k} {got[k]:#x} != {exp[k]:#x}")
        cs = np.cumsum(np.array(a, dtype=np.uint64)) & M32
        if not np.array_equal(scan[i].astype(np.uint64), cs):
            bad.append(f"{name}: incl_scan32")
        rows = np.array(a, dtype=np.uint64).reshape(4, 16)
        if not np.array_equal(rowmax[i].astype(np.uint64), np.repeat(rows.max(axis=1), 16)):
            bad.append(f"{name}: row_max32 lanes {np.nonzero(rowmax[i] != np.repeat(rows.max(axis=1), 16))[0][:8]}")
        if not np.array_equal(rowsum[i].astype(np.uint64), np.repeat(rows.sum(axis=1) & M32, 16)):
            bad.append(f"{name}: row_sum32")
        if not np.all(maxfl[i] == max(a)):
            bad.append(f"{name}: readfirstlane(wave_max32)")
    return bad


@pytest.mark.gpu
def test_wave_reductions_match_numpy_on_every_lane_pattern():
    bad = mismatches(*run("libwaveops.so"))
    assert not bad, "\n".join(bad[:40])


@pytest.mark.gpu
def test_ternary_fg_max_is_caught():
    """The pre-fix FG_MAX (a ternary that evaluates its DPP operand twice) must fail the test above
    on the single-hot-lane patterns: otherwise the test could not have caught the round-5 bug."""
    bad = mismatches(*run("libwaveops_ternary.so"))
    assert any("max" in b for b in bad), "the ternary FG_MAX passed: the test would not catch the bug"
    # and only the maximum (and the min idiom ~max(~x) built on it) is affected: sums / ORs / XORs /
    # scans are the same code in both builds
    other = [b for b in bad if "max" not in b and "min32" not in b]
    assert not other, "\n".join(other)[:2000]


def test_patterns_cover_every_lane_and_edge():
    """CPU: the pattern set puts a single hot (and cold) lane at every one of the 64 positions and
    carries the INT_MAX / 0x80000000 / 0xFFFFFFFF edges."""
    p32, p64, names = patterns()
    hot = {int(np.argmax(p32[i])) for i, nm in enumerate(names) if nm.startswith("hot") and "_on_0x0" in nm}
    assert hot == set(range(64))
    assert {0x7FFFFFFF, 0x80000000, 0xFFFFFFFF} <= set(int(x) for x in p32.reshape(-1))
    assert p32.shape[1] == 64 and p64.shape == p32.shape
