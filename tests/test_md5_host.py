"""The plan path's host MD5 engine (flacgpu_md5_many, include/flacgpu.h) against hashlib: the
digest the reference's Md5 wrapper (md5.zig:3-31) computes over the bytes wav_reader.zig:66
feeds it, finalised as encoder.zig:168-170.  Host-only calls: these run without a GPU."""
import hashlib
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "zig-flac_amd"))
import flacgpu  # noqa: E402


def _lib_or_skip():
    try:
        return flacgpu.load_library()
    except OSError as e:  # pragma: no cover - the build check covers the library itself
        pytest.skip(f"libflacgpu not built: {e}")


def _chunks(n, rng, sizes):
    return [rng.integers(0, 256, size=int(sizes[i]), dtype=np.uint8).tobytes() for i in range(n)]


@pytest.mark.parametrize("n", [1, 3, 8, 40])
def test_md5_many_fresh_matches_hashlib(n):
    _lib_or_skip()
    rng = np.random.default_rng(n)
    # empty, sub-block, one block +- 1, and pool-sized (>= 4 KiB: hashed on the pool workers)
    base = [0, 1, 55, 56, 63, 64, 65, 4095, 4096, 70000, 1 << 20]
    sizes = [base[i % len(base)] + (i // len(base)) * 3 for i in range(n)]
    chunks = _chunks(n, rng, sizes)
    got = flacgpu.md5_many(chunks)
    assert got == [hashlib.md5(c).digest() for c in chunks]


def test_md5_many_carried_segments_and_finished_rule():
    _lib_or_skip()
    rng = np.random.default_rng(7)
    n = 12
    segs = [[rng.integers(0, 256, size=64 * int(rng.integers(0, 300)), dtype=np.uint8).tobytes()
             for _ in range(3)] for _ in range(n)]
    tails = [rng.integers(0, 256, size=int(rng.integers(0, 9000)), dtype=np.uint8).tobytes() for _ in range(n)]
    states = (flacgpu.Md5State * n)()
    flacgpu.load_library().flacgpu_md5_state_init(states, n)
    for k in range(3):
        got = flacgpu.md5_many([segs[s][k] for s in range(n)], final=[False] * n, states=states)
        assert got == [None] * n
        assert all(states[s].bytes == sum(len(x) for x in segs[s][:k + 1]) for s in range(n))
    dig = flacgpu.md5_many(tails, final=[True] * n, states=states)
    want = [hashlib.md5(b"".join(segs[s]) + tails[s]).digest() for s in range(n)]
    assert dig == want
    assert all(states[s].finished == 1 for s in range(n))
    # finished: h is the digest (little-endian words), and later calls leave the state as it is
    assert bytes(states[0].h) == want[0]
    again = flacgpu.md5_many([b"x" * 64] * n, final=[True] * n, states=states)
    assert again == want
    flacgpu.md5_many([b"y" * 64] * n, final=[False] * n, states=states)
    assert bytes(states[3].h) == want[3] and states[3].finished == 1


def test_md5_many_rejects_partial_block_continuation():
    _lib_or_skip()
    states = (flacgpu.Md5State * 1)()
    flacgpu.load_library().flacgpu_md5_state_init(states, 1)
    with pytest.raises(flacgpu.FlacGpuError):
        flacgpu.md5_many([b"z" * 100], final=[False], states=states)
    with pytest.raises(flacgpu.FlacGpuError):
        flacgpu.md5_many([b"z" * 128], final=[False], states=None)  # nowhere to carry the chain


def test_md5_many_no_pool_matches(monkeypatch):
    """FLACGPU_MD5_THREADS=-1 (each chain on the caller) gives the same digests: run in a child so
    the pool's size is read afresh."""
    _lib_or_skip()
    import subprocess

    code = ("import sys, hashlib; sys.path.insert(0, %r); import flacgpu;"
            "c=[bytes([i]) * (5000 + 64 * i) for i in range(6)];"
            "assert flacgpu.md5_many(c) == [hashlib.md5(x).digest() for x in c]; print('ok')"
            % os.path.join(os.path.dirname(__file__), "..", "zig-flac_amd"))
    env = dict(os.environ, FLACGPU_MD5_THREADS="-1")
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and "ok" in r.stdout, r.stderr


def test_md5_many_more_chains_than_four_per_worker():
    """40 pool-sized messages of different lengths on 2 workers: each worker interleaves up to four
    chains (fg_md5_host.cpp kMaxChains) and, with chains waiting, yields them to the queue's tail
    after every chunk (time slicing), so every chain passes between workers many times; digests
    equal hashlib's.  In a child so the pool's size is read afresh."""
    _lib_or_skip()
    import subprocess

    code = ("import sys, hashlib; sys.path.insert(0, %r); import flacgpu;"
            "c=[bytes([i, 255 - i]) * (40000 + 4160 * i) for i in range(40)];"
            "assert flacgpu.md5_many(c) == [hashlib.md5(x).digest() for x in c]; print('ok')"
            % os.path.join(os.path.dirname(__file__), "..", "zig-flac_amd"))
    env = dict(os.environ, FLACGPU_MD5_THREADS="2")
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and "ok" in r.stdout, r.stderr


def _rates(host, workers, lane=72e6, chip=600e9):
    r = flacgpu.Md5Rates()
    for i, v in enumerate(host):
        r.host_chain[i] = v
    r.device_lane, r.device_chip, r.host_workers = lane, chip, workers
    return r


def test_md5_engine_picker_with_injected_rates():
    """flacgpu_md5_engine_for prices both engines with the rates it is given:
    the host pool's time = total / (k-chain rate x workers) (k = chains per worker, at most 4), the
    device's = max(longest chain / lane rate, total / chip rate).  CPU only."""
    _lib_or_skip()
    H, D = flacgpu.MD5_HOST, flacgpu.MD5_DEVICE
    try:
        flacgpu.set_md5_rates(_rates([1e9, 1.7e9, 2.2e9, 2.6e9], 16))
        per = 16 << 20
        # 8 long chains: host 8 workers x 1 GB/s (16 ms) vs one lane at 72 MB/s (233 ms)
        assert flacgpu.md5_engine_for(8, per, 8 * per) == H
        # 16384 chains of 256 KiB: host 4 GiB / (16 x 2.6 GB/s) = 103 ms; device max(3.6, 7.2) ms
        assert flacgpu.md5_engine_for(16384, 256 << 10, 16384 * (256 << 10)) == D
        # 256 chains of 16 MiB: host 4 GiB / 41.6 GB/s = 103 ms; device 233 ms -> host
        assert flacgpu.md5_engine_for(256, per, 256 * per) == H
        # ... but on a slow host (0.3 GB/s per chain) the device wins the same shape
        flacgpu.set_md5_rates(_rates([0.3e9, 0.5e9, 0.65e9, 0.78e9], 16))
        assert flacgpu.md5_engine_for(256, per, 256 * per) == D
        # no pool: chain after chain on the caller
        flacgpu.set_md5_rates(_rates([1e9, 1.7e9, 2.2e9, 2.6e9], 0))
        assert flacgpu.md5_engine_for(64, per, 64 * per) == D  # 1.07 s vs 0.23 s
        assert flacgpu.md5_engine_for(2, per, 2 * per) == H    # 34 ms vs 233 ms
        got = flacgpu.md5_rates()
        assert got.measured == 2 and got.host_workers == 0
        with pytest.raises(flacgpu.FlacGpuError):
            flacgpu.set_md5_rates(_rates([0.0, 1, 1, 1], 4))
    finally:
        flacgpu.set_md5_rates(None)  # measure again on next use


def test_md5_rates_measured_on_first_use():
    _lib_or_skip()
    flacgpu.set_md5_rates(None)
    r = flacgpu.md5_rates()
    assert r.measured == 1
    assert all(v > 1e7 for v in r.host_chain)  # any host hashes > 10 MB/s
    assert r.host_chain[3] > r.host_chain[0]  # interleaving four chains beats one on a core
    assert r.host_workers >= 0


@pytest.mark.parametrize("avx512", ["0", "1"])
def test_md5_many_vector_and_scalar_paths(avx512):
    """The pool's AVX-512 sixteen-chain path (compress_x16) and the scalar interleave give
    hashlib's digests for 1..70 chains of mixed lengths (partial blocks, empty chains) on 3 workers
    -- lane counts 1..16 and time slicing past 48 chains.  In a child: the path is chosen once."""
    _lib_or_skip()
    import subprocess

    code = ("import sys, hashlib, random; sys.path.insert(0, %r); import flacgpu; r = random.Random(5);"
            "ok = True\n"
            "for n in (1, 2, 5, 16, 17, 33, 70):\n"
            "    c = [bytes(r.getrandbits(8) for _ in range(r.choice([0, 63, 4096, 4160, 70000, 131072 + 7])))"
            " for _ in range(n)]\n"
            "    ok &= flacgpu.md5_many(c) == [hashlib.md5(x).digest() for x in c]\n"
            "print('ok' if ok else 'BAD')"
            % os.path.join(os.path.dirname(__file__), "..", "zig-flac_amd"))
    env = dict(os.environ, FLACGPU_MD5_THREADS="3", FLACGPU_MD5_AVX512=avx512)
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and r.stdout.strip().endswith("ok"), r.stdout + r.stderr


def _pool_workers(env, cpus=None):
    """host_workers of a fresh process (the pool is sized once per process), optionally pinned."""
    import subprocess

    code = ("import os, sys; sys.path.insert(0, %r)\n" % os.path.join(ROOT, "zig-flac_amd") +
            (f"os.sched_setaffinity(0, {set(cpus)!r})\n" if cpus else "") +
            "import flacgpu; print(flacgpu.md5_rates().host_workers)")
    e = {k: v for k, v in os.environ.items() if k not in ("FLACGPU_MD5_THREADS", "LOCAL_WORLD_SIZE")}
    e.update(env)
    r = subprocess.run([sys.executable, "-c", code], env=e, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    return int(r.stdout.strip().splitlines()[-1])


def _quota_cpus():
    try:
        q, period = open("/sys/fs/cgroup/cpu.max").read().split()
        return 0 if q == "max" else -(-int(q) // int(period))
    except (OSError, ValueError):
        return 0


@pytest.mark.skipif(len(os.sched_getaffinity(0)) < 2, reason="needs two CPUs")
def test_pool_share_respects_a_rank_bound_mask():
    """a process already bound to its share of the CPUs (numactl, SLURM
    --cpu-bind, a per-rank cgroup) keeps that whole share as its MD5 pool even when the launcher sets
    LOCAL_WORLD_SIZE; only a process that sees every online CPU divides by LOCAL_WORLD_SIZE."""
    mine = sorted(os.sched_getaffinity(0))[:2]
    quota = _quota_cpus()
    assert _pool_workers({"LOCAL_WORLD_SIZE": "8"}, cpus=mine) == (min(quota, 2) if 0 < quota < 2 else 2)
    aff = len(os.sched_getaffinity(0))
    online = os.cpu_count()
    whole = quota <= 0 and aff >= online
    base = quota if 0 < quota < aff else aff
    expect = max(1, base // 8) if whole else base
    assert _pool_workers({"LOCAL_WORLD_SIZE": "8"}) == min(expect, 64)
    assert _pool_workers({}) == min(base, 64)
