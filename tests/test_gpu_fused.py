"""The fused single-pass encode (FLACGPU_FUSED=1: k_analyze<..., FP> + fg_fused.hpp) against the CPU
restatement, byte for byte.

Full 16-bit stereo frames are analysed and packed by one kernel; each frame's byte offset comes from
an in-kernel look-back over per-slot status words (tail frames publish theirs from the tail analysis
launched first).  Covered: ragged streams with tails at every 4-byte alignment, repeated calls (the
status words and the frame queue are reset per call), plans of thousands of frames (look-back
windows of 64 slots, many windows deep), both MD5 schedules, carried MD5 state over several calls,
decision records equal to the split encode's, an output buffer too small (device error word), and
the file path (flacgpu_encode_frames).  The full GPU suite can also run with FLACGPU_FUSED=1.
"""
import hashlib

import numpy as np
import pytest

import oracle_ref
import synth
from test_gpu_plan import LENGTHS, _encoder, _layout, _run_plan

pytestmark = pytest.mark.gpu

CH, BITS, RATE = 2, 16, 44100


@pytest.fixture(autouse=True)
def _diag_only(diag_build):
    """The fused kernel ships in diagnostic builds only."""


@pytest.fixture
def fused(monkeypatch):
    monkeypatch.setenv("FLACGPU_FUSED", "1")


def _streams(lengths, aligns, seed0=0):
    offs, size = _layout(lengths, 4, aligns)
    buf = bytearray(size)
    pcms = []
    for s, n in enumerate(lengths):
        pcm = synth.synth_pcm(n, CH, BITS, RATE, stream=seed0 + s) if n else b""
        buf[offs[s]:offs[s] + len(pcm)] = pcm
        pcms.append(pcm)
    return offs, bytes(buf), pcms


@pytest.mark.parametrize("aligns", [(0,), (4, 8, 12, 0)])
def test_fused_streams_match_oracle(fused, aligns):
    offs, buf, pcms = _streams(LENGTHS, aligns, 500)
    with _encoder(CH, BITS, RATE) as enc:
        for md5 in ("join", "state", "join"):  # repeated calls reuse the status words and the queue
            res, _ = _run_plan(enc, buf, offs, LENGTHS, md5=md5)
            for s, (got, sizes, dig) in enumerate(res):
                ref, ref_sizes, ref_md5 = oracle_ref.encode_stream(pcms[s], CH, BITS, RATE)
                assert sizes == ref_sizes, f"stream {s}: frame sizes differ"
                assert got == ref, f"stream {s}: bytes differ"
                if md5 == "join":
                    assert dig == ref_md5 == hashlib.md5(pcms[s]).digest(), f"stream {s}: MD5"


@pytest.mark.parametrize("tail", [0, 777])
def test_fused_many_frames(fused, tail):
    """~2900 frames in one call: the look-back runs many 64-slot windows deep."""
    lengths = [4096 * 45 + tail] * 64
    offs, buf, pcms = _streams(lengths, (0, 8), 700)
    refs = [oracle_ref.encode_stream(p, CH, BITS, RATE)[:2] for p in pcms]
    with _encoder(CH, BITS, RATE, max_frames=4096) as enc:
        res, _ = _run_plan(enc, buf, offs, lengths, md5="none")
    for s, (got, sizes, _) in enumerate(res):
        assert (got, sizes) == (refs[s][0], refs[s][1]), f"stream {s}"


def test_fused_records_equal_split(monkeypatch):
    """Decision records of the fused kernel equal the split encode's (same analysis code)."""
    pcm = synth.synth_pcm(4096 * 40 + 1000, CH, BITS, RATE, stream=9)
    recs = {}
    for mode in ("0", "1"):
        monkeypatch.setenv("FLACGPU_FUSED", mode)
        with _encoder(CH, BITS, RATE, max_frames=64) as enc:
            enc.set_records(True)
            out, sizes = enc.encode_frames(pcm, first_frame=0)
            recs[mode] = (out, list(sizes), [bytes(r) for r in enc.records()])
    assert recs["0"][0] == recs["1"][0]
    assert recs["0"][1] == recs["1"][1]
    assert len(recs["1"][2]) > 0 and recs["0"][2] == recs["1"][2]


def test_fused_file_path_matches_oracle(fused):
    pcm = synth.synth_pcm(4096 * 300 + 1234, CH, BITS, RATE, stream=11)
    ref, ref_sizes, _ = oracle_ref.encode_stream(pcm, CH, BITS, RATE)
    with _encoder(CH, BITS, RATE, max_frames=128) as enc:  # pipelined chunks of the file path
        out, sizes = enc.encode_frames(pcm, first_frame=0)
    assert list(sizes) == ref_sizes
    assert out == ref


def test_fused_output_too_small_is_an_error(fused):
    import flacgpu

    lengths = [4096 * 8] * 6
    offs, buf, _ = _streams(lengths, (0,), 900)
    with _encoder(CH, BITS, RATE) as enc:
        with pytest.raises(flacgpu.FlacGpuError):
            _run_plan(enc, buf, offs, lengths, md5="none", out_cap=4096)
        # the context stays usable and the next call is exact
        res, _ = _run_plan(enc, buf, offs, lengths, md5="none")
        assert len(res) == len(lengths)
