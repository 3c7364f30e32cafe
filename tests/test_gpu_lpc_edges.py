"""The GPU LPC fast path's bound (fg_device.hpp k_analyze step 8b) at its edges, against the CPU
restatement (oracle/flac_oracle.c lpc_search, the build-defined LPC contract, :447-475).

VERDICT r5 item 3: a wrong wave maximum (the pre-fix FG_MAX) fed the fast path's xmax while the
suite stayed green.  tests/lpc_edges.py builds frames where that bug changes the bytes (the
maximum |x| in lane 63 only, a last-sample residual of about -2^32 that wraps into range) and
frames on both sides of the bound itself; here the GPU's bytes and per-candidate decision records
must equal the restatement's.  The fixtures' properties are checked on the CPU (no GPU mark)."""
import numpy as np
import pytest

import lpc_edges as E
import oracle_ref
import synth


def _pcm(x, ch, bits):
    cols = [x] * ch
    return synth.to_pcm_bytes(np.stack(cols, axis=1), bits)


def _frames(x, pad_frames=2, seed=3):
    """The edge frame followed by ordinary synthetic frames (so the kernel's persistent loop runs
    the edge frame beside others)."""
    rest = synth.synth_samples(pad_frames * 4096, 1, 32, 48000, stream=seed)[:, 0].astype(np.int64)
    return np.concatenate([x, rest])


def _check(x, ch, bits, rate, q):
    import flacgpu

    pcm = _pcm(x, ch, bits)
    n = len(x)
    enc = flacgpu.Encoder(ch, bits, rate, max_frames=64, lpc_order=q)
    try:
        enc.set_records(True)
        got, sizes = enc.encode_frames(pcm)
        recs = enc.records()
    finally:
        enc.close()
    ref, ref_sizes, _ = oracle_ref.encode_stream(pcm, ch, bits, rate, lpc=q)
    assert sizes == ref_sizes, "frame sizes differ from the restatement"
    assert got == ref, "bytes differ from the restatement"
    samples = synth.from_pcm_bytes(pcm, ch, bits)
    for f, rec in enumerate(recs):
        planes = [np.ascontiguousarray(samples[f * 4096:(f + 1) * 4096, c]).astype(np.int32) for c in range(ch)]
        _, orec = oracle_ref.encode_frame(planes, len(planes[0]), f, ch, bits, rate, lpc=q)
        assert rec.channel_code == orec.channel_code
        for c in range(orec.n_cand):
            g, o = rec.cand[c], orec.cand[c]
            assert (g.type, g.waste, g.estimate) == (o.type, o.waste, o.estimate), f"frame {f} cand {c}"
            if o.type >= 2:
                assert (g.order, g.part_order, g.method) == (o.order, o.part_order, o.method)
            if o.type == 3:
                assert (g.lpc_shift, list(g.lpc_coefs)[:o.order]) == (o.lpc_shift, list(o.lpc_coefs)[:o.order])
    dec, _ = oracle_ref.decode_frames(got, ch, bits, rate, n)
    assert dec == pcm
    return recs


HOT = [(q, s) for q in (8, 12) for s in (49, 40, 20)]


@pytest.mark.parametrize("q,start", HOT)
def test_hot_lane_fixture_bites(q, start):
    """CPU: the fixture would expose a partial maximum -- the true bound fails the fast-path test,
    the row heads' bound passes it, and the one large residual wraps into [-2^30, 2^30)."""
    x, _ = E.hot_lane_frame(q, start)
    p = E.hot_lane_properties(x, q)
    assert p["max_lane"] == 63
    assert p["true_bound"] >= E.LIMIT > p["head_bound"]
    assert len(p["big_residuals"]) == 1 and p["all_wrapped_in_range"]


@pytest.mark.parametrize("q", [8, 12])
def test_threshold_fixtures_straddle_the_bound(q):
    """CPU: the fast / slow fixtures sit on either side of 3 * 2^30 for the order the restatement
    selects, with the coefficients it selects for each."""
    _, f = E.threshold_frame("fast", q)
    _, s = E.threshold_frame("slow", q)
    assert f["bound"] < E.LIMIT <= s["bound"] and s["xmax"] == f["xmax"] + 1 and f["q"] == s["q"]


@pytest.mark.gpu
@pytest.mark.parametrize("q,start", HOT)
@pytest.mark.parametrize("ch", [1, 2])
def test_gpu_lpc_hot_lane_32bit(q, start, ch):
    x, _ = E.hot_lane_frame(q, start)
    recs = _check(_frames(x), ch, 32, 192000, q)
    # the edge frame: the restatement finds the flipped residual unusable, so no LPC subframe there
    assert all(recs[0].cand[c].type != 3 for c in range(recs[0].n_cand))


@pytest.mark.gpu
@pytest.mark.parametrize("q", [8, 12])
def test_gpu_lpc_hot_lane_24bit(q):
    """The same shape at 24-bit full scale (the fast path is always valid there; parity only)."""
    x, _ = E.hot_lane_frame(q, 40, small=2 ** 4)
    x = np.clip(x >> 8, -(2 ** 23) + 1, 2 ** 23 - 1)
    _check(np.concatenate([x, x[::-1]]), 2, 24, 96000, q)


@pytest.mark.gpu
@pytest.mark.parametrize("q", [8, 12])
@pytest.mark.parametrize("side", ["fast", "slow"])
def test_gpu_lpc_fast_path_threshold(q, side):
    x, info = E.threshold_frame(side, q)
    recs = _check(x, 1, 32, 192000, q)
    assert recs[0].cand[0].type == 3 and recs[0].cand[0].order == info["q"]  # LPC wins on a pure sinusoid
