"""GPU (libflacgpu.so on gfx950) vs the CPU restatement: bit-exact frames.

Every test calls through the C ABI and compares with oracle/ on the same
seeded input: whole-stream bytes, per-frame sizes, per-candidate decision
records, and a round trip through the independent verifier decoder.
"""
import hashlib

import numpy as np
import pytest

import oracle_ref
import synth

pytestmark = pytest.mark.gpu

CONFIGS = [
    # channels, bits, rate
    (2, 16, 44100),
    (2, 24, 96000),
    (2, 32, 192000),
    (1, 16, 44100),
    (8, 24, 96000),
    (3, 16, 48000),
    (2, 8, 8000),
    (1, 24, 96000),
    (1, 32, 48000),
    (8, 32, 192000),  # the largest frame the reference accepts: 8 x 4096 x 4 B
    (7, 16, 44100),
    (6, 32, 96000),   # channel-split analysis (halves of three 32-bit channels)
    (4, 24, 48000),   # a 6-byte half row: no split
]

_encoders = {}


def gpu_encoder(ch, bits, rate, **kw):
    import flacgpu

    key = (ch, bits, rate, tuple(sorted(kw.items())))
    if key not in _encoders:
        _encoders[key] = flacgpu.Encoder(ch, bits, rate, max_frames=1024, **kw)
    return _encoders[key]


def _diff_msg(a: bytes, b: bytes) -> str:
    n = min(len(a), len(b))
    for i in range(n):
        if a[i] != b[i]:
            return f"len gpu={len(a)} oracle={len(b)}; first diff at byte {i}: {a[i]:#x} vs {b[i]:#x}"
    return f"len gpu={len(a)} oracle={len(b)} (prefix equal)"


def check_stream(ch, bits, rate, n, stream=0, first_frame=0, specials=True, decodable=True, **kw):
    pcm = synth.synth_pcm(n, ch, bits, rate, stream=stream, specials=specials)
    enc = gpu_encoder(ch, bits, rate, **kw)
    okw = {}
    if "stereo_decorrelation" in kw:
        okw["stereo"] = kw["stereo_decorrelation"]
    if "max_rice_part_order" in kw:
        okw["part_order"] = kw["max_rice_part_order"]
    if "max_rice_param" in kw:
        okw["param"] = kw["max_rice_param"]
    if "lpc_order" in kw:
        okw["lpc"] = kw["lpc_order"]
    block = kw.get("block_size", 4096)
    ref, ref_sizes, ref_md5 = oracle_ref.encode_stream(pcm, ch, bits, rate, block=block, first_frame=first_frame,
                                                       **okw)
    got, sizes = enc.encode_frames(pcm, first_frame=first_frame)
    assert sizes == ref_sizes, "per-frame sizes differ"
    assert got == ref, _diff_msg(got, ref)
    if decodable:
        dec, _ = oracle_ref.decode_frames(got, ch, bits, rate, n, first_number=first_frame)
        assert dec == pcm
    return pcm, got


@pytest.mark.parametrize("ch,bits,rate", CONFIGS)
def test_stream_parity(ch, bits, rate):
    # 130 full blocks (includes the special blocks at 63 and 127) + a short tail
    check_stream(ch, bits, rate, 4096 * 130 + 1000)


@pytest.mark.parametrize("tail", [1, 2, 4, 5, 8, 16, 24, 64, 192, 255, 256, 512, 576, 1000, 1152, 2048, 4095])
def test_tail_lengths(tail):
    check_stream(2, 16, 44100, 4096 * 2 + tail, stream=tail)


@pytest.mark.parametrize("ch,bits", [(1, 16), (2, 24), (2, 32), (8, 24)])
@pytest.mark.parametrize("tail", [3, 17, 100, 333, 4000])
def test_tail_lengths_other(ch, bits, tail):
    check_stream(ch, bits, 48000, 4096 + tail, stream=tail)


@pytest.mark.parametrize("first", [0, 127, 128, 2047, 2048, 65535, 65536, (1 << 21) - 1, 1 << 21, (1 << 31),
                                   (1 << 36) - 4])
def test_frame_numbers(first):
    # UTF-8 coded frame numbers of every width (frame_writer.zig:235-251)
    check_stream(2, 16, 44100, 4096 * 3 + 10, first_frame=first)


@pytest.mark.parametrize("rate", [44100, 48000, 96000, 192000, 88200, 176400, 8000, 16000, 22050, 24000, 32000,
                                  11025, 37800, 200, 352800])
def test_sample_rates(rate):
    # includes the uncommon-rate header quirk (frame_writer.zig:258-262): for rates <= 255 the
    # reference ORs the (unmasked) block size into an 8-bit field, so its frames are not
    # decodable FLAC; parity is byte equality with the reference behaviour there.
    check_stream(2, 16, rate, 4096 + 300, decodable=rate > 255)


def test_stereo_off():
    check_stream(2, 16, 44100, 4096 * 65 + 7, stereo_decorrelation=False)


@pytest.mark.parametrize("po,pm", [(0, 30), (4, 30), (8, 14), (8, 5), (2, 1)])
def test_rice_caps(po, pm):
    check_stream(2, 24, 96000, 4096 * 3 + 77, max_rice_part_order=po, max_rice_param=pm)


def test_block_size_1152():
    check_stream(2, 16, 44100, 1152 * 40 + 5, block_size=1152)


def _records_match(ch, bits, rate, n, stream=0, lpc=0):
    pcm = synth.synth_pcm(n, ch, bits, rate, stream=stream)
    enc = gpu_encoder(ch, bits, rate, **({"lpc_order": lpc} if lpc else {}))
    enc.set_records(True)
    try:
        got, sizes = enc.encode_frames(pcm)
        recs = enc.records()
    finally:
        enc.set_records(False)
    B = bits // 8
    samples = synth.from_pcm_bytes(pcm, ch, bits)
    bs = 4096
    for f, rec in enumerate(recs):
        planes = [np.ascontiguousarray(samples[f * bs:(f + 1) * bs, c]).astype(np.int32) for c in range(ch)]
        nn = len(planes[0])
        ref_bytes, orec = oracle_ref.encode_frame(planes, nn, f, ch, bits, rate, lpc=lpc)
        assert rec.channel_code == orec.channel_code, f"frame {f} channel code"
        for c in range(orec.n_cand):
            g, o = rec.cand[c], orec.cand[c]
            ctx = f"frame {f} cand {c}"
            assert (g.type, g.waste, g.bits) == (o.type, o.waste, o.bits), ctx
            assert g.estimate == o.estimate, ctx + f" estimate {g.estimate} vs {o.estimate}"
            if o.type >= 2:
                assert (g.order, g.part_order, g.method) == (o.order, o.part_order, o.method), ctx
                np_ = 1 << o.part_order
                assert list(g.params)[:np_] == list(o.params)[:np_], ctx
            if o.type == 3:
                assert (g.lpc_precision, g.lpc_shift) == (o.lpc_precision, o.lpc_shift), ctx
                assert list(g.lpc_coefs)[:o.order] == list(o.lpc_coefs)[:o.order], ctx
            if o.type == 0:
                assert g.constant == o.constant, ctx
    return got


# (8, 24) and (8, 32): full frames analysed in channel halves (two workgroups per frame)
@pytest.mark.parametrize("ch,bits,rate", [(2, 16, 44100), (2, 24, 96000), (2, 32, 192000), (3, 16, 48000),
                                         (8, 24, 96000), (8, 32, 192000)])
def test_decision_records(ch, bits, rate):
    _records_match(ch, bits, rate, 4096 * 66 + 513)


def test_md5_matches_hashlib():
    enc = gpu_encoder(2, 16, 44100)
    for n in [0, 1, 55, 56, 63, 64, 65, 119, 120, 128, 1000, 65536 + 17]:
        data = np.random.default_rng(n).integers(0, 256, size=n, dtype=np.uint8).tobytes()
        assert enc.md5(data) == hashlib.md5(data).digest(), n
    # streaming updates in odd pieces
    data = synth.synth_pcm(50000, 2, 16, 44100)
    enc.lib.flacgpu_md5_init(enc.ctx)
    pos = 0
    for step in [1, 63, 64, 65, 1000, 4096 * 4]:
        enc.md5_update(data[pos:pos + step])
        pos += step
    enc.md5_update(data[pos:])
    assert enc.md5_final() == hashlib.md5(data).digest()


def test_write_frame_planar():
    ch, bits, rate = 2, 16, 44100
    enc = gpu_encoder(ch, bits, rate)
    s = synth.synth_samples(4096 * 3, ch, bits, rate, stream=9)
    for f, n in [(0, 4096), (1, 4096), (7, 1000), (300, 5), (2, 1)]:
        planes = [np.ascontiguousarray(s[f % 2 * 4096:f % 2 * 4096 + n, c]).astype(np.int32) for c in range(ch)]
        got = enc.write_frame(np.stack(planes), f)
        ref, _ = oracle_ref.encode_frame(planes, n, f, ch, bits, rate)
        assert got == ref, (f, n, _diff_msg(got, ref))


@pytest.mark.parametrize("stereo", [True, False])
def test_pack4_matches_general_pack(monkeypatch, stereo):
    """Full 16-bit two-channel frames go through k_pack4 (four waves per subframe); the
    general one-wave-per-subframe k_pack (FLACGPU_PACK4=0) must emit the same bytes."""
    import flacgpu

    n = 4096 * 48 + 77  # full frames (incl. the special blocks) and a short tail
    pcm = synth.synth_pcm(n, 2, 16, 44100, stream=5)
    outs = []
    for knob in ("1", "0"):
        monkeypatch.setenv("FLACGPU_PACK4", knob)
        with flacgpu.Encoder(2, 16, 44100, max_frames=64, stereo_decorrelation=stereo) as enc:
            outs.append(enc.encode_frames(pcm))
    assert outs[0][1] == outs[1][1], "frame sizes differ between k_pack4 and k_pack"
    assert outs[0][0] == outs[1][0], _diff_msg(outs[0][0], outs[1][0])
    ref, ref_sizes, _ = oracle_ref.encode_stream(pcm, 2, 16, 44100, stereo=stereo)
    assert outs[0][0] == ref, _diff_msg(outs[0][0], ref)


@pytest.mark.parametrize("ch,bits,rate", [(8, 24, 96000), (8, 16, 44100), (6, 32, 96000), (8, 32, 192000)])
def test_pack_split_matches_whole_frame(monkeypatch, ch, bits, rate):
    """Frames analysed in channel halves are also packed in channel halves (k_packw split mode:
    two workgroups per frame, CRC-16 joined as CRC(img0) z^(8 (Lb - e0)) ^ CRC(img1), the byte
    both halves share merged by the second to arrive); the whole-frame k_packw
    (FLACGPU_PACK_SPLIT=0) and the restatement must see the same bytes -- including the
    special blocks (all-zero, full-scale noise: the shared byte at every bit offset) and a tail."""
    import flacgpu

    n = 4096 * 40 + 333
    pcm = synth.synth_pcm(n, ch, bits, rate, stream=9)
    outs = []
    for knob in ("1", "0"):
        monkeypatch.setenv("FLACGPU_PACK_SPLIT", knob)
        with flacgpu.Encoder(ch, bits, rate, max_frames=24) as enc:
            outs.append(enc.encode_frames(pcm))
    assert outs[0][1] == outs[1][1], "frame sizes differ between the split and whole-frame pack"
    assert outs[0][0] == outs[1][0], _diff_msg(outs[0][0], outs[1][0])
    ref, ref_sizes, _ = oracle_ref.encode_stream(pcm, ch, bits, rate)
    assert outs[0][1] == ref_sizes and outs[0][0] == ref, _diff_msg(outs[0][0], ref)


@pytest.mark.parametrize("knobs", [{"FLACGPU_SPLIT_JIT": "3"}, {"FLACGPU_SPLIT_JIT": "0"},
                                   {"FLACGPU_SPLIT_JIT": "1", "FLACGPU_PACK_XCDQ": "0"},
                                   {"FLACGPU_XCD_QUEUE": "0", "FLACGPU_PACK_XCDQ": "0"}])
def test_split_item_schedules_match_oracle(monkeypatch, knobs):
    """The channel-half items of the split analysis and pack (c4) taken just in time from the
    per-XCD queues (FLACGPU_SPLIT_JIT bit 0 analysis, bit 1 pack), or ahead from them, or from
    one global ticket: the schedule only moves work between workgroups, the bytes are the
    restatement's."""
    import flacgpu

    ch, bits, rate = 8, 24, 96000
    n = 4096 * 300 + 333  # enough items that every XCD queue runs dry and hands over
    pcm = synth.synth_pcm(n, ch, bits, rate, stream=12)
    for k, v in knobs.items():
        monkeypatch.setenv(k, v)
    with flacgpu.Encoder(ch, bits, rate, max_frames=512) as enc:
        out, sizes = enc.encode_frames(pcm)
    ref, ref_sizes, _ = oracle_ref.encode_stream(pcm, ch, bits, rate)
    assert sizes == ref_sizes and out == ref, _diff_msg(out, ref)


@pytest.mark.parametrize("cfg,max_frames,n", [
    ((2, 16, 44100), 8, 4096 * 37 + 1001),   # 4-frame chunks: 10 chunks, both halves reused 5x, a tail
    ((2, 24, 96000), 6, 4096 * 13),          # 3-frame chunks, no tail
    ((1, 16, 44100), 2, 4096 * 5 + 3),       # 1-frame chunks
])
def test_host_pipeline_matches_sequential(cfg, max_frames, n):
    """flacgpu_encode_frames overlaps chunk i+1's upload and encode with chunk i's download
    (two halves of the context's buffers, a download thread) once an input spans more than
    one chunk; bytes and frame sizes must equal a single-chunk encode and the oracle."""
    import flacgpu

    ch, bits, rate = cfg
    pcm = synth.synth_pcm(n, ch, bits, rate, stream=11)
    with flacgpu.Encoder(ch, bits, rate, max_frames=max_frames) as enc:
        got, sizes = enc.encode_frames(pcm, first_frame=3)
        again, sizes2 = enc.encode_frames(pcm, first_frame=3)  # context reuse: halves and events recycled
    with flacgpu.Encoder(ch, bits, rate, max_frames=1024) as enc:
        seq, seq_sizes = enc.encode_frames(pcm, first_frame=3)
    assert sizes == seq_sizes and sizes2 == seq_sizes
    assert got == seq, _diff_msg(got, seq)
    assert again == seq
    ref, ref_sizes, _ = oracle_ref.encode_stream(pcm, ch, bits, rate, first_frame=3)
    assert sizes == ref_sizes
    assert got == ref, _diff_msg(got, ref)


@pytest.mark.parametrize("devices,n", [
    ([0, 0], 4096 * 21 + 77),     # two contexts on one GPU: 11 + 11 frames, ragged tail in the second
    ([0, 0, 0], 4096 * 2 + 5),    # more contexts than frames: one shard is empty
    ([0], 4096 * 9),
])
def test_multi_encode_matches_single(devices, n):
    """flacgpu_multi_encode_frames shards contiguous frame ranges over contexts (one per GPU in
    production; repeated ordinals here, on the one-GPU box) and concatenates them in frame
    order: the bytes and frame sizes equal one context's and the oracle's."""
    import flacgpu

    pcm = synth.synth_pcm(n, 2, 16, 44100, stream=13)
    with flacgpu.MultiEncoder(devices, 2, 16, 44100, max_frames=8) as me:
        got, sizes = me.encode_frames(pcm, first_frame=200)
    ref, ref_sizes, _ = oracle_ref.encode_stream(pcm, 2, 16, 44100, first_frame=200)
    assert sizes == ref_sizes
    assert got == ref, _diff_msg(got, ref)


def _wide_order_frames(ch):
    """32-bit frames at the edges of the u32 bestOrder certificate (fg_device.hpp step 5: the
    differences in u32 when every order's range over the frame fits i32, else the i64 totals):
    a sample range of exactly 2^31 - 1 (fast) and 2^31 (i64), INT_MIN present (order 0 null),
    first differences of +-(2^31 - 1) (order 1 valid, order 2 null), smooth frames on either side of
    the certificate (a ramp over exactly 2^31 - 1, sines of 0.49 and 0.999 full scale), and for
    stereo a side channel outside i32 (L = INT_MAX, R = INT_MIN)."""
    lo, hi = -(1 << 31), (1 << 31) - 1
    rng = np.random.Generator(np.random.PCG64(55))
    i = np.arange(4096)
    frames = []
    a = rng.integers(-(1 << 30), (1 << 30), size=4096)
    a[100], a[200] = -(1 << 30), (1 << 30) - 1                     # range exactly 2^31 - 1
    frames.append(a)
    b = a.copy()
    b[300] = 1 << 30                                                 # range 2^31
    frames.append(b)
    c = rng.integers(-1000, 1000, size=4096)
    c[2000] = lo                                                     # INT_MIN: order 0 null
    frames.append(c)
    frames.append(np.where(i % 2 == 0, (1 << 30) - 1, -(1 << 30)))  # e1 = +-(2^31 - 1)
    frames.append((np.sin(i / 700.0) * 0.999 * hi).astype(np.int64))  # large, smooth: i64 totals
    frames.append((np.sin(i / 700.0) * 0.49 * hi).astype(np.int64))   # smooth, range < 2^31 - 1: u32
    frames.append(np.round(np.linspace(-(1 << 30), (1 << 30) - 1, 4096)).astype(np.int64))  # range 2^31 - 1: u32
    frames.append(rng.integers(lo, hi + 1, size=4096))              # full-scale noise
    out = []
    for f in frames:
        f = np.clip(f.astype(np.int64), lo, hi)
        if ch == 1:
            out.append(f[:, None])
        else:
            r = np.clip(f // 2 + rng.integers(-5, 5, size=4096), lo, hi)
            out.append(np.stack([f, r], axis=1))
    if ch == 2:  # side outside i32 in some samples, inside in others
        l_ = np.where(i % 3 == 0, hi, rng.integers(-1000, 1000, size=4096))
        r_ = np.where(i % 3 == 0, lo, rng.integers(-1000, 1000, size=4096))
        out.append(np.stack([l_, r_], axis=1))
    return np.concatenate(out, axis=0)


@pytest.mark.parametrize("ch,lpc", [(1, 0), (2, 0), (2, 12), (1, 12)])
def test_32bit_fixed_order_certificate_edges(ch, lpc):
    """bestOrder of 32-bit full frames (u32 fast path or the exact i64 totals) equals the oracle's
    at every edge of the fast path's validity certificate."""
    s = _wide_order_frames(ch)
    pcm = synth.to_pcm_bytes(s, 32)
    enc = gpu_encoder(ch, 32, 192000, **({"lpc_order": lpc} if lpc else {}))
    ref, ref_sizes, _ = oracle_ref.encode_stream(pcm, ch, 32, 192000, **({"lpc": lpc} if lpc else {}))
    got, sizes = enc.encode_frames(pcm)
    assert sizes == ref_sizes, "per-frame sizes differ"
    assert got == ref, _diff_msg(got, ref)
    dec, _ = oracle_ref.decode_frames(got, ch, 32, 192000, len(s))
    assert dec == pcm
