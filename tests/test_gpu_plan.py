"""The device-resident plan path -- the path bench.py times -- against the CPU
restatement, byte for byte.

flacgpu_plan_create[_segments] + flacgpu_encode_plan_device[_md5_async|_ex]
over many independent streams in one device PCM buffer: every stream's
bitstream, per-frame sizes and MD5 digest are compared with
oracle_ref.encode_stream / hashlib on the same PCM (the reference's per-file
block loop, wav2flac.zig:66-97, with the MD5 of wav_reader.zig:66 finalised as
in encoder.zig:168-170).  Covers ragged lengths (0 and 1 sample, tails,
multiples of 4096), stream offsets at every 4-byte alignment mod 16, plans
larger than the context (plan-owned descriptors), both MD5 schedules, streams
spanning several calls with carried MD5 state, frame-number windows
(flacgpu_plan_advance), and the device error word (flacgpu_sync_check).
"""
import ctypes
import hashlib

import numpy as np
import pytest

import oracle_ref
import synth

pytestmark = pytest.mark.gpu


def _torch():
    import torch

    return torch, torch.device("cuda", 0)


def _layout(lengths, fb, aligns, gap=36):
    """Byte offsets for streams of `lengths` interchannel samples; offset % 16 cycles through aligns."""
    offs, pos = [], 0
    for i, n in enumerate(lengths):
        want = aligns[i % len(aligns)]
        pos += (want - pos) % 16
        offs.append(pos)
        pos += n * fb + gap
        pos = (pos + 3) & ~3
    return offs, pos + 64


def _run_plan(enc, pcm_all, offs, lengths, md5="join", first_frames=None, final=None, states=None, out_cap=None,
              advance=0):
    import flacgpu

    torch, dev = _torch()
    plan = enc.plan(offs, lengths, first_frames=first_frames, final=final)
    d_pcm = torch.from_numpy(np.frombuffer(pcm_all, dtype=np.uint8).copy()).to(dev)
    cap = int(plan.out_bound) if out_cap is None else out_cap
    d_out = torch.zeros(max(int(plan.out_bound), 1), dtype=torch.uint8, device=dev)
    nfr = max(int(plan.n_frames), 1)
    d_fb = torch.zeros(nfr, dtype=torch.int32, device=dev)
    d_off = torch.zeros(nfr, dtype=torch.int64, device=dev)
    d_tot = torch.zeros(2, dtype=torch.int64, device=dev)
    d_md5 = torch.zeros(max(len(offs), 1) * 16, dtype=torch.uint8, device=dev)
    st = torch.cuda.current_stream(dev)
    if advance:
        plan.advance(advance, st.cuda_stream)
    if md5 == "state":
        d_state = states if states is not None else torch.from_numpy(
            np.frombuffer(flacgpu.md5_states(len(offs)), dtype=np.uint8).copy()).to(dev)
        enc.encode_plan_device_ex(plan, d_pcm.data_ptr(), d_out.data_ptr(), cap, d_fb.data_ptr(), d_off.data_ptr(),
                                  d_tot.data_ptr(), d_state.data_ptr(), d_md5.data_ptr(), stream=st.cuda_stream)
    elif md5 == "async":
        ms = torch.cuda.Stream(dev)
        enc.encode_plan_device(plan, d_pcm.data_ptr(), d_out.data_ptr(), cap, d_fb.data_ptr(), d_off.data_ptr(),
                               d_tot.data_ptr(), d_md5.data_ptr(), st.cuda_stream, md5_stream=ms.cuda_stream)
        ms.synchronize()
        d_state = None
    else:
        enc.encode_plan_device(plan, d_pcm.data_ptr(), d_out.data_ptr(), cap, d_fb.data_ptr(), d_off.data_ptr(),
                               d_tot.data_ptr(), d_md5.data_ptr() if md5 == "join" else None, st.cuda_stream)
        d_state = None
    enc.sync_check(st.cuda_stream)
    total = int(d_tot[0].item())
    out = d_out[:total].cpu().numpy().tobytes()
    fb = d_fb.cpu().numpy()
    fo = d_off.cpu().numpy()
    res = []
    for s in range(len(offs)):
        f0 = plan.first_frame[s]
        f1 = plan.first_frame[s + 1] if s + 1 < len(offs) else int(plan.n_frames)
        a = int(fo[f0]) if f0 < int(plan.n_frames) else total
        b = int(fo[f1]) if f1 < int(plan.n_frames) else total
        res.append((out[a:b], [int(x) for x in fb[f0:f1]], d_md5[16 * s:16 * s + 16].cpu().numpy().tobytes()))
    # offsets are an exclusive scan of the sizes, the total their sum
    assert int(fb[: int(plan.n_frames)].astype(np.int64).sum()) == total
    plan.close()
    return res, d_state


def _encoder(ch, bits, rate, max_frames=64, **kw):
    import flacgpu

    return flacgpu.Encoder(ch, bits, rate, device=0, max_frames=max_frames, **kw)


LENGTHS = [0, 1, 3, 4096, 5000, 8192, 4095, 3 * 4096 + 77, 1152, 4097, 6 * 4096, 255, 2 * 4096 + 4095, 64, 12345]


@pytest.mark.parametrize("ch,bits,rate,lpc", [(2, 16, 44100, 0), (2, 24, 96000, 0), (1, 16, 48000, 0),
                                              (2, 32, 192000, 0), (8, 24, 96000, 0), (2, 24, 96000, 8)])
@pytest.mark.parametrize("aligns", [(0,), (4, 8, 12, 0)])
def test_plan_streams_match_oracle(ch, bits, rate, lpc, aligns):
    fb = ch * (bits // 8)
    offs, size = _layout(LENGTHS, fb, aligns)
    buf = bytearray(size)
    pcms = []
    for s, n in enumerate(LENGTHS):
        pcm = synth.synth_pcm(n, ch, bits, rate, stream=s) if n else b""
        buf[offs[s]:offs[s] + len(pcm)] = pcm
        pcms.append(pcm)
    with _encoder(ch, bits, rate, lpc_order=lpc) as enc:  # 64 frames per context < the plan's frames
        res, _ = _run_plan(enc, bytes(buf), offs, LENGTHS)
    for s, (got, sizes, md5) in enumerate(res):
        ref, ref_sizes, ref_md5 = oracle_ref.encode_stream(pcms[s], ch, bits, rate, lpc=lpc)
        assert sizes == ref_sizes, f"stream {s}: frame sizes differ"
        assert got == ref, f"stream {s}: bytes differ"
        assert md5 == ref_md5 == hashlib.md5(pcms[s]).digest(), f"stream {s}: MD5"


@pytest.mark.parametrize("md5", ["join", "async", "none", "state"])
def test_plan_md5_schedules(md5):
    ch, bits, rate = 2, 16, 44100
    lengths = [4096 * 8] * 40 + [4096 * 3 + 100] * 9 + [1]
    offs, size = _layout(lengths, 4, (0, 4))
    buf = bytearray(size)
    pcms = []
    for s, n in enumerate(lengths):
        pcm = synth.synth_pcm(n, ch, bits, rate, stream=100 + s)
        buf[offs[s]:offs[s] + len(pcm)] = pcm
        pcms.append(pcm)
    with _encoder(ch, bits, rate, max_frames=512) as enc:
        res, _ = _run_plan(enc, bytes(buf), offs, lengths, md5=md5)
    for s, (got, sizes, dig) in enumerate(res):
        ref, ref_sizes, ref_md5 = oracle_ref.encode_stream(pcms[s], ch, bits, rate)
        assert sizes == ref_sizes and got == ref, f"stream {s}"
        if md5 != "none":
            assert dig == ref_md5, f"stream {s}: MD5"
        else:
            assert dig == bytes(16)


@pytest.mark.parametrize("ch,bits,rate", [(2, 16, 44100), (2, 24, 96000), (8, 24, 96000), (2, 32, 192000)])
def test_streams_spanning_calls_carry_md5_state(ch, bits, rate):
    """Each stream is cut into segments encoded by successive calls: frame numbers continue,
    the MD5 state is carried on the device, only the last segment is padded."""
    torch, dev = _torch()
    import flacgpu

    fb = ch * (bits // 8)
    totals = [4096 * 7 + 1234, 4096 * 5, 4096 * 2 + 1, 4096 * 9 + 4095, 4096]
    seg_frames = [3, 2, 1, 4, 1]  # whole frames per non-final segment, per stream
    full = [synth.synth_pcm(n, ch, bits, rate, stream=300 + s) for s, n in enumerate(totals)]
    pos = [0] * len(totals)
    fnum = [0] * len(totals)
    outs = [b""] * len(totals)
    sizes = [[] for _ in totals]
    state = torch.from_numpy(np.frombuffer(flacgpu.md5_states(len(totals)), dtype=np.uint8).copy()).to(dev)
    digest = [None] * len(totals)
    with _encoder(ch, bits, rate, max_frames=32) as enc:
        while any(pos[s] < totals[s] or digest[s] is None for s in range(len(totals))):
            # every stream advances by its segment length (streams that are done take an empty final segment)
            lens, fin = [], []
            for s in range(len(totals)):
                left = totals[s] - pos[s]
                take = min(left, seg_frames[s] * 4096)
                last = take == left
                lens.append(take if digest[s] is None else 0)
                fin.append(last)
            offs, size = _layout(lens, fb, (4, 0))
            buf = bytearray(size)
            for s in range(len(totals)):
                a = pos[s] * fb
                buf[offs[s]:offs[s] + lens[s] * fb] = full[s][a:a + lens[s] * fb]
            res, state = _run_plan(enc, bytes(buf), offs, lens, md5="state", first_frames=fnum, final=fin,
                                   states=state)
            for s, (got, sz, dig) in enumerate(res):
                if digest[s] is not None:
                    # a finished state passed again is left as it is: the same digest, no re-padding
                    assert dig == digest[s], f"stream {s}: finished MD5 state changed"
                    continue
                outs[s] += got
                sizes[s] += sz
                pos[s] += lens[s]
                fnum[s] += (lens[s] + 4095) // 4096
                if fin[s]:
                    digest[s] = dig
    for s in range(len(totals)):
        ref, ref_sizes, ref_md5 = oracle_ref.encode_stream(full[s], ch, bits, rate)
        assert sizes[s] == ref_sizes and outs[s] == ref, f"stream {s}"
        assert digest[s] == ref_md5 == hashlib.md5(full[s]).digest(), f"stream {s}: carried MD5"


def test_host_md5_engine_matches_device_state_by_state():
    """flacgpu_md5_plan_host (the plan path's host engine) carries the same per-stream state as the
    device MD5, call by call, segments final and not, finished states left alone; and the engine
    pick is the host pool for a few long streams, the GPU lanes for many short ones."""
    torch, dev = _torch()
    import flacgpu

    ch, bits, rate = 2, 16, 44100
    fb = ch * (bits // 8)
    totals = [4096 * 5 + 77, 4096 * 3, 4096 * 4 + 4095, 4096]
    seg = 2 * 4096
    full = [synth.synth_pcm(n, ch, bits, rate, stream=700 + s) for s, n in enumerate(totals)]
    pos = [0] * len(totals)
    fnum = [0] * len(totals)
    d_state = torch.from_numpy(np.frombuffer(flacgpu.md5_states(len(totals)), dtype=np.uint8).copy()).to(dev)
    h_state = (flacgpu.Md5State * len(totals))()
    flacgpu.load_library().flacgpu_md5_state_init(h_state, len(totals))
    done = [False] * len(totals)
    with _encoder(ch, bits, rate, max_frames=32) as enc:
        for _ in range(4):
            lens, fin = [], []
            for s in range(len(totals)):
                take = 0 if done[s] else min(totals[s] - pos[s], seg)
                lens.append(take)
                fin.append(done[s] or pos[s] + take == totals[s])
            offs, size = _layout(lens, fb, (4, 0))
            buf = bytearray(size)
            for s in range(len(totals)):
                buf[offs[s]:offs[s] + lens[s] * fb] = full[s][pos[s] * fb:(pos[s] + lens[s]) * fb]
            res, d_state = _run_plan(enc, bytes(buf), offs, lens, md5="state", first_frames=fnum, final=fin,
                                     states=d_state)
            plan = enc.plan(offs, lens, first_frames=fnum, final=fin)
            h_buf = np.frombuffer(bytes(buf), dtype=np.uint8)
            dig = (ctypes.c_uint8 * (16 * len(totals)))()
            plan.md5_host(h_buf.ctypes.data, h_state, ctypes.addressof(dig))
            plan.close()
            assert bytes(h_state) == d_state.cpu().numpy().tobytes(), "host and device MD5 states differ"
            for s in range(len(totals)):
                if fin[s]:
                    assert bytes(dig)[16 * s:16 * s + 16] == res[s][2] == hashlib.md5(full[s]).digest()
                pos[s] += lens[s]
                fnum[s] += (lens[s] + 4095) // 4096
                done[s] = fin[s]
        assert all(done)
        few = enc.plan([s * 4096 * 1024 * fb for s in range(8)], [4096 * 1024] * 8, final=[False] * 8)
        many = enc.plan([s * 4096 * 16 * fb for s in range(16384)], [4096 * 16] * 16384, final=[False] * 16384)
        assert few.md5_engine() == flacgpu.MD5_HOST and many.md5_engine() == flacgpu.MD5_DEVICE
        few.close()
        many.close()


def test_host_md5_plan_rules():
    """flacgpu_md5_plan_host's input rules match the device path's: no state with a non-final
    segment is an error, an empty plan is a no-op on the device engine's side of the pick."""
    import flacgpu

    ch, bits, rate = 2, 16, 44100
    with _encoder(ch, bits, rate, max_frames=8) as enc:
        plan = enc.plan([0], [4096], final=[False])
        buf = np.zeros(4096 * 4, dtype=np.uint8)
        with pytest.raises(flacgpu.FlacGpuError):
            plan.md5_host(buf.ctypes.data, None, None)  # nowhere to carry the chain
        plan.close()
        empty = enc.plan([], [])
        assert empty.md5_engine() == flacgpu.MD5_DEVICE
        empty.md5_host(buf.ctypes.data, None, None)
        empty.close()


def test_non_final_segment_must_be_whole_frames():
    import flacgpu

    with _encoder(2, 16, 44100) as enc:
        with pytest.raises(flacgpu.FlacGpuError):
            enc.plan([0], [4096 + 5], final=[False])
        with pytest.raises(flacgpu.FlacGpuError):  # offsets are 4-byte aligned
            enc.plan([2], [4096])
        with pytest.raises(flacgpu.FlacGpuError):  # u36 frame numbers
            enc.plan([0], [8192], first_frames=[(1 << 36) - 1])


@pytest.mark.parametrize("delta", [1, 127, 2048, (1 << 31) + 5])
def test_plan_advance_renumbers_frames(delta):
    ch, bits, rate = 2, 16, 44100
    lengths = [4096 * 4, 4096 * 2 + 9]
    offs, size = _layout(lengths, 4, (0,))
    buf = bytearray(size)
    pcms = []
    for s, n in enumerate(lengths):
        pcm = synth.synth_pcm(n, ch, bits, rate, stream=7 + s)
        buf[offs[s]:offs[s] + len(pcm)] = pcm
        pcms.append(pcm)
    with _encoder(ch, bits, rate) as enc:
        res, _ = _run_plan(enc, bytes(buf), offs, lengths, first_frames=[10, 0], advance=delta)
    for s, (got, sizes, _) in enumerate(res):
        ref, ref_sizes, _ = oracle_ref.encode_stream(pcms[s], ch, bits, rate, first_frame=[10, 0][s] + delta)
        assert sizes == ref_sizes and got == ref, f"stream {s}"


def test_sync_check_reports_output_too_small():
    import flacgpu

    ch, bits, rate = 2, 16, 44100
    lengths = [4096 * 16]
    pcm = synth.synth_pcm(lengths[0], ch, bits, rate)
    with _encoder(ch, bits, rate) as enc:
        with pytest.raises(flacgpu.FlacGpuError) as e:
            _run_plan(enc, pcm + bytes(64), [0], lengths, out_cap=4096)
        assert e.value.code == -4
        # the error word is cleared: the next call is clean
        res, _ = _run_plan(enc, pcm + bytes(64), [0], lengths)
        ref, _, _ = oracle_ref.encode_stream(pcm, ch, bits, rate)
        assert res[0][0] == ref


@pytest.mark.parametrize("misalign", [False, True])
def test_plan_scan_spans_blocks(misalign):
    # > 2 x 4096 frames (block size 16): the multi-workgroup scan's block sums; the size and
    # offset arrays optionally at 4- / 8-byte (not 16-byte) alignment, its element-wise path
    torch, dev = _torch()
    ch, bits, rate, bs = 2, 16, 44100, 16
    n = 16 * 9000 + 5
    pcm = synth.synth_pcm(n, ch, bits, rate, stream=3)
    with _encoder(ch, bits, rate, max_frames=64, block_size=bs) as enc:
        plan = enc.plan([0], [n])
        nf = int(plan.n_frames)
        assert nf == 9001
        d_pcm = torch.from_numpy(np.frombuffer(pcm, dtype=np.uint8).copy()).to(dev)
        d_out = torch.zeros(int(plan.out_bound), dtype=torch.uint8, device=dev)
        fb_buf = torch.zeros(nf + 4, dtype=torch.int32, device=dev)
        off_buf = torch.zeros(nf + 2, dtype=torch.int64, device=dev)
        d_tot = torch.zeros(2, dtype=torch.int64, device=dev)
        sh_fb, sh_off = (1, 1) if misalign else (0, 0)
        st = torch.cuda.current_stream(dev)
        enc.encode_plan_device(plan, d_pcm.data_ptr(), d_out.data_ptr(), int(plan.out_bound),
                               fb_buf.data_ptr() + 4 * sh_fb, off_buf.data_ptr() + 8 * sh_off, d_tot.data_ptr(), None,
                               st.cuda_stream)
        enc.sync_check(st.cuda_stream)
        plan.close()
        sizes = fb_buf[sh_fb:sh_fb + nf].cpu().numpy().astype(np.int64)
        offs = off_buf[sh_off:sh_off + nf].cpu().numpy()
        total = int(d_tot[0].item())
    assert offs[0] == 0 and (np.diff(offs) == sizes[:-1]).all() and total == int(sizes.sum())
    ref, ref_sizes, _ = oracle_ref.encode_stream(pcm, ch, bits, rate, block=bs)
    assert [int(x) for x in sizes] == ref_sizes
    assert d_out[:total].cpu().numpy().tobytes() == ref


def test_default_stream_producer_is_ordered():
    """d_pcm written by a GPU kernel on torch's default (legacy null) stream and encoded at once
    through stream handle 0: the wrapper passes FLACGPU_STREAM_LEGACY, so the encode is queued
    behind the producer (and behind the default-stream zero-fill of the result buffers) instead of
    running unordered on the context's non-blocking stream."""
    torch, dev = _torch()
    import flacgpu

    n = 48 * 4096 + 333
    pcm = synth.synth_pcm(n, 2, 16, 44100, stream=77)
    key = 0x5A
    src = torch.from_numpy(np.frombuffer(pcm, dtype=np.uint8) ^ np.uint8(key)).to(dev)
    torch.cuda.synchronize()
    assert torch.cuda.current_stream(dev).cuda_stream == 0
    a = torch.randn(4096, 4096, device=dev)
    for _ in range(6):  # keep the default stream busy for a while before the producer runs
        a = (a @ a) * 1e-3
    d_pcm = torch.bitwise_xor(src, key)  # the producer kernel, queued behind the matmuls
    with flacgpu.Encoder(2, 16, 44100, max_frames=64) as enc:
        frames, sizes = enc.encode_frames_device(d_pcm.data_ptr(), n)  # current stream: handle 0
        got, got_sizes = frames.cpu().numpy().tobytes(), [int(x) for x in sizes.cpu()]
    ref, ref_sizes, _ = oracle_ref.encode_stream(pcm, 2, 16, 44100)
    assert got_sizes == ref_sizes and got == ref
    assert flacgpu._stream(0) == flacgpu.STREAM_LEGACY and flacgpu._stream(None) is None


@pytest.mark.parametrize("kernel", ["0", "1", "2", "3", "4", "5"])
def test_md5_kernels_ragged(kernel, monkeypatch):
    """Every stream-MD5 kernel geometry (FLACGPU_MD5_KERNEL: 0 per-lane loads, 1 the default
    coalesced LDS-DMA ring, 2..5 ring variants) on 300 streams whose whole-block counts run
    0..47 with ragged tails (odd and even chunk counts, lanes ending at every ring slot, partial
    waves and workgroups), 4-byte aligned offsets: digests == hashlib."""
    monkeypatch.setenv("FLACGPU_MD5_KERNEL", kernel)
    rng = np.random.Generator(np.random.PCG64(4242))
    n_streams = 300
    lengths = [int(x) for x in rng.integers(0, 48 * 16 + 16, size=n_streams)]  # samples (4 B each)
    lengths[:6] = [0, 1, 16, 32, 47 * 16 + 15, 5000]
    offs, size = _layout(lengths, 4, (0, 4, 8, 12), gap=12)
    buf = bytearray(rng.integers(0, 256, size=size, dtype=np.uint8).tobytes())
    with _encoder(2, 16, 44100, max_frames=512) as enc:
        res, _ = _run_plan(enc, bytes(buf), offs, lengths, md5="join")
    for s, (_, _, dig) in enumerate(res):
        want = hashlib.md5(bytes(buf[offs[s]:offs[s] + 4 * lengths[s]])).digest()
        assert dig == want, f"stream {s} ({lengths[s]} samples): MD5 kernel {kernel}"


# ---- the overlapped encode schedule (flacgpu_set_overlap): the full frames in ranges, the
# analysis of range i+1 beside the scan (carried base) + pack of range i on a second HIP stream,
# per-range ticket sets, tail frames analysed first and packed last.  Same bytes as the oracle.
@pytest.mark.parametrize("ch,bits,rate,lpc", [(2, 16, 44100, 0), (8, 24, 96000, 0), (2, 24, 96000, 8),
                                              (2, 32, 192000, 0), (1, 16, 48000, 0)])
@pytest.mark.parametrize("ranges,ana,pack", [(4, 2, 2), (3, 0, 0), (7, 1, 3)])
def test_overlapped_schedule_matches_oracle(ch, bits, rate, lpc, ranges, ana, pack, diag_build):
    fb = ch * (bits // 8)
    offs, size = _layout(LENGTHS, fb, (4, 8, 12, 0))
    buf = bytearray(size)
    pcms = []
    for s, n in enumerate(LENGTHS):
        pcm = synth.synth_pcm(n, ch, bits, rate, stream=300 + s) if n else b""
        buf[offs[s]:offs[s] + len(pcm)] = pcm
        pcms.append(pcm)
    with _encoder(ch, bits, rate, lpc_order=lpc) as enc:
        enc.set_overlap(ranges, ana, pack, min_frames=2)
        for md5 in ("join", "state"):  # twice: the per-range ticket sets are reused by the second call
            res, _ = _run_plan(enc, bytes(buf), offs, LENGTHS, md5=md5)
            for s, (got, sizes, dig) in enumerate(res):
                ref, ref_sizes, ref_md5 = oracle_ref.encode_stream(pcms[s], ch, bits, rate, lpc=lpc)
                assert sizes == ref_sizes, f"stream {s}: frame sizes differ"
                assert got == ref, f"stream {s}: bytes differ"
                if md5 == "join":
                    assert dig == ref_md5, f"stream {s}: MD5"


def test_overlapped_schedule_many_ranges_and_serial_again(diag_build):
    """64 ranges of a long plan, then the serial schedule on the same context (ticket sets shared)."""
    ch, bits, rate = 2, 16, 44100
    lengths = [4096 * 16 + 5] * 24 + [4096 * 7] * 8
    offs, size = _layout(lengths, 4, (0, 8))
    buf = bytearray(size)
    pcms = []
    for s, n in enumerate(lengths):
        pcm = synth.synth_pcm(n, ch, bits, rate, stream=400 + s)
        buf[offs[s]:offs[s] + len(pcm)] = pcm
        pcms.append(pcm)
    refs = [oracle_ref.encode_stream(p, ch, bits, rate)[:2] for p in pcms]
    with _encoder(ch, bits, rate, max_frames=512) as enc:
        for ranges in (64, 0, 5, 1):
            enc.set_overlap(ranges, 2, 2, min_frames=1)
            res, _ = _run_plan(enc, bytes(buf), offs, lengths, md5="none")
            for s, (got, sizes, _) in enumerate(res):
                assert (got, sizes) == (refs[s][0], refs[s][1]), f"ranges {ranges} stream {s}"


def test_overlap_refused_in_release_build():
    """The release library refuses ranges > 1 (the schedule is a diagnostic-build alternative);
    ranges <= 1 (the serial schedule) is accepted."""
    import flacgpu

    if flacgpu.diag_build():
        pytest.skip("release build only")
    with _encoder(2, 16, 44100) as enc:
        enc.set_overlap(1, 2, 2)
        with pytest.raises(flacgpu.FlacGpuError):
            enc.set_overlap(4, 2, 2)


def _host_replay(sizes, lo=0xFFFFFF, hi=0):
    """StreamInfo.updateFrameSize (metadata.zig:35-40) through the C ABI's host restatement."""
    import flacgpu

    si = flacgpu.StreamInfo.new(44100, 2, 16, 0)
    si.min_frame_size, si.max_frame_size = lo, hi
    for v in sizes:
        si.update_frame_size(int(v))
    return [int(si.min_frame_size), int(si.max_frame_size)]


@pytest.mark.parametrize("n", [1, 64, 1023, 1025, 5000, 70000])
@pytest.mark.parametrize("shape", ["random", "rising", "falling", "sawtooth"])
@pytest.mark.parametrize("carried", [False, True])
def test_streaminfo_replay_device_matches_host(n, shape, carried):
    """flacgpu_streaminfo_replay_device (k_streaminfo_replay: per-thread runs past 1024 frames,
    cross-wave max scan with a carried {min, max}) == the host loop of
    flacgpu_streaminfo_update_frame_size, including the reference's else-if quirk (a frame that
    raises the running max never lowers the min)."""
    import flacgpu

    torch, dev = _torch()
    rng = np.random.default_rng(n * 7 + len(shape))
    if shape == "random":
        sizes = rng.integers(10, 20000, n)
    elif shape == "rising":
        sizes = np.arange(n) * 3 + 100
    elif shape == "falling":
        sizes = 400000 - np.arange(n) * 5
    else:
        sizes = (np.arange(n) % 97) * 11 + rng.integers(0, 3, n)
    sizes = sizes.astype(np.int32)
    start = [1500, 9000] if carried else [0xFFFFFF, 0]
    want = _host_replay(sizes, *start)
    with flacgpu.Encoder(2, 16, 44100, device=0, max_frames=64) as enc:
        d_fb = torch.from_numpy(sizes).to(dev)
        mm = torch.tensor(start, dtype=torch.int32, device=dev)
        enc.streaminfo_replay_device(d_fb.data_ptr(), n, mm.data_ptr())
        torch.cuda.synchronize()
        assert mm.cpu().tolist() == want


@pytest.mark.parametrize("variant", ["1", "2"])
def test_one_wave_analysis_matches_oracle(variant, monkeypatch, diag_build):
    """k_ana1 (fg_ana1.hpp: one wave per full 16-bit stereo frame, FLACGPU_ANA1=1 / 2) writes the
    same frames and sizes as the restatement (and so as k_analyze), and the same decision records."""
    monkeypatch.setenv("FLACGPU_ANA1", variant)
    ch, bits, rate = 2, 16, 44100
    lengths = [4096 * 9 + 17, 4096 * 3, 1, 4096 * 5 - 1, 4096 * 64]
    fb = ch * bits // 8
    offs, total = _layout(lengths, fb, [0, 4, 8, 12])
    pcm_all = bytearray(total)
    pcms = []
    for s, n in enumerate(lengths):
        pcm = synth.synth_pcm(n, ch, bits, rate, stream=40 + s)
        pcm_all[offs[s]:offs[s] + len(pcm)] = pcm
        pcms.append(pcm)
    with _encoder(ch, bits, rate, max_frames=128) as enc:
        res, _ = _run_plan(enc, bytes(pcm_all), offs, lengths, md5="join")
    for s, n in enumerate(lengths):
        ref, ref_sizes, ref_md5 = oracle_ref.encode_stream(pcms[s], ch, bits, rate)
        got, sizes, md5 = res[s]
        assert sizes == ref_sizes and got == ref and md5 == ref_md5, f"stream {s}"
    # decision records of every candidate (66 frames incl. the special blocks) against the oracle's,
    # from a fresh encoder (test_gpu_parity caches its encoders; this one must see FLACGPU_ANA1)
    import test_gpu_parity as tp

    saved = dict(tp._encoders)
    tp._encoders.clear()
    try:
        tp._records_match(ch, bits, rate, 4096 * 66)
    finally:
        for e in tp._encoders.values():
            e.close()
        tp._encoders.clear()
        tp._encoders.update(saved)
