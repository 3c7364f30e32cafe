"""File-level host code of libflacgpu.so (fg_file.cpp): WAV header parsing,
StreamInfo, the metadata writers, and (GPU) whole-file encodes, against the
restatement's oracle_encode_file (wav2flac.zig:10-97, metadata.zig, encoder.zig:177-226)."""
import ctypes
import hashlib
import io
import struct
import wave

import numpy as np
import pytest

import flacgpu
import oracle_ref
import synth


def make_wav(pcm: bytes, ch: int, bits: int, rate: int) -> bytes:
    b = io.BytesIO()
    with wave.open(b, "wb") as w:
        w.setnchannels(ch)
        w.setsampwidth(bits // 8)
        w.setframerate(rate)
        w.writeframes(pcm)
    return b.getvalue()


def make_wav_extensible(pcm: bytes, ch: int, bits: int, rate: int, valid_bits: int, junk: bool = True) -> bytes:
    B = bits // 8
    fmt = struct.pack("<HHIIHH", 0xFFFE, ch, rate, rate * ch * B, ch * B, bits)
    fmt += struct.pack("<HHI", 22, valid_bits, 0) + b"\x01\x00\x00\x00\x00\x00\x10\x00\x80\x00\x00\xaa\x00\x38\x9b\x71"
    chunks = b""
    if junk:
        chunks += b"JUNK" + struct.pack("<I", 6) + b"\x00" * 6
    chunks += b"fmt " + struct.pack("<I", len(fmt)) + fmt
    if junk:
        chunks += b"LIST" + struct.pack("<I", 4) + b"INFO"
    chunks += b"data" + struct.pack("<I", len(pcm)) + pcm
    return b"RIFF" + struct.pack("<I", 4 + len(chunks)) + b"WAVE" + chunks


@pytest.mark.parametrize("ch,bits,rate", [(2, 16, 44100), (1, 24, 96000), (8, 32, 48000), (3, 8, 22050)])
def test_wav_parse_plain(ch, bits, rate):
    pcm = synth.synth_pcm(1000, ch, bits, rate)
    w = make_wav(pcm, ch, bits, rate)
    info = flacgpu.wav_parse(w)
    assert (info.channels, info.bits_per_sample, info.sample_rate, info.samples) == (ch, bits, rate, 1000)
    assert w[info.data_offset:info.data_offset + info.data_bytes] == pcm


def test_wav_parse_extensible_and_chunks():
    pcm = synth.synth_pcm(333, 2, 24, 96000)
    w = make_wav_extensible(pcm, 2, 24, 96000, 24)
    info = flacgpu.wav_parse(w)
    assert (info.channels, info.bits_per_sample, info.bytes_per_sample, info.samples) == (2, 24, 3, 333)
    assert w[info.data_offset:info.data_offset + info.data_bytes] == pcm


@pytest.mark.parametrize("mutate", ["riff", "wave", "codec", "byterate", "datalen", "nodata"])
def test_wav_parse_rejects(mutate):
    pcm = synth.synth_pcm(100, 2, 16, 44100)
    w = bytearray(make_wav(pcm, 2, 16, 44100))
    if mutate == "riff":
        w[0:4] = b"RIFX"
    elif mutate == "wave":
        w[8:12] = b"AVI "
    elif mutate == "codec":
        w[20:22] = struct.pack("<H", 3)  # IEEE float
    elif mutate == "byterate":
        w[28:32] = struct.pack("<I", 1)
    elif mutate == "datalen":
        w[40:44] = struct.pack("<I", len(pcm) - 1)
    elif mutate == "nodata":
        w[36:40] = b"dat_"
    with pytest.raises(flacgpu.FlacGpuError):
        flacgpu.wav_parse(bytes(w))


def test_streaminfo_update_quirk_and_bytes():
    si = flacgpu.StreamInfo.new(44100, 2, 16, 123456)
    si.update_frame_size(1000)   # raises max only: min stays 0xFFFFFF
    assert (si.min_frame_size, si.max_frame_size) == (0xFFFFFF, 1000)
    si.update_frame_size(900)    # below max: lowers min
    si.update_frame_size(1200)
    si.update_frame_size(950)
    assert (si.min_frame_size, si.max_frame_size) == (900, 1200)
    b = si.bytes()
    assert b[0:4] == bytes([0x10, 0x00, 0x10, 0x00])
    assert b[4:7] == (900).to_bytes(3, "big") and b[7:10] == (1200).to_bytes(3, "big")
    packed = int.from_bytes(b[10:18], "big")
    assert packed >> 44 == 44100 and (packed >> 41) & 7 == 1 and (packed >> 36) & 31 == 15
    assert packed & ((1 << 36) - 1) == 123456


@pytest.mark.parametrize("ch,bits,rate,n", [(2, 16, 44100, 2 * 4096 + 333), (1, 24, 96000, 4096),
                                             (2, 32, 192000, 5000), (8, 24, 96000, 100)])
def test_header_bytes_match_oracle_file(ch, bits, rate, n):
    pcm = synth.synth_pcm(n, ch, bits, rate)
    ref = oracle_ref.encode_file(pcm, ch, bits, rate)
    _, sizes, md5 = oracle_ref.encode_stream(pcm, ch, bits, rate)
    si = flacgpu.StreamInfo.new(rate, ch, bits, n)
    for s in sizes:
        si.update_frame_size(s)
    ctypes.memmove(si.md5, hashlib.md5(pcm).digest(), 16)
    hdr = flacgpu.header_bytes(si, False) + flacgpu.vorbis_comment_bytes(True)
    assert len(hdr) == 73 and hdr == ref[:73]


@pytest.mark.gpu
@pytest.mark.parametrize("ch,bits,rate,n", [(2, 16, 44100, 3 * 4096 + 1000), (1, 16, 44100, 4096),
                                             (2, 24, 96000, 2 * 4096 + 7), (2, 32, 192000, 4096 + 1),
                                             (8, 24, 96000, 4096 + 100), (2, 16, 44100, 1)])
def test_gpu_encode_file_matches_oracle(ch, bits, rate, n):
    pcm = synth.synth_pcm(n, ch, bits, rate)
    with flacgpu.Encoder(ch, bits, rate, max_frames=16) as enc:
        out = enc.encode_file(pcm)
    assert out == oracle_ref.encode_file(pcm, ch, bits, rate)


@pytest.mark.gpu
@pytest.mark.parametrize("ch,bits,rate", [(2, 16, 44100), (2, 24, 96000), (8, 24, 96000)])
@pytest.mark.parametrize("engine", ["host", "device"])
def test_gpu_encode_files_matches_oracle(ch, bits, rate, engine):
    """flacgpu_encode_files: each file byte-identical to the oracle's whole-file encode; the
    pipeline runs on across files (max_frames=8: 4-frame chunks, so files end mid-pipeline and
    chunks never span two files), empty and sub-frame files included."""
    lens = [3 * 4096 + 1000, 1, 0, 9 * 4096, 4096 + 5, 17 * 4096 + 4095, 7]
    pcms = [synth.synth_pcm(n, ch, bits, rate, stream=40 + i) if n else b"" for i, n in enumerate(lens)]
    with flacgpu.Encoder(ch, bits, rate, max_frames=8) as enc:
        if engine == "device":
            enc.set_md5_engine(flacgpu.MD5_DEVICE)
        outs = enc.encode_files(pcms)
        again = enc.encode_files(pcms[::-1])
    for i, pcm in enumerate(pcms):
        ref = oracle_ref.encode_file(pcm, ch, bits, rate)
        assert outs[i] == ref, f"file {i}"
        assert again[len(pcms) - 1 - i] == ref, f"file {i} (reversed batch)"


@pytest.mark.gpu
def test_gpu_encode_files_without_md5_diagnostic(monkeypatch):
    """FLACGPU_FILES_MD5=0 (diagnostic builds only: the schedule without its hashing) changes nothing
    but the STREAMINFO MD5, written as zero ("not computed"; bytes 26..41 of the file).  The release
    library ignores it: every file is byte-identical to the restatement's, MD5 included."""
    ch, bits, rate = 2, 16, 44100
    lens = [3 * 4096 + 1000, 0, 9 * 4096]
    pcms = [synth.synth_pcm(n, ch, bits, rate, stream=60 + i) if n else b"" for i, n in enumerate(lens)]
    monkeypatch.setenv("FLACGPU_FILES_MD5", "0")
    with flacgpu.Encoder(ch, bits, rate, max_frames=8) as enc:
        outs = enc.encode_files(pcms)
    diag = flacgpu.diag_build()
    for i, pcm in enumerate(pcms):
        ref = oracle_ref.encode_file(pcm, ch, bits, rate)
        assert outs[i][:26] == ref[:26] and outs[i][42:] == ref[42:], f"file {i}"
        assert outs[i][26:42] == (bytes(16) if diag else ref[26:42])


@pytest.mark.gpu
@pytest.mark.parametrize("sets", ["2", "3"])
def test_gpu_encode_files_pipe_sets(sets, monkeypatch):
    """The pipelined schedule with two or three chunk sets (FLACGPU_PIPE_SETS, output-invariant):
    files several chunks long (6-frame chunks), ragged and empty, byte-identical to the oracle."""
    monkeypatch.setenv("FLACGPU_PIPE_SETS", sets)
    ch, bits, rate = 2, 16, 44100
    lens = [40 * 4096 + 333, 0, 13 * 4096, 7 * 4096 + 1]
    pcms = [synth.synth_pcm(n, ch, bits, rate, stream=80 + i) if n else b"" for i, n in enumerate(lens)]
    with flacgpu.Encoder(ch, bits, rate, max_frames=18) as enc:
        outs = enc.encode_files(pcms)
        one = enc.encode_file(pcms[0])
    for i, pcm in enumerate(pcms):
        assert outs[i] == oracle_ref.encode_file(pcm, ch, bits, rate), f"file {i}"
    assert one == outs[0]


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["max_frames_1", "records_on"])
def test_gpu_encode_files_where_the_pipeline_cannot_run(mode):
    """flacgpu_encode_files on the contexts its pipelined schedule cannot serve (one frame per call;
    decision records on) encodes file by file, as flacgpu_encode_file does."""
    ch, bits, rate = 2, 16, 44100
    lens = [2 * 4096 + 77, 0, 4096]
    pcms = [synth.synth_pcm(n, ch, bits, rate, stream=70 + i) if n else b"" for i, n in enumerate(lens)]
    with flacgpu.Encoder(ch, bits, rate, max_frames=1 if mode == "max_frames_1" else 8) as enc:
        if mode == "records_on":
            enc.set_records(True)
        outs = enc.encode_files(pcms)
        recs = enc.records() if mode == "records_on" else None
    for i, pcm in enumerate(pcms):
        assert outs[i] == oracle_ref.encode_file(pcm, ch, bits, rate), f"file {i}"
    if recs is not None:
        # the records of EVERY file, file after file in frame order, each frame's
        # size equal to the one the restatement writes
        nfs = [(n + 4095) // 4096 for n in lens]
        assert len(recs) == sum(nfs)
        ref_sizes = [s for pcm in pcms if pcm for s in oracle_ref.encode_stream(pcm, ch, bits, rate)[1]]
        assert [r.frame_bytes for r in recs] == ref_sizes


@pytest.mark.gpu
@pytest.mark.parametrize("block", [1152, 4096, 192, 4000])
def test_gpu_encode_file_block_sizes(block):
    """STREAMINFO min/max block size follows the context's block size (the reference only
    runs 4096, wav_reader.zig:106-107, where both agree)."""
    ch, bits, rate = 2, 16, 44100
    n = 7 * block + 321
    pcm = synth.synth_pcm(n, ch, bits, rate)
    with flacgpu.Encoder(ch, bits, rate, max_frames=16, block_size=block) as enc:
        out = enc.encode_file(pcm)
    ref = oracle_ref.encode_file(pcm, ch, bits, rate, block=block)
    assert out == ref
    assert int.from_bytes(out[8:10], "big") == int.from_bytes(out[10:12], "big") == block


@pytest.mark.gpu
@pytest.mark.parametrize("engine", ["host", "device"])
@pytest.mark.parametrize("n", [0, 1, 3 * 4096 + 1000, 40 * 4096])
def test_md5_engines_match_hashlib(engine, n):
    """flacgpu_md5_*: the default host engine and the opt-in one-GPU-lane engine, fed in
    uneven pieces (Md5.update per block, wav_reader.zig:66), and encode_file with either."""
    ch, bits, rate = 2, 16, 44100
    pcm = synth.synth_pcm(n, ch, bits, rate) if n else b""
    with flacgpu.Encoder(ch, bits, rate, max_frames=16) as enc:
        if engine == "device":
            enc.set_md5_engine(flacgpu.MD5_DEVICE)
        assert enc.lib.flacgpu_md5_get_engine(enc.ctx) == (1 if engine == "device" else 0)
        enc.lib.flacgpu_md5_init(enc.ctx)
        for a in range(0, len(pcm), 1000 * 4 + 12):
            enc.md5_update(pcm[a:a + 1000 * 4 + 12])
        assert enc.md5_final() == hashlib.md5(pcm).digest()
        out = enc.encode_file(pcm)
    assert out == oracle_ref.encode_file(pcm, ch, bits, rate)


@pytest.mark.gpu
@pytest.mark.parametrize("ch,bits,rate", [(2, 16, 44100), (2, 24, 96000), (1, 32, 48000)])
def test_gpu_wav_to_flac(ch, bits, rate):
    n = 2 * 4096 + 77
    pcm = synth.synth_pcm(n, ch, bits, rate)
    out = flacgpu.wav_to_flac(make_wav(pcm, ch, bits, rate))
    assert out == oracle_ref.encode_file(pcm, ch, bits, rate)
    dec, _ = oracle_ref.decode_frames(out[73:], ch, bits, rate, n)
    assert dec == pcm and out[8 + 18:8 + 34] == hashlib.md5(pcm).digest()


CPP_DIR = __import__("os").path.join(__import__("os").path.dirname(__import__("os").path.abspath(__file__)), "cpp")


def _cpp_driver():
    import os
    import subprocess

    subprocess.check_call(["make", "-s", "-C", CPP_DIR])
    return os.path.join(CPP_DIR, "build", "encoder_api_test")


def _has_gpu():
    try:
        import torch

        return torch.cuda.device_count() > 0
    except Exception:
        return False


@pytest.mark.skipif(_has_gpu(), reason="checks the no-device failure path")
def test_cpp_api_driver_builds_and_fails_loudly_without_gpu(tmp_path):
    import subprocess

    exe = _cpp_driver()
    raw = tmp_path / "x.raw"
    raw.write_bytes(synth.synth_pcm(100, 2, 16, 44100))
    r = subprocess.run([exe, str(raw), "2", "16", "44100", str(tmp_path / "o.flac")], capture_output=True, text=True)
    assert r.returncode == 1 and "HIP device error" in r.stderr


@pytest.mark.gpu
@pytest.mark.parametrize("ch,bits,rate,n", [(2, 16, 44100, 3 * 4096 + 1000), (1, 24, 96000, 4096 + 3),
                                             (8, 16, 48000, 4096 + 64)])
def test_cpp_encoder_api_matches_oracle_file(tmp_path, ch, bits, rate, n):
    import subprocess

    exe = _cpp_driver()
    pcm = synth.synth_pcm(n, ch, bits, rate)
    raw = tmp_path / "x.raw"
    raw.write_bytes(pcm)
    out = tmp_path / "o.flac"
    subprocess.check_call([exe, str(raw), str(ch), str(bits), str(rate), str(out)])
    assert out.read_bytes() == oracle_ref.encode_file(pcm, ch, bits, rate)


@pytest.mark.gpu
@pytest.mark.parametrize("world,ch,bits,n,maxf", [(1, 2, 16, 21 * 4096 + 99, 8), (1, 8, 24, 5 * 4096, 2),
                                                  (2, 2, 16, 21 * 4096 + 99, 4), (8, 2, 16, 64 * 4096 + 1, 4)])
def test_cpp_sharded_encode_matches_oracle_file(tmp_path, world, ch, bits, n, maxf):
    """tests/cpp/sharded_encode_test.cpp: BASELINE config 4's path driven through the C ABI alone
    (no Python, no torch in the ranks): fork one process per GPU, flacgpu_comm_unique_id /
    flacgpu_comm_init / flacgpu_encode_frames_sharded, rank 0 assembles the file.  One rank per GPU:
    world > visible GPUs is skipped (RCCL refuses two ranks on one device)."""
    import os
    import subprocess

    if not _has_gpu() or __import__("torch").cuda.device_count() < world:
        pytest.skip(f"{world} rank(s) need {world} GPU(s)")
    subprocess.check_call(["make", "-s", "-C", CPP_DIR, "build/sharded_encode_test"])
    pcm = synth.synth_pcm(n, ch, bits, 44100)
    raw = tmp_path / "x.raw"
    raw.write_bytes(pcm)
    out = tmp_path / "o.flac"
    r = subprocess.run([os.path.join(CPP_DIR, "build", "sharded_encode_test"), str(raw), str(ch), str(bits), "44100",
                        str(world), str(maxf), str(out)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    assert out.read_bytes() == oracle_ref.encode_file(pcm, ch, bits, 44100)


@pytest.mark.parametrize("threads", ["1", "3"])
def test_host_md5_pool_matches_plain_chain(threads):
    """fg_md5_host.cpp's hashing pool (the file path's MD5 engine: up to eight callers' chains
    interleaved per worker; one worker holds all eight here) equals one plain chain per message, many callers at once, updates split
    at odd offsets (tests/cpp/md5_pool_test.cpp)."""
    import os
    import subprocess

    subprocess.check_call(["make", "-s", "-C", CPP_DIR, "build/md5_pool_test"])
    r = subprocess.run([os.path.join(CPP_DIR, "build", "md5_pool_test")], capture_output=True, text=True,
                       env=dict(os.environ, FLACGPU_MD5_THREADS=threads), timeout=120)
    assert r.returncode == 0 and r.stdout.strip() == "ok", r.stdout + r.stderr


@pytest.mark.gpu
@pytest.mark.parametrize("ch,bits,rate", [(2, 16, 44100), (2, 24, 96000)])
def test_concurrent_encode_file_share_the_device_pipeline(ch, bits, rate, monkeypatch):
    """flacgpu_encode_file from many threads, one context each (the reference's
    one-encoder-per-file shape, wav2flac.zig:10-63), runs through the device's shared file pipeline
    (fg_file.cpp); every file must still be byte-identical to the restatement's whole-file encode,
    including empty and sub-block files, and a caller with too small an output buffer gets
    WriteFailed without disturbing the others' files."""
    import ctypes
    import threading

    import flacgpu

    lens = [0, 1, 4095, 4096, 3 * 4096 + 7, 20 * 4096 + 333, 9000, 12 * 4096, 5, 2 * 4096 + 1, 40000, 7 * 4096]
    pcms = [synth.synth_pcm(n, ch, bits, rate, stream=i) for i, n in enumerate(lens)]
    encs = [flacgpu.Encoder(ch, bits, rate, max_frames=64) for _ in pcms]
    outs, errs = [None] * len(pcms), [None] * len(pcms)
    small = 5  # this caller's buffer is too small

    def run(i):
        try:
            if i == small:
                e = encs[i]
                n = lens[i]
                out = ctypes.create_string_buffer(100)
                ol = ctypes.c_size_t(0)
                errs[i] = e.lib.flacgpu_encode_file(e.ctx, pcms[i], e.bytes_per_sample, n, out, 100, ctypes.byref(ol))
            else:
                outs[i] = encs[i].encode_file(pcms[i])
        except Exception as ex:  # noqa: BLE001
            errs[i] = ex

    try:
        for _ in range(2):
            th = [threading.Thread(target=run, args=(i,)) for i in range(len(pcms))]
            for t in th:
                t.start()
            for t in th:
                t.join()
            assert errs[small] == -4, errs[small]  # FLACGPU_ERR_OUTPUT_TOO_SMALL
            for i, pcm in enumerate(pcms):
                if i == small:
                    continue
                assert errs[i] is None, errs[i]
                assert outs[i] == oracle_ref.encode_file(pcm, ch, bits, rate), f"file {i} ({lens[i]} samples)"
    finally:
        for e in encs:
            e.close()
