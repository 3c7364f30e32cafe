"""ctypes binding of libflacgpu.so (include/flacgpu.h) for tests and the benchmark.

This is plumbing over the C ABI: every encode runs in the gfx950 HIP kernels
of libflacgpu.so.  There is no CPU fallback -- if the library or a gfx950
device is missing, construction raises.

The class names mirror the reference's Zig interface (src/lib.zig):
`Encoder.write_frame` is `Encoder.writeFrame` (src/lib/encoder.zig:234),
`Config.default` is `Config.default` (encoder.zig:642-655).
"""
from __future__ import annotations

import ctypes
import os
from typing import Optional, Sequence

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("FLACGPU_LIB", os.path.join(HERE, "build", "libflacgpu.so"))

OK = 0
ERRORS = {
    -1: "InvalidConfig",
    -2: "InvalidInput",
    -3: "OutOfMemory",
    -4: "WriteFailed (output too small)",
    -5: "DeviceError",
    -6: "InternalError",
}

K_ANALYZE, K_ANALYZE_TAIL, K_SCAN, K_PACK, K_MD5 = range(5)
MD5_HOST, MD5_DEVICE = 0, 1
KERNEL_NAMES = ["analyze", "analyze_tail", "scan", "pack", "md5"]


class FlacGpuError(RuntimeError):
    def __init__(self, code: int, where: str):
        super().__init__(f"{where}: {ERRORS.get(code, code)} ({code})")
        self.code = code


class Config(ctypes.Structure):
    """flacgpu_config == Encoder.Config + Feature (encoder.zig:609-656)."""

    _fields_ = [
        ("sample_rate", ctypes.c_uint32),
        ("block_size", ctypes.c_uint16),
        ("channels", ctypes.c_uint8),
        ("bits_per_sample", ctypes.c_uint8),
        ("stereo_decorrelation", ctypes.c_uint8),
        ("max_rice_part_order", ctypes.c_uint8),
        ("max_rice_param", ctypes.c_uint8),
        ("prediction", ctypes.c_uint8),
    ]

    @classmethod
    def default(cls, channels: int, bits: int, sample_rate: int) -> "Config":
        return cls(sample_rate, 4096, channels, bits, 1, 8, 30, 0)


class SubframeRecord(ctypes.Structure):
    _fields_ = [
        ("type", ctypes.c_uint8),
        ("waste", ctypes.c_uint8),
        ("bits", ctypes.c_uint8),
        ("order", ctypes.c_uint8),
        ("part_order", ctypes.c_uint8),
        ("method", ctypes.c_uint8),
        ("written", ctypes.c_uint8),
        ("pad", ctypes.c_uint8),
        ("pad2", ctypes.c_uint32),
        ("estimate", ctypes.c_uint64),
        ("constant", ctypes.c_int64),
        ("params", ctypes.c_uint8 * 256),
        ("lpc_precision", ctypes.c_uint8),
        ("lpc_shift", ctypes.c_int8),
        ("pad3", ctypes.c_uint8 * 6),
        ("lpc_coefs", ctypes.c_int32 * 32),
    ]


class FrameRecord(ctypes.Structure):
    _fields_ = [
        ("channel_code", ctypes.c_uint32),
        ("n_cand", ctypes.c_uint32),
        ("frame_bytes", ctypes.c_uint32),
        ("pad", ctypes.c_uint32),
        ("cand", SubframeRecord * 8),
    ]


class Md5State(ctypes.Structure):
    """flacgpu_md5_state: one stream's MD5 chaining value carried across calls."""
    _fields_ = [("h", ctypes.c_uint32 * 4), ("bytes", ctypes.c_uint64), ("finished", ctypes.c_uint32),
                ("reserved", ctypes.c_uint32)]


def md5_states(n: int) -> bytes:
    """n freshly initialised flacgpu_md5_state records (32 bytes each), ready to upload."""
    arr = (Md5State * max(n, 1))()
    load_library().flacgpu_md5_state_init(arr, n)
    return bytes(arr)[: 32 * n]


def md5_many(chunks: Sequence, final: Optional[Sequence[bool]] = None, states=None) -> list:
    """flacgpu_md5_many: advance len(chunks) independent MD5 chains on the library's host pool
    (md5.zig:3-31).  `states` (an (Md5State * n) array, or None for fresh chains) is updated in
    place; returns the digests (16 bytes each; None for a chain that is not final)."""
    import numpy as np

    n = len(chunks)
    views = [np.frombuffer(c, dtype=np.uint8) if len(c) else np.zeros(1, np.uint8) for c in chunks]
    ptrs = (ctypes.c_void_p * max(n, 1))(*[v.ctypes.data for v in views])
    lens = (ctypes.c_uint64 * max(n, 1))(*[len(c) for c in chunks])
    fin = (ctypes.c_uint8 * max(n, 1))(*[1 if f else 0 for f in final]) if final is not None else None
    dig = (ctypes.c_uint8 * max(16 * n, 1))()
    _check(load_library().flacgpu_md5_many(n, ptrs, lens, fin, states, dig), "md5_many")
    raw = bytes(dig)
    return [raw[16 * i:16 * i + 16] if final is None or final[i] else None for i in range(n)]


class Md5Rates(ctypes.Structure):
    """flacgpu_md5_rates: the rates the MD5 engine choice is priced with (bytes/s)."""
    _fields_ = [("host_chain", ctypes.c_double * 4), ("host_chains", ctypes.c_uint32 * 4), ("device_lane", ctypes.c_double),
                ("device_chip", ctypes.c_double), ("host_workers", ctypes.c_int32), ("measured", ctypes.c_int32)]

    def as_dict(self) -> dict:
        return {"host_chain": list(self.host_chain), "host_chains": list(self.host_chains), "device_lane": self.device_lane, "device_chip": self.device_chip,
                "host_workers": self.host_workers, "measured": self.measured}


def md5_rates() -> Md5Rates:
    r = Md5Rates()
    _check(load_library().flacgpu_md5_get_rates(ctypes.byref(r)), "md5_get_rates")
    return r


def set_md5_rates(r: Optional[Md5Rates]) -> None:
    _check(load_library().flacgpu_md5_set_rates(ctypes.byref(r) if r is not None else None), "md5_set_rates")


def md5_engine_for(n_streams: int, max_len: int, total_len: int) -> int:
    return int(load_library().flacgpu_md5_engine_for(n_streams, max_len, total_len))


class WavInfo(ctypes.Structure):
    """flacgpu_wav_info: WavReader's view of a WAV header (wav_reader.zig:116-170)."""
    _fields_ = [("sample_rate", ctypes.c_uint32), ("channels", ctypes.c_uint16), ("bits_per_sample", ctypes.c_uint16),
                ("bytes_per_sample", ctypes.c_uint16), ("pad", ctypes.c_uint16), ("samples", ctypes.c_uint64),
                ("data_offset", ctypes.c_uint64), ("data_bytes", ctypes.c_uint64)]


class StreamInfo(ctypes.Structure):
    """flacgpu_streaminfo == metadata.StreamInfo (metadata.zig:18-33)."""
    _fields_ = [("md5", ctypes.c_uint8 * 16), ("interchannel_samples", ctypes.c_uint64),
                ("min_frame_size", ctypes.c_uint32), ("max_frame_size", ctypes.c_uint32),
                ("sample_rate", ctypes.c_uint32), ("min_block_size", ctypes.c_uint16),
                ("max_block_size", ctypes.c_uint16), ("channels", ctypes.c_uint8), ("bit_depth", ctypes.c_uint8),
                ("pad", ctypes.c_uint8 * 6)]

    def update_frame_size(self, size: int) -> None:
        load_library().flacgpu_streaminfo_update_frame_size(ctypes.byref(self), size)

    def bytes(self) -> bytes:
        out = ctypes.create_string_buffer(34)
        load_library().flacgpu_streaminfo_bytes(ctypes.byref(self), out)
        return out.raw

    @classmethod
    def new(cls, sample_rate: int, channels: int, bit_depth: int, samples: int, block_size: int = 4096):
        si = cls()
        load_library().flacgpu_streaminfo_init(ctypes.byref(si), sample_rate, channels, bit_depth, samples, block_size)
        return si


def wav_parse(wav: bytes) -> WavInfo:
    info = WavInfo()
    _check(load_library().flacgpu_wav_parse(wav, len(wav), ctypes.byref(info)), "wav_parse")
    return info


def header_bytes(si: StreamInfo, last: bool) -> bytes:
    out = ctypes.create_string_buffer(42)
    n = load_library().flacgpu_header_bytes(ctypes.byref(si), 1 if last else 0, out)
    return out.raw[:n]


def vorbis_comment_bytes(last: bool) -> bytes:
    out = ctypes.create_string_buffer(31)
    n = load_library().flacgpu_vorbis_comment_bytes(1 if last else 0, out)
    return out.raw[:n]


def wav_to_flac(wav: bytes, device: int = 0) -> bytes:
    """wav2flac (wav2flac.zig:10-97) of an in-memory WAV file on the GPU."""
    info = wav_parse(wav)
    cfg = Config.default(info.channels, info.bits_per_sample, info.sample_rate)
    cap = 200 + ((info.samples + 4095) // 4096 + 1) * load_library().flacgpu_frame_bound_bytes(ctypes.byref(cfg))
    out = ctypes.create_string_buffer(cap)
    n = ctypes.c_size_t(0)
    _check(load_library().flacgpu_wav_to_flac(device, wav, len(wav), out, cap, ctypes.byref(n)), "wav_to_flac")
    return out.raw[: n.value]


class Comm:
    """flacgpu_comm: one rank of a multi-GPU communicator (RCCL over xGMI inside libflacgpu.so):
    the bitstream gather of the sharded encode (wav2flac.zig:66-97 cut into
    ranks, updateFrameSize replayed in frame order on rank 0, metadata.zig:35-40)."""

    ID_BYTES = 128

    def __init__(self, comm_id: bytes, world: int, rank: int, device: int):
        self.world, self.rank, self.device = world, rank, device
        self.comm = ctypes.c_void_p()
        cid = (ctypes.c_uint8 * self.ID_BYTES).from_buffer_copy(comm_id)
        _check(load_library().flacgpu_comm_init(cid, world, rank, device, ctypes.byref(self.comm)), "comm_init")

    @staticmethod
    def unique_id() -> bytes:
        cid = (ctypes.c_uint8 * Comm.ID_BYTES)()
        _check(load_library().flacgpu_comm_unique_id(cid), "comm_unique_id")
        return bytes(cid)

    @classmethod
    def from_process_group(cls, dist, group=None, device: int = 0) -> "Comm":
        """Rank 0 of `group` makes the id, torch.distributed hands it to every rank (any backend)."""
        rank = dist.get_rank(group)
        box = [cls.unique_id() if rank == 0 else None]
        dist.broadcast_object_list(box, src=dist.get_global_rank(group, 0) if group is not None else 0, group=group)
        return cls(box[0], dist.get_world_size(group), rank, device)

    def gather_device(self, d_frames: int, nbytes: int, d_sizes: int, n_frames: int, d_recv: int = 0,
                      recv_cap: int = 0, d_recv_sizes: int = 0, recv_sizes_cap: int = 0, d_nbytes: int = 0,
                      stream=None):
        """flacgpu_gather_frames_device -> (total bytes, total frames) gathered on rank 0."""
        tb, tf = ctypes.c_uint64(0), ctypes.c_uint64(0)
        _check(load_library().flacgpu_gather_frames_device(
            self.comm, d_frames or None, nbytes, d_nbytes or None, d_sizes or None, n_frames, d_recv or None,
            recv_cap, d_recv_sizes or None, recv_sizes_cap, ctypes.byref(tb), ctypes.byref(tf), stream),
            "gather_frames_device")
        return tb.value, tf.value

    def encode_frames_sharded(self, enc, pcm: bytes, first_frame: int = 0):
        """flacgpu_encode_frames_sharded: every rank passes the whole stream; rank 0 gets (frames,
        sizes) exactly as flacgpu_encode_frames would write them, the others (b"", [])."""
        B = enc.bits // 8
        n = len(pcm) // (enc.channels * B)
        nf = (n + enc.block_size - 1) // enc.block_size
        cap = max(nf, 1) * enc.frame_bound() + 64 if self.rank == 0 else 0
        out = ctypes.create_string_buffer(max(cap, 1))
        fb = (ctypes.c_uint32 * max(nf, 1))()
        n_out = ctypes.c_size_t(0)
        _check(load_library().flacgpu_encode_frames_sharded(enc.ctx, self.comm, pcm, B, n, first_frame, out, cap,
                                                            ctypes.byref(n_out), fb), "encode_frames_sharded")
        if self.rank != 0:
            return b"", []
        return out.raw[: n_out.value], list(fb)[:nf]

    def close(self):
        if self.comm:
            load_library().flacgpu_comm_destroy(self.comm)
            self.comm = ctypes.c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


_lib = None


def load_library(path: str = LIB_PATH) -> ctypes.CDLL:
    """Load libflacgpu.so; raise (never fall back) if it is absent."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise FileNotFoundError(f"{path} not built: run `make -C zig-flac_amd` (or __graft_entry__.build())")
    # PyTorch-ROCm bundles its own HIP/HSA runtime under the same SONAME (libamdhip64.so.7).
    # Loaded first, it is the one libflacgpu.so binds to, so device pointers and streams of
    # torch tensors and of this library share one runtime.  Loaded after /opt/rocm's copy,
    # it would start a second HSA runtime on the same device, which fails to initialise
    # ("No HIP GPUs are available").  So torch, when present, is imported before the library.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    L = ctypes.CDLL(path)
    P, U32, U64, I32, SZ = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_int, ctypes.c_size_t
    sig = {
        "flacgpu_config_default": (Config, [U32, U32, U32]),
        "flacgpu_open": (I32, [I32, ctypes.POINTER(Config), U32, ctypes.POINTER(P)]),
        "flacgpu_close": (None, [P]),
        "flacgpu_strerror": (ctypes.c_char_p, [I32]),
        "flacgpu_abi_version": (I32, []),
        "flacgpu_build_flags": (U32, []),
        "flacgpu_md5_get_rates": (I32, [P]),
        "flacgpu_md5_set_rates": (I32, [P]),
        "flacgpu_md5_engine_for": (I32, [U32, U64, U64]),
        "flacgpu_reference_max_frame_bytes": (SZ, [ctypes.POINTER(Config)]),
        "flacgpu_frame_bound_bytes": (SZ, [ctypes.POINTER(Config)]),
        "flacgpu_encode_frames": (I32, [P, P, U32, U64, U64, P, SZ, ctypes.POINTER(SZ), P]),
        "flacgpu_encode_frame_planar": (I32, [P, P, U32, U64, P, SZ, ctypes.POINTER(U32)]),
        "flacgpu_md5_init": (I32, [P]),
        "flacgpu_md5_update": (I32, [P, P, SZ]),
        "flacgpu_md5_final": (I32, [P, P]),
        "flacgpu_plan_create": (I32, [P, U32, P, P, U32, ctypes.POINTER(P)]),
        "flacgpu_plan_create_segments": (I32, [P, U32, P, P, U32, P, P, ctypes.POINTER(P)]),
        "flacgpu_plan_advance": (I32, [P, U64, P]),
        "flacgpu_encode_plan_device_ex": (I32, [P, P, P, P, U64, P, P, P, P, P, P, P]),
        "flacgpu_sync_check": (I32, [P, P]),
        "flacgpu_streaminfo_replay_device": (I32, [P, P, U64, P, P]),
        "flacgpu_md5_set_engine": (I32, [P, I32]),
        "flacgpu_md5_get_engine": (I32, [P]),
        "flacgpu_md5_state_init": (None, [P, SZ]),
        "flacgpu_md5_many": (I32, [U32, P, P, P, P, P]),
        "flacgpu_md5_plan_host": (I32, [P, P, P, P]),
        "flacgpu_plan_md5_engine": (I32, [P]),
        "flacgpu_plan_destroy": (None, [P]),
        "flacgpu_plan_frames": (U64, [P]),
        "flacgpu_plan_out_bound": (U64, [P]),
        "flacgpu_plan_stream_first_frame": (U64, [P, U32]),
        "flacgpu_encode_plan_device": (I32, [P, P, P, P, U64, P, P, P, P, P]),
        "flacgpu_encode_plan_device_md5_async": (I32, [P, P, P, P, U64, P, P, P, P, P, P]),
        "flacgpu_set_timing": (I32, [P, I32]),
        "flacgpu_kernel_time": (I32, [P, I32, ctypes.POINTER(U64), ctypes.POINTER(ctypes.c_double)]),
        "flacgpu_reset_timing": (I32, [P]),
        "flacgpu_set_records": (I32, [P, I32]),
        "flacgpu_set_overlap": (I32, [P, U32, U32, U32, U32]),
        "flacgpu_get_records": (I32, [P, P, U64, ctypes.POINTER(U64)]),
        "flacgpu_get_config": (I32, [P, ctypes.POINTER(Config)]),
        "flacgpu_wav_parse": (I32, [P, SZ, ctypes.POINTER(WavInfo)]),
        "flacgpu_streaminfo_init": (None, [ctypes.POINTER(StreamInfo), U32, U32, U32, U64, U32]),
        "flacgpu_streaminfo_update_frame_size": (None, [ctypes.POINTER(StreamInfo), U32]),
        "flacgpu_streaminfo_bytes": (None, [ctypes.POINTER(StreamInfo), P]),
        "flacgpu_header_bytes": (SZ, [ctypes.POINTER(StreamInfo), I32, P]),
        "flacgpu_vorbis_comment_bytes": (SZ, [I32, P]),
        "flacgpu_encode_file": (I32, [P, P, U32, U64, P, SZ, ctypes.POINTER(SZ)]),
        "flacgpu_encode_files": (I32, [P, U32, P, U32, P, P, P, P]),
        "flacgpu_wav_to_flac": (I32, [I32, P, SZ, P, SZ, ctypes.POINTER(SZ)]),
        "flacgpu_open_multi": (I32, [I32, P, ctypes.POINTER(Config), U32, ctypes.POINTER(P)]),
        "flacgpu_close_multi": (None, [P]),
        "flacgpu_multi_encode_frames": (I32, [P, P, U32, U64, U64, P, SZ, ctypes.POINTER(SZ), P]),
        "flacgpu_comm_unique_id": (I32, [P]),
        "flacgpu_comm_init": (I32, [P, I32, I32, I32, ctypes.POINTER(P)]),
        "flacgpu_comm_destroy": (None, [P]),
        "flacgpu_comm_rank": (I32, [P]),
        "flacgpu_comm_size": (I32, [P]),
        "flacgpu_gather_frames_device": (I32, [P, P, U64, P, P, U64, P, U64, P, U64, ctypes.POINTER(U64),
                                               ctypes.POINTER(U64), P]),
        "flacgpu_encode_frames_sharded": (I32, [P, P, P, U32, U64, U64, P, SZ, ctypes.POINTER(SZ), P]),
    }
    # an older build named by FLACGPU_LIB (same-box A/B runs, tools/ab.sh) may predate later entry
    # points: those stay unbound there; the in-tree library must export every one
    other_build = path != os.path.join(HERE, "build", "libflacgpu.so")
    for name, (res, args) in sig.items():
        if other_build and not hasattr(L, name):
            continue
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    _lib = L
    return L


def exported_symbols() -> list:
    return [
        "flacgpu_config_default", "flacgpu_open", "flacgpu_close", "flacgpu_strerror", "flacgpu_abi_version",
        "flacgpu_build_flags", "flacgpu_md5_get_rates", "flacgpu_md5_set_rates", "flacgpu_md5_engine_for",
        "flacgpu_reference_max_frame_bytes", "flacgpu_frame_bound_bytes", "flacgpu_encode_frames",
        "flacgpu_encode_frame_planar", "flacgpu_md5_init", "flacgpu_md5_update", "flacgpu_md5_final",
        "flacgpu_plan_create", "flacgpu_plan_destroy", "flacgpu_plan_frames", "flacgpu_plan_out_bound",
        "flacgpu_plan_stream_first_frame", "flacgpu_encode_plan_device", "flacgpu_encode_plan_device_md5_async",
        "flacgpu_plan_create_segments", "flacgpu_plan_advance", "flacgpu_encode_plan_device_ex", "flacgpu_sync_check",
        "flacgpu_streaminfo_replay_device",
        "flacgpu_md5_set_engine", "flacgpu_md5_get_engine", "flacgpu_md5_state_init",
        "flacgpu_md5_many", "flacgpu_md5_plan_host", "flacgpu_plan_md5_engine",
        "flacgpu_set_timing",
        "flacgpu_kernel_time", "flacgpu_reset_timing", "flacgpu_set_records", "flacgpu_set_overlap", "flacgpu_get_records",
        "flacgpu_get_config", "flacgpu_wav_parse", "flacgpu_streaminfo_init", "flacgpu_streaminfo_update_frame_size",
        "flacgpu_streaminfo_bytes", "flacgpu_header_bytes", "flacgpu_vorbis_comment_bytes", "flacgpu_encode_file", "flacgpu_encode_files",
        "flacgpu_wav_to_flac", "flacgpu_open_multi", "flacgpu_close_multi", "flacgpu_multi_encode_frames",
        "flacgpu_comm_unique_id", "flacgpu_comm_init", "flacgpu_comm_destroy", "flacgpu_comm_rank",
        "flacgpu_comm_size", "flacgpu_gather_frames_device", "flacgpu_encode_frames_sharded",
    ]


BUILD_DIAG = 1  # FLACGPU_BUILD_DIAG
BUILD_STAMPS = 2  # FLACGPU_BUILD_STAMPS


def build_flags() -> int:
    """flacgpu_build_flags(): BUILD_DIAG for a diagnostic build (`make diag`), else 0."""
    L = load_library()
    return int(L.flacgpu_build_flags()) if hasattr(L, "flacgpu_build_flags") else BUILD_DIAG


def diag_build() -> bool:
    return bool(build_flags() & BUILD_DIAG)


STREAM_LEGACY = 1  # FLACGPU_STREAM_LEGACY: the library maps it to the HIP null stream


def _stream(h: Optional[int]) -> Optional[int]:
    """A torch/HIP stream handle as the C ABI's `void *hip_stream`: None -> NULL (the context's
    own non-blocking stream); 0 (the legacy null stream, torch's default) -> FLACGPU_STREAM_LEGACY,
    so the work stays ordered against default-stream producers and consumers."""
    if h is None:
        return None
    return STREAM_LEGACY if h == 0 else h


def _check(rc: int, where: str) -> None:
    if rc != OK:
        raise FlacGpuError(rc, where)


class Plan:
    """flacgpu_plan: a batch of streams (or stream segments) laid out in one device PCM buffer."""

    def __init__(self, enc: "Encoder", offsets: Sequence[int], samples: Sequence[int],
                 first_frames: Optional[Sequence[int]] = None, final: Optional[Sequence[bool]] = None):
        self.enc = enc
        n = len(offsets)
        self._offs = (ctypes.c_uint64 * max(n, 1))(*offsets)
        self._samp = (ctypes.c_uint64 * max(n, 1))(*samples)
        ff = (ctypes.c_uint64 * max(n, 1))(*first_frames) if first_frames is not None else None
        fin = (ctypes.c_uint8 * max(n, 1))(*[1 if f else 0 for f in final]) if final is not None else None
        h = ctypes.c_void_p()
        _check(enc.lib.flacgpu_plan_create_segments(enc.ctx, n, self._offs, self._samp, enc.bytes_per_sample, ff, fin,
                                                    ctypes.byref(h)), "plan_create_segments")
        self.handle = h
        self.n_streams = n
        self.n_frames = enc.lib.flacgpu_plan_frames(h)
        self.out_bound = enc.lib.flacgpu_plan_out_bound(h)
        self.first_frame = [enc.lib.flacgpu_plan_stream_first_frame(h, s) for s in range(n)]

    def advance(self, frames: int, stream: Optional[int] = None) -> None:
        """flacgpu_plan_advance: the next window of the same streams (frame numbers + frames)."""
        _check(self.enc.lib.flacgpu_plan_advance(self.handle, frames, _stream(stream)), "plan_advance")

    def md5_engine(self) -> int:
        """flacgpu_plan_md5_engine: MD5_HOST below the stream-count crossover, else MD5_DEVICE."""
        return self.enc.lib.flacgpu_plan_md5_engine(self.handle)

    def md5_host(self, h_pcm: int, states=None, digests: Optional[int] = None) -> None:
        """flacgpu_md5_plan_host: every segment's MD5 on the host pool from the host copy h_pcm
        (address; same offsets as the device buffer), states/digests in host memory."""
        _check(self.enc.lib.flacgpu_md5_plan_host(self.handle, h_pcm, states, digests), "md5_plan_host")

    def close(self) -> None:
        if self.handle:
            self.enc.lib.flacgpu_plan_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Encoder:
    """GPU block encoder context == Encoder.init / deinit (encoder.zig:44-164)."""

    def __init__(self, channels: int, bits: int, sample_rate: int, device: int = 0, max_frames: int = 32768,
                 block_size: int = 4096, stereo_decorrelation: bool = True, max_rice_part_order: int = 8,
                 max_rice_param: int = 30, lpc_order: int = 0):
        self.lib = load_library()
        self.cfg = Config(sample_rate, block_size, channels, bits, 1 if stereo_decorrelation else 0,
                          max_rice_part_order, max_rice_param, lpc_order)
        self.channels, self.bits, self.sample_rate, self.block_size = channels, bits, sample_rate, block_size
        self.bytes_per_sample = bits // 8
        self.max_frames = max_frames
        h = ctypes.c_void_p()
        _check(self.lib.flacgpu_open(device, ctypes.byref(self.cfg), max_frames, ctypes.byref(h)), "open")
        self.ctx = h

    def close(self) -> None:
        if getattr(self, "ctx", None):
            self.lib.flacgpu_close(self.ctx)
            self.ctx = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---- bounds
    def frame_bound(self) -> int:
        return self.lib.flacgpu_frame_bound_bytes(ctypes.byref(self.cfg))

    def reference_max_frame_bytes(self) -> int:
        return self.lib.flacgpu_reference_max_frame_bytes(ctypes.byref(self.cfg))

    # ---- encode
    def encode_frames(self, pcm: bytes, first_frame: int = 0):
        """Encode interleaved LE PCM -> (frame bytes, [per-frame sizes])."""
        per = self.channels * self.bytes_per_sample
        assert len(pcm) % per == 0
        n = len(pcm) // per
        nf = (n + self.block_size - 1) // self.block_size
        cap = nf * self.frame_bound() + 64
        out = ctypes.create_string_buffer(cap)
        sizes = (ctypes.c_uint32 * max(nf, 1))()
        out_len = ctypes.c_size_t(0)
        src = ctypes.create_string_buffer(bytes(pcm), len(pcm)) if pcm else None
        _check(self.lib.flacgpu_encode_frames(self.ctx, src, self.bytes_per_sample, n, first_frame, out, cap,
                                              ctypes.byref(out_len), sizes), "encode_frames")
        return out.raw[: out_len.value], list(sizes)[:nf]

    def encode_file(self, pcm: bytes) -> bytes:
        """Whole .flac file (73-byte header + frames) for interleaved LE PCM (wav2flac.zig:10-97)."""
        per = self.channels * self.bytes_per_sample
        n = len(pcm) // per
        nf = (n + self.block_size - 1) // self.block_size
        cap = 200 + nf * self.frame_bound()
        out = ctypes.create_string_buffer(cap)
        out_len = ctypes.c_size_t(0)
        src = ctypes.create_string_buffer(bytes(pcm), len(pcm)) if pcm else None
        _check(self.lib.flacgpu_encode_file(self.ctx, src, self.bytes_per_sample, n, out, cap, ctypes.byref(out_len)),
               "encode_file")
        return out.raw[: out_len.value]

    def encode_files(self, pcms: Sequence[bytes]) -> list:
        """flacgpu_encode_files: encode_file of every buffer, in one call (one pipelined schedule,
        the MD5s batched on the host pool)."""
        per = self.channels * self.bytes_per_sample
        n = len(pcms)
        ns = [len(p) // per for p in pcms]
        caps = [200 + ((k + self.block_size - 1) // self.block_size) * self.frame_bound() for k in ns]
        outs = [ctypes.create_string_buffer(c) for c in caps]
        srcs = [ctypes.create_string_buffer(bytes(p), len(p)) if p else None for p in pcms]
        src_p = (ctypes.c_void_p * max(n, 1))(*[ctypes.cast(b, ctypes.c_void_p).value if b is not None else None
                                                 for b in srcs])
        out_p = (ctypes.c_void_p * max(n, 1))(*[ctypes.cast(b, ctypes.c_void_p).value for b in outs])
        ns_a = (ctypes.c_uint64 * max(n, 1))(*ns)
        cap_a = (ctypes.c_size_t * max(n, 1))(*caps)
        len_a = (ctypes.c_size_t * max(n, 1))()
        _check(self.lib.flacgpu_encode_files(self.ctx, n, src_p, self.bytes_per_sample, ns_a, out_p, cap_a, len_a),
               "encode_files")
        return [outs[i].raw[: len_a[i]] for i in range(n)]

    def write_frame(self, planes, frame_number: int) -> bytes:
        """Encoder.writeFrame: planar int32 samples (C x n) -> one frame."""
        import numpy as np

        planes = np.ascontiguousarray(np.asarray(planes, dtype=np.int32))
        C, n = planes.shape
        assert C == self.channels
        ptrs = (ctypes.c_void_p * 8)()
        for c in range(C):
            ptrs[c] = planes[c].ctypes.data
        cap = self.frame_bound() + 64
        out = ctypes.create_string_buffer(cap)
        fb = ctypes.c_uint32(0)
        _check(self.lib.flacgpu_encode_frame_planar(self.ctx, ptrs, n, frame_number, out, cap, ctypes.byref(fb)),
               "encode_frame_planar")
        return out.raw[: fb.value]

    # ---- MD5 (md5.zig): the context's engine (host core by default, one GPU lane opt-in)
    def set_md5_engine(self, engine: int) -> None:
        _check(self.lib.flacgpu_md5_set_engine(self.ctx, engine), "md5_set_engine")

    def md5_engine(self) -> int:
        e = self.lib.flacgpu_md5_get_engine(self.ctx)
        if e < 0:
            raise FlacGpuError(e, "md5_get_engine")
        return e

    def md5(self, data: bytes) -> bytes:
        _check(self.lib.flacgpu_md5_init(self.ctx), "md5_init")
        buf = ctypes.create_string_buffer(bytes(data), len(data))
        _check(self.lib.flacgpu_md5_update(self.ctx, buf, len(data)), "md5_update")
        d = ctypes.create_string_buffer(16)
        _check(self.lib.flacgpu_md5_final(self.ctx, d), "md5_final")
        return d.raw

    def md5_update(self, data: bytes) -> None:
        buf = ctypes.create_string_buffer(bytes(data), len(data))
        _check(self.lib.flacgpu_md5_update(self.ctx, buf, len(data)), "md5_update")

    def md5_final(self) -> bytes:
        d = ctypes.create_string_buffer(16)
        _check(self.lib.flacgpu_md5_final(self.ctx, d), "md5_final")
        return d.raw

    # ---- device-resident batches
    def plan(self, offsets: Sequence[int], samples: Sequence[int], first_frames: Optional[Sequence[int]] = None,
             final: Optional[Sequence[bool]] = None) -> Plan:
        return Plan(self, offsets, samples, first_frames, final)

    def encode_plan_device_ex(self, plan: Plan, d_pcm: int, d_out: int, out_cap: int, d_frame_bytes: int,
                              d_frame_offsets: int, d_total: int, d_md5_state: Optional[int] = None,
                              d_md5: Optional[int] = None, stream: Optional[int] = None,
                              md5_stream: Optional[int] = None) -> None:
        """flacgpu_encode_plan_device_ex: MD5 state carried in d_md5_state (32 B per stream).
        md5_stream None: the MD5 is joined back into `stream`; any handle (0 = the legacy null
        stream) queues it there unjoined, as in encode_plan_device."""
        _check(self.lib.flacgpu_encode_plan_device_ex(
            self.ctx, plan.handle, d_pcm, d_out, out_cap, d_frame_bytes, d_frame_offsets, d_total,
            d_md5_state or None, d_md5 or None, _stream(stream), _stream(md5_stream)), "encode_plan_device_ex")

    def sync_check(self, stream: Optional[int] = None) -> None:
        """Synchronise `stream` and raise if a kernel flagged a device-side error."""
        _check(self.lib.flacgpu_sync_check(self.ctx, _stream(stream)), "sync_check")

    def streaminfo_replay_device(self, d_frame_bytes: int, n_frames: int, d_minmax: int,
                                 stream: Optional[int] = None) -> None:
        """StreamInfo.updateFrameSize (metadata.zig:35-40) over device frame sizes; d_minmax = u32
        {min, max} in/out on the device ({0xFFFFFF, 0} for a new stream)."""
        _check(self.lib.flacgpu_streaminfo_replay_device(self.ctx, d_frame_bytes, n_frames, d_minmax,
                                                         _stream(stream)), "streaminfo_replay_device")

    def encode_frames_device(self, d_pcm: int, n_samples: int, first_frame: int = 0, stream: Optional[int] = None):
        """Frames of n_samples interleaved samples at device address d_pcm, numbered from first_frame, kept in
        device memory: returns (torch uint8 tensor of the bitstream, torch int32 tensor of frame sizes)."""
        import torch

        dev = torch.device("cuda", torch.cuda.current_device())
        plan = self.plan([0], [n_samples], first_frames=[first_frame])
        try:
            d_out = torch.empty(max(int(plan.out_bound), 1), dtype=torch.uint8, device=dev)
            d_fb = torch.empty(max(int(plan.n_frames), 1), dtype=torch.int32, device=dev)
            d_off = torch.empty(max(int(plan.n_frames), 1), dtype=torch.int64, device=dev)
            d_tot = torch.zeros(2, dtype=torch.int64, device=dev)
            st = stream if stream is not None else torch.cuda.current_stream(dev).cuda_stream
            self.encode_plan_device_ex(plan, d_pcm, d_out.data_ptr(), int(plan.out_bound), d_fb.data_ptr(),
                                       d_off.data_ptr(), d_tot.data_ptr(), stream=st)
            self.sync_check(st)
            total = int(d_tot[0].item())
            return d_out[:total], d_fb[: int(plan.n_frames)]
        finally:
            plan.close()

    def encode_plan_device(self, plan: Plan, d_pcm: int, d_out: int, out_cap: int, d_frame_bytes: int,
                           d_frame_offsets: int, d_total: int, d_md5: Optional[int] = None,
                           stream: Optional[int] = None, md5_stream: Optional[int] = None) -> None:
        """md5_stream: queue the MD5 there without joining it back into `stream` (the caller
        synchronises it); None joins it (flacgpu_encode_plan_device).  As in encode_plan_device_ex,
        only None means "joined": a handle of 0 is the legacy null stream (_stream), like any
        other stream handle."""
        if md5_stream is not None:
            _check(self.lib.flacgpu_encode_plan_device_md5_async(
                self.ctx, plan.handle, d_pcm, d_out, out_cap, d_frame_bytes, d_frame_offsets, d_total,
                d_md5 or None, _stream(stream), _stream(md5_stream)), "encode_plan_device_md5_async")
            return
        _check(self.lib.flacgpu_encode_plan_device(self.ctx, plan.handle, d_pcm, d_out, out_cap, d_frame_bytes,
                                                   d_frame_offsets, d_total, d_md5 or None, _stream(stream)),
               "encode_plan_device")

    # ---- instrumentation
    def set_timing(self, on: bool) -> None:
        _check(self.lib.flacgpu_set_timing(self.ctx, 1 if on else 0), "set_timing")

    def reset_timing(self) -> None:
        _check(self.lib.flacgpu_reset_timing(self.ctx), "reset_timing")

    def kernel_time(self, k: int):
        n = ctypes.c_uint64(0)
        ms = ctypes.c_double(0)
        _check(self.lib.flacgpu_kernel_time(self.ctx, k, ctypes.byref(n), ctypes.byref(ms)), "kernel_time")
        return n.value, ms.value

    def set_overlap(self, ranges: int, ana_per_cu: int = 2, pack_per_cu: int = 2, min_frames: int = 4096) -> None:
        """Encode schedule (flacgpu_set_overlap): ranges > 1 overlaps the analysis of range i+1 with the
        scan + pack of range i on a second HIP stream; output bytes are unchanged."""
        _check(self.lib.flacgpu_set_overlap(self.ctx, ranges, ana_per_cu, pack_per_cu, min_frames), "set_overlap")

    def set_records(self, on: bool) -> None:
        _check(self.lib.flacgpu_set_records(self.ctx, 1 if on else 0), "set_records")

    def records(self) -> list:
        n = ctypes.c_uint64(0)
        _check(self.lib.flacgpu_get_records(self.ctx, None, 0, ctypes.byref(n)), "get_records")
        arr = (FrameRecord * max(n.value, 1))()
        _check(self.lib.flacgpu_get_records(self.ctx, arr, n.value, ctypes.byref(n)), "get_records")
        return list(arr)[: n.value]


class MultiEncoder:
    """One input's frames sharded over several GPUs of this process (flacgpu_open_multi):
    contiguous frame ranges encoded concurrently, concatenated in frame order."""

    def __init__(self, devices: Sequence[int], channels: int, bits: int, sample_rate: int, max_frames: int = 32768,
                 block_size: int = 4096):
        self.lib = load_library()
        self.cfg = Config(sample_rate, block_size, channels, bits, 1, 8, 30, 0)
        self.channels, self.bytes_per_sample, self.block_size = channels, bits // 8, block_size
        devs = (ctypes.c_int * len(devices))(*devices)
        h = ctypes.c_void_p()
        _check(self.lib.flacgpu_open_multi(len(devices), devs, ctypes.byref(self.cfg), max_frames, ctypes.byref(h)),
               "open_multi")
        self.m = h

    def close(self) -> None:
        if getattr(self, "m", None):
            self.lib.flacgpu_close_multi(self.m)
            self.m = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def encode_frames(self, pcm: bytes, first_frame: int = 0):
        per = self.channels * self.bytes_per_sample
        n = len(pcm) // per
        nf = (n + self.block_size - 1) // self.block_size
        cap = nf * self.lib.flacgpu_frame_bound_bytes(ctypes.byref(self.cfg)) + 64
        out = ctypes.create_string_buffer(cap)
        sizes = (ctypes.c_uint32 * max(nf, 1))()
        out_len = ctypes.c_size_t(0)
        src = ctypes.create_string_buffer(bytes(pcm), len(pcm)) if pcm else None
        _check(self.lib.flacgpu_multi_encode_frames(self.m, src, self.bytes_per_sample, n, first_frame, out, cap,
                                                    ctypes.byref(out_len), sizes), "multi_encode_frames")
        return out.raw[: out_len.value], list(sizes)[:nf]
