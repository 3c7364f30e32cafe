"""ctypes access to the CPU restatement (oracle/) and the verifier decoder.

Test infrastructure only: the oracle is the checker, never the thing under test.
"""
from __future__ import annotations

import ctypes
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "oracle", "build", "liboracle.so")
LIB_FAST = os.path.join(ROOT, "oracle", "build", "liboracle_fast.so")  # -O3 build: bench.py cpu_baseline only


class OConfig(ctypes.Structure):
    _fields_ = [("sample_rate", ctypes.c_uint32), ("block_size", ctypes.c_uint16), ("channels", ctypes.c_uint8),
                ("bits_per_sample", ctypes.c_uint8), ("stereo_decorrelation", ctypes.c_uint8),
                ("max_rice_part_order", ctypes.c_uint8), ("max_rice_param", ctypes.c_uint8),
                ("prediction", ctypes.c_uint8)]


class OSub(ctypes.Structure):
    _fields_ = [("type", ctypes.c_uint8), ("waste", ctypes.c_uint8), ("bits", ctypes.c_uint8),
                ("order", ctypes.c_uint8), ("part_order", ctypes.c_uint8), ("method", ctypes.c_uint8),
                ("wide", ctypes.c_uint8), ("ub_clamped", ctypes.c_uint8), ("estimate", ctypes.c_uint64),
                ("constant", ctypes.c_int64), ("params", ctypes.c_uint8 * 256),
                ("lpc_precision", ctypes.c_uint8), ("lpc_shift", ctypes.c_int8), ("pad2", ctypes.c_uint8 * 6),
                ("lpc_coefs", ctypes.c_int32 * 32)]


class ORec(ctypes.Structure):
    _fields_ = [("channel_code", ctypes.c_uint8), ("n_sub", ctypes.c_uint8), ("n_cand", ctypes.c_uint8),
                ("pad", ctypes.c_uint8), ("frame_bytes", ctypes.c_uint32), ("written", OSub * 8),
                ("cand", OSub * 8)]


_L = None
_LF = None


def lib(fast: bool = False):
    global _L, _LF
    if fast:
        if _LF is None:
            if not os.path.exists(LIB_FAST):
                import subprocess
                subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle")])
            _LF = ctypes.CDLL(LIB_FAST)
            _LF.oracle_encode_stream.restype = ctypes.c_long
            _LF.oracle_max_frame_bytes.restype = ctypes.c_size_t
        return _LF
    if _L is None:
        if not os.path.exists(LIB):
            import subprocess
            subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle")])
        L = ctypes.CDLL(LIB)
        L.oracle_crc8.restype = ctypes.c_uint8
        L.oracle_crc16.restype = ctypes.c_uint16
        L.oracle_crc16_bitwise.restype = ctypes.c_uint16
        L.oracle_encode_frame.restype = ctypes.c_long
        L.oracle_encode_stream.restype = ctypes.c_long
        L.oracle_encode_file.restype = ctypes.c_long
        L.oracle_rice_part_size.restype = ctypes.c_uint64
        L.oracle_rice_part_size.argtypes = [ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint64]
        L.oracle_best_order.restype = ctypes.c_int
        L.oracle_max_frame_bytes.restype = ctypes.c_size_t
        L.oracle_utf8_number.restype = ctypes.c_int
        L.oracle_utf8_number.argtypes = [ctypes.c_uint64, ctypes.c_char_p]
        L.fdec_frames_to_pcm.restype = ctypes.c_long
        _L = L
    return _L


def config(channels, bits, rate, block=4096, stereo=True, part_order=8, param=30, lpc=0):
    return OConfig(rate, block, channels, bits, 1 if stereo else 0, part_order, param, lpc)


def encode_stream(pcm: bytes, channels: int, bits: int, rate: int, block: int = 4096, first_frame: int = 0,
                  **kw):
    L = lib()
    B = bits // 8
    n = len(pcm) // (channels * B)
    nf = (n + block - 1) // block
    cfg = config(channels, bits, rate, block, **kw)
    cap = nf * L.oracle_max_frame_bytes(block, bits, channels) + 64
    out = ctypes.create_string_buffer(cap)
    fb = (ctypes.c_uint32 * max(nf, 1))()
    md5 = ctypes.create_string_buffer(16)
    r = L.oracle_encode_stream(ctypes.byref(cfg), pcm, B, ctypes.c_uint64(n), ctypes.c_uint64(first_frame), out,
                               ctypes.c_size_t(cap), fb, md5)
    if r < 0:
        raise RuntimeError(f"oracle_encode_stream failed {r}")
    return out.raw[:r], list(fb)[:nf], md5.raw


def encode_frame(planes, n: int, frame_number: int, channels: int, bits: int, rate: int, block: int = 4096, **kw):
    """planes: sequence of int32 numpy arrays (channels x >= n)."""
    import numpy as np

    L = lib()
    cfg = config(channels, bits, rate, block, **kw)
    arrs = [np.ascontiguousarray(np.asarray(p, dtype=np.int32)) for p in planes]
    ptrs = (ctypes.c_void_p * 8)(*[a.ctypes.data for a in arrs])
    cap = L.oracle_max_frame_bytes(max(n, 1), bits, channels) + 64
    out = ctypes.create_string_buffer(cap)
    rec = ORec()
    r = L.oracle_encode_frame(ctypes.byref(cfg), ptrs, n, ctypes.c_uint64(frame_number), out, ctypes.c_size_t(cap),
                              ctypes.byref(rec))
    if r < 0:
        raise RuntimeError(f"oracle_encode_frame failed {r}")
    return out.raw[:r], rec


def encode_file(pcm: bytes, channels: int, bits: int, rate: int, block: int = 4096, **kw):
    L = lib()
    B = bits // 8
    n = len(pcm) // (channels * B)
    cfg = config(channels, bits, rate, block, **kw)
    nf = (n + block - 1) // block
    cap = 200 + nf * L.oracle_max_frame_bytes(block, bits, channels)
    out = ctypes.create_string_buffer(cap)
    r = L.oracle_encode_file(ctypes.byref(cfg), pcm, B, ctypes.c_uint64(n), out, ctypes.c_size_t(cap))
    if r < 0:
        raise RuntimeError(f"oracle_encode_file failed {r}")
    return out.raw[:r]


def decode_frames(frames: bytes, channels: int, bits: int, rate: int, n_samples: int, first_number: int = 0):
    """Decode concatenated frames -> (pcm bytes, frame sizes).  Raises on any CRC/format error."""
    L = lib()
    B = bits // 8
    out = ctypes.create_string_buffer(max(n_samples * channels * B, 1))
    maxf = n_samples + 1
    sizes = (ctypes.c_uint32 * maxf)()
    r = L.fdec_frames_to_pcm(frames, ctypes.c_size_t(len(frames)), channels, bits, rate, B, out,
                             ctypes.c_uint64(n_samples), ctypes.c_uint64(first_number), sizes, ctypes.c_uint64(maxf))
    if r < 0:
        raise RuntimeError(f"decoder rejected the stream: code {r}")
    nf = 0
    while nf < maxf and sizes[nf]:
        nf += 1
    return out.raw[: r * channels * B], list(sizes)[:nf]
