"""The C-ABI library: loads, exports every symbol include/flacgpu.h declares,
validates configs, and refuses to run without a gfx950 device (no CPU fallback).
No compute calls here (CPU-only container)."""
import ctypes
import os
import re

import pytest

import flacgpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_functions():
    text = open(os.path.join(ROOT, "include", "flacgpu.h")).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(flacgpu_[a-z0-9_]+)\s*\(", text)))


def test_library_exports_every_declared_symbol():
    lib = flacgpu.load_library()
    declared = header_functions()
    assert len(declared) >= 20
    for name in declared:
        assert hasattr(lib, name), f"{name} declared in flacgpu.h but not exported"
    assert sorted(flacgpu.exported_symbols()) == declared


def test_abi_version():
    assert flacgpu.load_library().flacgpu_abi_version() == 5


def test_config_default_matches_reference():
    c = flacgpu.load_library().flacgpu_config_default(2, 16, 44100)
    # Config.default (encoder.zig:642-655)
    assert (c.block_size, c.stereo_decorrelation, c.max_rice_part_order, c.max_rice_param, c.prediction) == \
        (4096, 1, 8, 30, 0)


def test_reference_max_frame_bytes():
    import oracle_ref

    lib = flacgpu.load_library()
    for ch, bits in [(1, 16), (2, 16), (2, 24), (2, 32), (8, 24), (3, 8)]:
        cfg = flacgpu.Config.default(ch, bits, 44100)
        assert lib.flacgpu_reference_max_frame_bytes(ctypes.byref(cfg)) == \
            oracle_ref.lib().oracle_max_frame_bytes(4096, bits, ch)
        # the GPU slot bound is tighter than the reference buffer but never below what a frame can take
        assert lib.flacgpu_frame_bound_bytes(ctypes.byref(cfg)) <= lib.flacgpu_reference_max_frame_bytes(
            ctypes.byref(cfg))


@pytest.mark.parametrize("field,value", [("bits_per_sample", 12), ("bits_per_sample", 20), ("channels", 0),
                                         ("channels", 9), ("block_size", 0), ("block_size", 8192),
                                         ("max_rice_part_order", 9), ("max_rice_param", 0), ("max_rice_param", 31),
                                         ("prediction", 13), ("prediction", 32), ("sample_rate", 1 << 20)])
def test_invalid_configs_rejected(field, value):
    lib = flacgpu.load_library()
    cfg = flacgpu.Config.default(2, 16, 44100)
    setattr(cfg, field, value)
    h = ctypes.c_void_p()
    rc = lib.flacgpu_open(0, ctypes.byref(cfg), 16, ctypes.byref(h))
    assert rc == -1 and not h.value


def _has_gpu():
    try:
        import torch

        return torch.cuda.device_count() > 0
    except Exception:
        return False


@pytest.mark.skipif(_has_gpu(), reason="checks the no-device failure path")
def test_fails_loudly_without_device():
    with pytest.raises(flacgpu.FlacGpuError) as e:
        flacgpu.Encoder(2, 16, 44100)
    assert e.value.code == -5


def test_strerror():
    lib = flacgpu.load_library()
    assert lib.flacgpu_strerror(-5).decode().startswith("HIP device error")


@pytest.mark.skipif(_has_gpu(), reason="checks the no-device failure path")
def test_multi_fails_loudly_without_device():
    with pytest.raises(flacgpu.FlacGpuError) as e:
        flacgpu.MultiEncoder([0, 0], 2, 16, 44100)
    assert e.value.code == -5


def test_multi_rejects_bad_arguments():
    lib = flacgpu.load_library()
    cfg = lib.flacgpu_config_default(2, 16, 44100)
    h = ctypes.c_void_p()
    devs = (ctypes.c_int * 1)(0)
    assert lib.flacgpu_open_multi(0, devs, ctypes.byref(cfg), 16, ctypes.byref(h)) == -2 and not h.value
    assert lib.flacgpu_open_multi(1, None, ctypes.byref(cfg), 16, ctypes.byref(h)) == -2 and not h.value
    n = ctypes.c_size_t(0)
    assert lib.flacgpu_multi_encode_frames(None, None, 2, 0, 0, None, 0, ctypes.byref(n), None) == -2
    lib.flacgpu_close_multi(None)  # no-op


def _kernel_symbols():
    import subprocess

    nm = "/opt/rocm/lib/llvm/bin/llvm-nm"
    if not os.path.exists(nm):
        nm = "nm"
    out = subprocess.run([nm, "-C", flacgpu.LIB_PATH], capture_output=True, text=True, check=True).stdout
    return out


@pytest.mark.skipif(os.environ.get("FLACGPU_LIB") is not None, reason="checks the in-tree release library")
def test_release_library_has_no_diagnostic_kernels():
    """the release libflacgpu.so carries neither the one-wave analysis (k_ana1)
    nor the fused single-pass kernel (k_analyze<..., FP = true>); they live in `make diag` only."""
    assert flacgpu.build_flags() & flacgpu.BUILD_DIAG == 0
    syms = _kernel_symbols()
    assert "k_analyze<2, 16, true, 256, 2, 0, false>" in syms  # the C2 analysis is there
    assert "k_ana1" not in syms
    assert "k_analyze<2, 16, true, 256, 2, 0, true>" not in syms


@pytest.mark.skipif(os.environ.get("FLACGPU_LIB") is not None, reason="checks the in-tree release library")
def test_release_library_ignores_diagnostic_knobs():
    """FLACGPU_FILES_MD5=0 (and the other diagnostic knobs) exist only in diagnostic builds: the
    release library's code never reads them, so a stray environment variable cannot make it
    write a zero STREAMINFO MD5 (encoder.zig:168-170 always finalises it)."""
    import subprocess

    strings = subprocess.run(["strings", flacgpu.LIB_PATH], capture_output=True, text=True, check=True).stdout
    for knob in ("FLACGPU_FILES_MD5", "FLACGPU_FUSED", "FLACGPU_ANA1", "FLACGPU_OVERLAP", "FLACGPU_ENC_PRIO",
                 "FLACGPU_MD5_RESERVE", "FLACGPU_SPIN_SYNC"):
        assert knob not in strings, knob


def _gpu_present():
    try:
        import torch

        return torch.cuda.device_count() > 0
    except Exception:
        return False


def test_comm_unique_id_and_argument_checks():
    """The multi-rank C ABI (fg_comm.cpp): librccl.so.1 opens without a GPU, the communicator id is
    128 fresh bytes per call, and malformed calls are rejected before any collective."""
    import ctypes

    a, b = flacgpu.Comm.unique_id(), flacgpu.Comm.unique_id()
    assert len(a) == len(b) == flacgpu.Comm.ID_BYTES and a != b
    L = flacgpu.load_library()
    out = ctypes.c_void_p()
    cid = (ctypes.c_uint8 * 128).from_buffer_copy(a)
    for world, rank, dev in ((0, 0, 0), (2, 2, 0), (1, -1, 0), (1, 0, -1)):
        assert L.flacgpu_comm_init(cid, world, rank, dev, ctypes.byref(out)) == -2, (world, rank, dev)
    assert L.flacgpu_comm_init(None, 1, 0, 0, ctypes.byref(out)) == -2
    assert L.flacgpu_comm_rank(None) == -2 and L.flacgpu_comm_size(None) == -2
    tb, tf = ctypes.c_uint64(0), ctypes.c_uint64(0)
    assert L.flacgpu_gather_frames_device(None, None, 0, None, None, 0, None, 0, None, 0, ctypes.byref(tb),
                                          ctypes.byref(tf), None) == -2
    n = ctypes.c_size_t(0)
    assert L.flacgpu_encode_frames_sharded(None, None, None, 2, 0, 0, None, 0, ctypes.byref(n), None) == -2
    L.flacgpu_comm_destroy(None)  # a no-op


@pytest.mark.skipif(_gpu_present(), reason="checks the no-device failure path")
def test_comm_init_fails_loudly_without_gpu():
    with pytest.raises(flacgpu.FlacGpuError) as e:
        flacgpu.Comm(flacgpu.Comm.unique_id(), 1, 0, 0)
    assert e.value.code == -5  # DeviceError, never a CPU fallback
