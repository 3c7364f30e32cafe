"""The multi-rank C ABI (fg_comm.cpp) on one GPU, in this process: a one-rank RCCL communicator
(ncclCommInitRank with world 1, no torch.distributed) and its error agreements -- rank 0's receive
capacities too small, malformed arguments, an output buffer too small for the sharded encode --
plus the device-side byte count of flacgpu_gather_frames_device, each with and without
FLACGPU_COMM_SELF_P2P (read at flacgpu_comm_init).  Bytes vs the restatement
(oracle_ref.encode_stream, frame_writer.zig / encoder.zig restated)."""
import ctypes

import pytest

import flacgpu
import oracle_ref
import synth

pytestmark = pytest.mark.gpu

ERR_INVALID_INPUT, ERR_OUTPUT_TOO_SMALL = -2, -4


@pytest.fixture(params=["copy", "self_p2p"])
def comm(request, monkeypatch):
    import torch

    torch.cuda.set_device(0)
    if request.param == "self_p2p":
        monkeypatch.setenv("FLACGPU_COMM_SELF_P2P", "1")
    else:
        monkeypatch.delenv("FLACGPU_COMM_SELF_P2P", raising=False)
    c = flacgpu.Comm(flacgpu.Comm.unique_id(), 1, 0, 0)
    yield c
    c.close()


def _code(fn):
    with pytest.raises(flacgpu.FlacGpuError) as e:
        fn()
    return e.value.code


def test_gather_device_one_rank(comm):
    import torch

    dev = torch.device("cuda", 0)
    frames = torch.randint(0, 256, (10007,), dtype=torch.uint8, device=dev)
    sizes = torch.randint(1, 1 << 20, (37,), dtype=torch.int32, device=dev)
    body = torch.zeros(20000, dtype=torch.uint8, device=dev)
    fsz = torch.zeros(64, dtype=torch.int32, device=dev)
    # the byte count from the host, then from the device (d_nbytes overrides nbytes)
    tb, tf = comm.gather_device(frames.data_ptr(), frames.numel(), sizes.data_ptr(), sizes.numel(),
                                d_recv=body.data_ptr(), recv_cap=body.numel(), d_recv_sizes=fsz.data_ptr(),
                                recv_sizes_cap=fsz.numel())
    torch.cuda.synchronize()
    assert (tb, tf) == (10007, 37)
    assert torch.equal(body[:tb], frames) and torch.equal(fsz[:tf], sizes)
    nb = torch.tensor([4321], dtype=torch.int64, device=dev)
    body.zero_()
    tb, tf = comm.gather_device(frames.data_ptr(), 0, sizes.data_ptr(), sizes.numel(), d_recv=body.data_ptr(),
                                recv_cap=body.numel(), d_recv_sizes=fsz.data_ptr(), recv_sizes_cap=fsz.numel(),
                                d_nbytes=nb.data_ptr())
    torch.cuda.synchronize()
    assert tb == 4321 and torch.equal(body[:4321], frames[:4321]) and int(body[4321:].sum()) == 0
    # rank 0's capacities too small: OutputTooSmall on every rank, nothing moved
    body.zero_()
    assert _code(lambda: comm.gather_device(frames.data_ptr(), frames.numel(), sizes.data_ptr(), sizes.numel(),
                                            d_recv=body.data_ptr(), recv_cap=10006, d_recv_sizes=fsz.data_ptr(),
                                            recv_sizes_cap=fsz.numel())) == ERR_OUTPUT_TOO_SMALL
    assert _code(lambda: comm.gather_device(frames.data_ptr(), frames.numel(), sizes.data_ptr(), sizes.numel(),
                                            d_recv=body.data_ptr(), recv_cap=body.numel(),
                                            d_recv_sizes=fsz.data_ptr(), recv_sizes_cap=36)) == ERR_OUTPUT_TOO_SMALL
    torch.cuda.synchronize()
    assert int(body.sum()) == 0
    # malformed arguments are agreed through the count exchange, not left hanging in it
    assert _code(lambda: comm.gather_device(frames.data_ptr(), frames.numel(), 0, 5, d_recv=body.data_ptr(),
                                            recv_cap=body.numel())) == ERR_INVALID_INPUT
    assert _code(lambda: comm.gather_device(0, 100, 0, 0, d_recv=body.data_ptr(),
                                            recv_cap=body.numel())) == ERR_INVALID_INPUT
    # nothing at all: a valid empty gather
    assert comm.gather_device(0, 0, 0, 0) == (0, 0)


@pytest.mark.parametrize("ch,bits,n,maxf", [(2, 16, 23 * 4096 + 11, 4), (1, 24, 5 * 4096, 2), (8, 16, 3 * 4096 + 1, 1)])
def test_encode_frames_sharded_one_rank(comm, ch, bits, n, maxf):
    pcm = synth.synth_pcm(n, ch, bits, 48000)
    with flacgpu.Encoder(ch, bits, 48000, device=0, max_frames=maxf) as enc:
        got, sizes = comm.encode_frames_sharded(enc, pcm, first_frame=77)
        ref, ref_sizes, _ = oracle_ref.encode_stream(pcm, ch, bits, 48000, first_frame=77)
        assert sizes == ref_sizes and got == ref
        # an output buffer one byte short: OutputTooSmall, agreed after the window that overflows
        L = flacgpu.load_library()
        cap = len(ref) - 1
        out = ctypes.create_string_buffer(cap)
        n_out = ctypes.c_size_t(0)
        rc = L.flacgpu_encode_frames_sharded(enc.ctx, comm.comm, pcm, bits // 8, n, 77, out, cap,
                                             ctypes.byref(n_out), None)
        assert rc == ERR_OUTPUT_TOO_SMALL and n_out.value == 0
        # the communicator and the context stay usable
        got2, _ = comm.encode_frames_sharded(enc, pcm, first_frame=77)
        assert got2 == ref
