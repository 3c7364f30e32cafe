"""Sharded single-stream encode (zig-flac_amd/parallel.py): frame ranges, the
gather over torch.distributed, and file assembly on rank 0, bit-exact against
the restatement's whole-file encode."""
import os
import socket
import subprocess
import sys

import pytest

import oracle_ref
import parallel
import synth

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.mark.parametrize("n,world", [(0, 2), (1, 3), (4096, 2), (10 * 4096 + 5, 4), (7 * 4096, 8), (3 * 4096, 5)])
def test_shard_frames_partition(n, world):
    nf = (n + 4095) // 4096
    ranges = [parallel.shard_frames(n, 4096, world, r) for r in range(world)]
    assert ranges[0][0] == 0 and ranges[-1][1] == nf
    for (a0, a1), (b0, b1) in zip(ranges, ranges[1:]):
        assert a1 == b0
    lens = [b - a for a, b in ranges]
    assert max(lens) - min(lens) <= 1


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def run_workers(tmp_path, nproc, *args):
    out = tmp_path / "out.flac"
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.join(HERE, "dist_worker.py"),
           "--out", str(out), *args]
    env = dict(os.environ, OMP_NUM_THREADS="1")
    r = subprocess.run(cmd, timeout=300, env=env, capture_output=True, text=True)
    if r.returncode:
        raise AssertionError(f"workers failed ({r.returncode}):\n{r.stderr[-3000:]}")
    return out.read_bytes()


@pytest.mark.parametrize("nproc,ch,bits,n", [(2, 2, 16, 10 * 4096 + 123), (3, 1, 24, 5 * 4096),
                                             (2, 2, 16, 4096 + 1)])
def test_sharded_gather_gloo_matches_whole_file(tmp_path, nproc, ch, bits, n):
    out = run_workers(tmp_path, nproc, "--encoder", "oracle", "--channels", str(ch), "--bits", str(bits),
                      "--samples", str(n))
    pcm = synth.synth_pcm(n, ch, bits, 44100)
    assert out == oracle_ref.encode_file(pcm, ch, bits, 44100)


@pytest.mark.gpu
@pytest.mark.parametrize("nproc,ch,bits,n,md5", [(2, 2, 16, 12 * 4096 + 999, "gpu"), (3, 8, 24, 7 * 4096 + 5, "host"),
                                                 (4, 1, 32, 9 * 4096, "host"), (3, 2, 16, 2 * 4096 + 1, "gpu")])
def test_sharded_gpu_ranks_one_device(tmp_path, nproc, ch, bits, n, md5):
    """The GPU encoder on every rank (ranks share the one device), the gather over gloo (CPU
    tensors): uneven frame ranges, a rank with one frame, 24-bit 8-channel and 32-bit mono."""
    out = run_workers(tmp_path, nproc, "--encoder", "gpu", "--channels", str(ch), "--bits", str(bits), "--samples",
                      str(n), "--md5", md5)
    pcm = synth.synth_pcm(n, ch, bits, 44100)
    assert out == oracle_ref.encode_file(pcm, ch, bits, 44100)


def _gpus():
    try:
        import torch

        return torch.cuda.device_count()
    except Exception:
        return 0


@pytest.mark.gpu
@pytest.mark.parametrize("nproc,n", [(1, 12 * 4096 + 999), (2, 12 * 4096 + 999), (3, 5 * 4096), (2, 4096 + 1)])
def test_sharded_gpu_rccl_device_gather(tmp_path, nproc, n):
    """The device-resident path: frames encoded into HBM and gathered by RCCL (backend
    "nccl") into one device buffer on rank 0, one GPU per rank (RCCL refuses two ranks on
    one device, so the multi-rank cases need that many GPUs; nproc 1 runs the same code
    with a one-rank RCCL communicator on the one-GPU box)."""
    if _gpus() < nproc:
        pytest.skip(f"RCCL needs one GPU per rank: {nproc} ranks, {_gpus()} GPU(s)")
    out = run_workers(tmp_path, nproc, "--encoder", "gpu", "--backend", "nccl", "--samples", str(n))
    pcm = synth.synth_pcm(n, 2, 16, 44100)
    assert out == oracle_ref.encode_file(pcm, 2, 16, 44100)


@pytest.mark.gpu
@pytest.mark.parametrize("mode,ch,bits", [("gather", 2, 16), ("capi", 2, 16), ("capi", 8, 24), ("windows", 2, 16)])
def test_comm_self_p2p_one_rank(tmp_path, monkeypatch, mode, ch, bits):
    """FLACGPU_COMM_SELF_P2P=1: rank 0 moves its own slice into the receive buffer by RCCL
    send/recv to itself instead of a device copy, so the grouped ncclSend / ncclRecv code that the
    other ranks' slices take (fg_comm.cpp transfer) runs on the one-GPU box: the count exchange of
    parallel.gather_comm, flacgpu_encode_frames_sharded's windows (max_frames 4: 11 gathers), and
    ShardedStream (frames in place, sizes by send/recv).  Same file as the restatement's."""
    monkeypatch.setenv("FLACGPU_COMM_SELF_P2P", "1")
    n = 40 * 4096 + 777 if mode != "windows" else 3 * 5 * 4096
    extra = {"gather": ["--gather", "capi"], "capi": ["--mode", "capi", "--max-frames", "4"],
             "windows": ["--mode", "windows", "--windows", "3", "--frames-per-rank", "5"]}[mode]
    out = run_workers(tmp_path, 1, "--encoder", "gpu", "--backend", "nccl", "--channels", str(ch), "--bits",
                      str(bits), "--samples", str(n), *extra)
    pcm = synth.synth_pcm(n, ch, bits, 44100)
    assert out == oracle_ref.encode_file(pcm, ch, bits, 44100)


@pytest.mark.parametrize("nproc,ch,bits,windows,f", [(2, 2, 16, 3, 2), (2, 8, 24, 2, 1), (3, 1, 16, 2, 3)])
def test_sharded_stream_windows_gloo(tmp_path, nproc, ch, bits, windows, f):
    """parallel.ShardedStream (the bench's sharded-stream mode) on world_size > 1 with gloo:
    each rank encodes only its shard of each window, rank 0 gathers in frame order and carries
    the STREAMINFO frame-size replay across windows; the file equals the whole-file encode."""
    out = run_workers(tmp_path, nproc, "--encoder", "oracle", "--mode", "windows", "--channels", str(ch),
                      "--bits", str(bits), "--windows", str(windows), "--frames-per-rank", str(f))
    n = windows * nproc * f * 4096
    pcm = synth.synth_pcm(n, ch, bits, 44100)
    assert out == oracle_ref.encode_file(pcm, ch, bits, 44100)


@pytest.mark.gpu
@pytest.mark.parametrize("ch,bits", [(2, 16), (8, 24)])
def test_sharded_stream_windows_rccl_one_rank(tmp_path, ch, bits):
    """The same ShardedStream on the GPU: device plan advanced window to window, rank 0 encodes
    into its receive buffer, one-rank RCCL communicator, STREAMINFO replayed on the device."""
    out = run_workers(tmp_path, 1, "--encoder", "gpu", "--backend", "nccl", "--mode", "windows", "--channels",
                      str(ch), "--bits", str(bits), "--windows", "3", "--frames-per-rank", "5")
    n = 3 * 5 * 4096
    pcm = synth.synth_pcm(n, ch, bits, 44100)
    assert out == oracle_ref.encode_file(pcm, ch, bits, 44100)


@pytest.mark.gpu
@pytest.mark.parametrize("nproc,ch,bits,n,maxf", [(1, 2, 16, 40 * 4096 + 777, 16), (1, 8, 24, 9 * 4096 + 5, 4),
                                                  (1, 2, 32, 3 * 4096, 1), (2, 2, 16, 40 * 4096 + 777, 16),
                                                  (4, 2, 24, 11 * 4096 + 1, 2), (8, 2, 16, 70 * 4096 + 3, 4)])
def test_encode_frames_sharded_c_abi(tmp_path, nproc, ch, bits, n, maxf):
    """the sharded encode behind the C ABI (flacgpu_encode_frames_sharded): every
    rank passes the whole stream, encodes its slice of each window of world x max_frames frames, and
    libflacgpu.so gathers the windows over its own RCCL communicator into rank 0's output in frame
    order; the assembled file equals the restatement's whole-file encode.  Windows smaller than the
    stream (max_frames 1..16) make every rank run several gather rounds and the last window ragged.
    More than one rank needs that many GPUs (RCCL refuses two ranks on one device)."""
    if _gpus() < nproc:
        pytest.skip(f"RCCL needs one GPU per rank: {nproc} ranks, {_gpus()} GPU(s)")
    out = run_workers(tmp_path, nproc, "--encoder", "gpu", "--backend", "nccl", "--mode", "capi", "--channels",
                      str(ch), "--bits", str(bits), "--samples", str(n), "--max-frames", str(maxf))
    pcm = synth.synth_pcm(n, ch, bits, 44100)
    assert out == oracle_ref.encode_file(pcm, ch, bits, 44100)


@pytest.mark.gpu
@pytest.mark.parametrize("gather", ["capi", "torch"])
def test_sharded_gpu_gather_paths_one_rank(tmp_path, gather):
    """parallel.encode_sharded with the C-ABI gather (flacgpu.Comm) and with the torch.distributed
    one: the same file."""
    n = 12 * 4096 + 999
    out = run_workers(tmp_path, 1, "--encoder", "gpu", "--backend", "nccl", "--gather", gather, "--samples", str(n))
    pcm = synth.synth_pcm(n, 2, 16, 44100)
    assert out == oracle_ref.encode_file(pcm, 2, 16, 44100)
