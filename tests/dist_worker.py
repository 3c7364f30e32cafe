"""Worker for the multi-process tests of zig-flac_amd/parallel.py (launched by
torch.distributed.run).  --encoder oracle: frames from the CPU restatement (test
infrastructure standing in for the GPU, to exercise sharding + gather + file
assembly on a CPU-only machine); --encoder gpu: flacgpu.Encoder on cuda:0.
Rank 0 writes the assembled file to --out."""
import argparse
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "zig-flac_amd"))


class OracleFrames:
    """encode_frames() of the restatement, with the attributes parallel.encode_sharded reads."""

    def __init__(self, ch, bits, rate, block=4096):
        self.channels, self.bits, self.sample_rate, self.block_size = ch, bits, rate, block
        self.bytes_per_sample = bits // 8

    def encode_frames(self, pcm, first_frame=0):
        import oracle_ref

        out, sizes, _ = oracle_ref.encode_stream(pcm, self.channels, self.bits, self.sample_rate, self.block_size,
                                                 first_frame=first_frame)
        return out, sizes


def run_capi(a, enc, comm, pcm):
    """flacgpu_encode_frames_sharded (C ABI): every rank passes the whole stream, each encodes its
    slice of every window, the library gathers over its own RCCL communicator; rank 0 assembles."""
    import ctypes
    import hashlib

    import flacgpu

    frames, sizes = comm.encode_frames_sharded(enc, pcm)
    if comm.rank != 0:
        assert frames == b"" and sizes == []
        return None
    n = len(pcm) // (a.channels * (a.bits // 8))
    si = flacgpu.StreamInfo.new(a.rate, a.channels, a.bits, n, 4096)
    for v in sizes:
        si.update_frame_size(v)
    ctypes.memmove(si.md5, hashlib.md5(pcm).digest(), 16)
    return flacgpu.header_bytes(si, False) + flacgpu.vorbis_comment_bytes(True) + frames


def run_windows(a, enc, dist, device, comm=None):
    """parallel.ShardedStream over a stream of windows x world x F whole frames: each rank holds
    only its shard of each window; rank 0 assembles the file (the bench's C4 sharded mode)."""
    import ctypes
    import hashlib

    import numpy as np
    import torch

    import flacgpu
    import parallel
    import synth

    world, rank = dist.get_world_size(), dist.get_rank()
    F, B = a.frames_per_rank, 4096
    per = a.channels * (a.bits // 8)
    n = a.windows * world * F * B
    pcm = synth.synth_pcm(n, a.channels, a.bits, a.rate)
    ss = parallel.ShardedStream(enc, F, dist=dist, device=device, comm=comm)
    body = []
    for w in range(a.windows):
        s0 = (w * world + rank) * F * B
        shard = pcm[s0 * per:(s0 + F * B) * per]
        if ss.gpu:
            d = torch.from_numpy(np.frombuffer(shard, dtype=np.uint8).copy()).to(device)
            got = ss.step(d.data_ptr())
        else:
            got = ss.step(shard)
        if rank == 0:
            body.append(got[0].cpu().numpy().tobytes())
    ss.close()
    if rank != 0:
        return None
    lo, hi = ss.frame_size_minmax()
    si = flacgpu.StreamInfo.new(a.rate, a.channels, a.bits, n, B)
    si.min_frame_size, si.max_frame_size = lo, hi
    ctypes.memmove(si.md5, hashlib.md5(pcm).digest(), 16)
    return flacgpu.header_bytes(si, False) + flacgpu.vorbis_comment_bytes(True) + b"".join(body)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--encoder", choices=["oracle", "gpu"], default="oracle")
    p.add_argument("--channels", type=int, default=2)
    p.add_argument("--bits", type=int, default=16)
    p.add_argument("--rate", type=int, default=44100)
    p.add_argument("--samples", type=int, default=10 * 4096 + 123)
    p.add_argument("--md5", default="host")
    p.add_argument("--backend", choices=["gloo", "nccl"], default="gloo")
    p.add_argument("--out", required=True)
    p.add_argument("--mode", choices=["file", "windows", "capi"], default="file",
                   help="file: parallel.encode_sharded; windows: parallel.ShardedStream over --windows windows; "
                        "capi: flacgpu_encode_frames_sharded")
    p.add_argument("--gather", choices=["capi", "torch"], default="capi",
                   help="GPU encoder under nccl: the gather through the C ABI (flacgpu.Comm) or torch.distributed")
    p.add_argument("--max-frames", type=int, default=256, help="GPU encoder: frames per context call")
    p.add_argument("--windows", type=int, default=3)
    p.add_argument("--frames-per-rank", type=int, default=2)
    a = p.parse_args()
    import torch.distributed as dist

    import parallel
    import synth

    import torch

    pcm = synth.synth_pcm(a.samples, a.channels, a.bits, a.rate)
    if a.backend == "nccl":  # RCCL: one GPU per rank
        local = int(os.environ.get("LOCAL_RANK", "0"))
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        device = f"cuda:{local}"
    else:
        dist.init_process_group("gloo")
        device = "cpu"
    if a.encoder == "gpu":
        import flacgpu

        enc = flacgpu.Encoder(a.channels, a.bits, a.rate, device=torch.cuda.current_device() if a.backend == "nccl"
                              else 0, max_frames=max(a.max_frames, a.frames_per_rank))
    else:
        enc = OracleFrames(a.channels, a.bits, a.rate)
    comm = None
    if a.encoder == "gpu" and a.backend == "nccl" and a.gather == "capi":
        comm = flacgpu.Comm.from_process_group(dist, None, torch.cuda.current_device())
    if a.mode == "capi":
        out = run_capi(a, enc, comm, pcm)
    elif a.mode == "windows":
        out = run_windows(a, enc, dist, device, comm)
    else:
        out = parallel.encode_sharded(enc, pcm, dist=dist, device=device, md5=a.md5, comm=comm)
    if comm is not None:
        comm.close()
    if dist.get_rank() == 0:
        open(a.out, "wb").write(out)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
