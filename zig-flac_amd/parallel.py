"""Multi-GPU encode of one stream: frames sharded across ranks, one gather.

Frame f of a stream depends only on samples [f*B, f*B + n) and on f itself (the
UTF-8 frame number, frame_writer.zig:235-251), so rank r of W encodes the
contiguous frame range shard_frames(...) with its own GPU and numbers its frames
from the range start (the block loop of wav2flac.zig:66-97, cut into W pieces).
The only exchange is the gather of the per-rank bitstreams and per-frame sizes
to the rank that writes the file:

  * each rank's frames stay where its encoder put them (device memory on a GPU:
    flacgpu.Encoder.encode_frames_device, no host round trip);
  * an all-gather of the (frames, bytes) counts, then point-to-point transfers
    straight into slices of ONE receive buffer on rank 0, so the whole bitstream
    arrives contiguous and in frame order (RCCL over xGMI with backend "nccl";
    gloo moves the same tensors between CPU processes in the tests);
  * rank 0 replays updateFrameSize in frame order (metadata.zig:35-40), copies the
    bitstream to the host once and writes the 73-byte header (encoder.zig:177-226).

The stream MD5 is sequential over the whole stream and does not shard: rank 0
computes it on a host thread that overlaps the encode and the gather (md5="host",
the Amdahl term of SURVEY.md section 8e), or with the context's opt-in GPU lane
(md5="gpu").
"""
from __future__ import annotations

import hashlib
import threading
from typing import Optional, Tuple

import flacgpu


def shard_frames(n_samples: int, block: int, world: int, rank: int) -> Tuple[int, int]:
    """Contiguous frame range [f0, f1) of `rank`: frames split as evenly as possible."""
    n_frames = (n_samples + block - 1) // block
    base, extra = divmod(n_frames, world)
    f0 = rank * base + min(rank, extra)
    return f0, f0 + base + (1 if rank < extra else 0)


def gather_frames(dist, group, frames, sizes, rank: int, world: int):
    """Gather every rank's (bitstream, frame sizes) tensors to rank 0.

    frames: uint8 tensor, sizes: int32 tensor, both on this rank's communication
    device.  Rank 0 gets (one uint8 tensor holding all ranks' bitstreams in rank
    order, one int32 tensor of all frame sizes); other ranks get None.
    """
    import torch

    device = frames.device
    counts = torch.tensor([sizes.numel(), frames.numel()], dtype=torch.int64, device=device)
    allc = [torch.zeros(2, dtype=torch.int64, device=device) for _ in range(world)]
    dist.all_gather(allc, counts, group=group)
    nfr = [int(c[0].item()) for c in allc]
    nby = [int(c[1].item()) for c in allc]
    if rank == 0:
        body = torch.empty(sum(nby), dtype=torch.uint8, device=device)
        fsz = torch.empty(sum(nfr), dtype=torch.int32, device=device)
        body[: nby[0]].copy_(frames)
        fsz[: nfr[0]].copy_(sizes)
        ops, ob, of = [], nby[0], nfr[0]
        for r in range(1, world):
            if nfr[r]:
                ops.append(dist.P2POp(dist.irecv, fsz[of:of + nfr[r]], r, group=group))
            if nby[r]:
                ops.append(dist.P2POp(dist.irecv, body[ob:ob + nby[r]], r, group=group))
            ob += nby[r]
            of += nfr[r]
        for req in (dist.batch_isend_irecv(ops) if ops else []):
            req.wait()
        return body, fsz
    ops = []
    if nfr[rank]:
        ops.append(dist.P2POp(dist.isend, sizes.contiguous(), 0, group=group))
    if nby[rank]:
        ops.append(dist.P2POp(dist.isend, frames.contiguous(), 0, group=group))
    for req in (dist.batch_isend_irecv(ops) if ops else []):
        req.wait()
    return None


def _encode_shard(encoder, pcm: bytes, per: int, s0: int, s1: int, f0: int, device):
    """This rank's frames as tensors on `device`: on a GPU the bitstream never leaves HBM."""
    import numpy as np
    import torch

    if s1 <= s0:
        return torch.empty(0, dtype=torch.uint8, device=device), torch.empty(0, dtype=torch.int32, device=device)
    if hasattr(encoder, "encode_frames_device"):
        src = torch.from_numpy(np.frombuffer(pcm, dtype=np.uint8, count=(s1 - s0) * per, offset=s0 * per).copy())
        d_pcm = src.to(torch.device("cuda", torch.cuda.current_device()))
        frames, sizes = encoder.encode_frames_device(d_pcm.data_ptr(), s1 - s0, first_frame=f0)
        return frames.to(device), sizes.to(device)  # no copy when `device` is this GPU (RCCL)
    frames, sizes = encoder.encode_frames(pcm[s0 * per:s1 * per], first_frame=f0)
    return (torch.from_numpy(np.frombuffer(frames, dtype=np.uint8).copy()).to(device),
            torch.tensor(sizes, dtype=torch.int32, device=device))


def encode_sharded(encoder, pcm: bytes, dist=None, group=None, device="cpu", md5: str = "host") -> Optional[bytes]:
    """Encode one stream (interleaved LE PCM, identical on every rank) across the ranks of
    `group`; returns the whole .flac file on rank 0 and None elsewhere.

    `encoder` provides channels, bits, sample_rate, bytes_per_sample, block_size and either
    encode_frames_device(d_pcm, n, first_frame) -> (uint8 tensor, int32 tensor) on a GPU
    (flacgpu.Encoder; frames stay in HBM) or encode_frames(pcm, first_frame) -> (bytes,
    sizes).  `device` is where the gather's tensors live ("cuda:k" for RCCL, "cpu" for gloo).
    """
    import ctypes

    world = dist.get_world_size(group) if dist else 1
    rank = dist.get_rank(group) if dist else 0
    per = encoder.channels * encoder.bytes_per_sample
    n = len(pcm) // per
    f0, f1 = shard_frames(n, encoder.block_size, world, rank)
    s0, s1 = f0 * encoder.block_size, min(n, f1 * encoder.block_size)

    digest = {}
    th = None
    if rank == 0 and md5 == "host":
        th = threading.Thread(target=lambda: digest.setdefault("md5", hashlib.md5(pcm).digest()))
        th.start()
    frames, sizes = _encode_shard(encoder, pcm, per, s0, s1, f0, device)
    if rank == 0 and md5 == "gpu":
        digest["md5"] = encoder.md5(pcm)
    got = gather_frames(dist, group, frames, sizes, rank, world) if dist else (frames, sizes)
    if rank != 0:
        return None
    body, fsz = got
    if th:
        th.join()
    si = flacgpu.StreamInfo.new(encoder.sample_rate, encoder.channels, encoder.bits, n, encoder.block_size)
    for sz in fsz.cpu().tolist():
        si.update_frame_size(sz)
    ctypes.memmove(si.md5, digest["md5"], 16)
    return flacgpu.header_bytes(si, False) + flacgpu.vorbis_comment_bytes(True) + body.cpu().numpy().tobytes()
