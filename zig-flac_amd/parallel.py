"""Multi-GPU encode of one stream: frames sharded across ranks, one gather.

Frame f of a stream depends only on samples [f*B, f*B + n) and on f itself (the
UTF-8 frame number, frame_writer.zig:235-251), so rank r of W encodes the
contiguous frame range shard_frames(...) with its own GPU and numbers its frames
from the range start.  The only exchange is the gather of the per-rank
bitstreams and per-frame sizes to the rank that writes the file (SURVEY.md
section 8e): an all-gather of (bytes, frames) counts, then point-to-point
transfers of the variable-length pieces (RCCL over xGMI with backend "nccl",
gloo in the CPU tests).  Rank 0 then replays updateFrameSize in frame order
(metadata.zig:35-40) and writes the 73-byte header (encoder.zig:177-226).

The stream MD5 is sequential over the whole stream and does not shard: rank 0
computes it (md5="gpu": the context's streaming GPU MD5; md5="host": a host
thread overlapping the encode, the Amdahl term of SURVEY.md section 8e).
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


def _gather_bytes(dist, group, payload: bytes, device, rank: int, world: int):
    """Rank 0 receives every rank's payload (variable length); returns the list on rank 0."""
    import torch

    n = torch.tensor([len(payload)], dtype=torch.int64, device=device)
    sizes = [torch.zeros(1, dtype=torch.int64, device=device) for _ in range(world)]
    dist.all_gather(sizes, n, group=group)
    sizes = [int(s.item()) for s in sizes]
    if rank == 0:
        out = [payload]
        bufs = {r: torch.empty(max(sizes[r], 1), dtype=torch.uint8, device=device) for r in range(1, world)}
        ops = [dist.P2POp(dist.irecv, bufs[r], r, group=group) for r in range(1, world) if sizes[r]]
        for req in (dist.batch_isend_irecv(ops) if ops else []):
            req.wait()
        for r in range(1, world):
            out.append(bytes(bufs[r][: sizes[r]].cpu().numpy().tobytes()) if sizes[r] else b"")
        return out
    if sizes[rank]:
        import numpy as np

        t = torch.from_numpy(np.frombuffer(payload, dtype=np.uint8).copy()).to(device)
        for req in dist.batch_isend_irecv([dist.P2POp(dist.isend, t, 0, group=group)]):
            req.wait()
    return None


def encode_sharded(encoder, pcm: bytes, dist=None, group=None, device="cpu", md5: str = "host") -> Optional[bytes]:
    """Encode one stream (interleaved LE PCM, identical on every rank) across the ranks of
    `group`; returns the whole .flac file on rank 0 and None elsewhere.

    `encoder` provides channels, bits, sample_rate, bytes_per_sample, block_size and
    encode_frames(pcm, first_frame) -> (bytes, sizes) (flacgpu.Encoder on a GPU).
    """
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
    frames, sizes = encoder.encode_frames(pcm[s0 * per:s1 * per], first_frame=f0) if s1 > s0 else (b"", [])
    if rank == 0 and md5 == "gpu":
        digest["md5"] = encoder.md5(pcm)

    # payload: u32 frame count, u32 sizes..., frame bytes
    import struct

    payload = struct.pack(f"<I{len(sizes)}I", len(sizes), *sizes) + frames
    parts = _gather_bytes(dist, group, payload, device, rank, world) if dist else [payload]
    if rank != 0:
        return None
    if th:
        th.join()
    all_sizes, body = [], []
    for p in parts:
        k = struct.unpack_from("<I", p)[0]
        all_sizes += list(struct.unpack_from(f"<{k}I", p, 4))
        body.append(p[4 + 4 * k:])
    si = flacgpu.StreamInfo.new(encoder.sample_rate, encoder.channels, encoder.bits, n)
    for sz in all_sizes:
        si.update_frame_size(sz)
    import ctypes

    ctypes.memmove(si.md5, digest["md5"], 16)
    return flacgpu.header_bytes(si, False) + flacgpu.vorbis_comment_bytes(True) + b"".join(body)
