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

With a GPU encoder the gather runs inside libflacgpu.so (flacgpu.Comm: the C ABI's
flacgpu_gather_frames_device over the library's own RCCL communicator, so a host in any
language -- the reference's Zig -- drives the same path); torch.distributed moves the
tensors only for the CPU encoder of the gloo tests.

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


def gather_frames(dist, group, frames, sizes, rank: int, world: int, nbytes=None, recv=None):
    """Gather every rank's (bitstream, frame sizes) tensors to rank 0.

    frames: uint8 tensor, sizes: int32 tensor, both on this rank's communication
    device; nbytes (optional): an int64 scalar tensor on that device with the count of
    valid leading bytes of `frames` (a device encode's total, read without a separate
    host sync: it travels in the one all-gather of the counts).  recv (rank 0,
    optional): preallocated (body, fsz) receive buffers; rank 0's own frames/sizes
    may already be their heads (encoded in place), which skips the local copy.
    Rank 0 gets (one uint8 tensor holding all ranks' bitstreams in rank order, one
    int32 tensor of all frame sizes); other ranks get None.
    """
    import torch

    device = frames.device
    nb = nbytes.reshape(1).to(torch.int64) if nbytes is not None else torch.tensor([frames.numel()], dtype=torch.int64,
                                                                                    device=device)
    counts = torch.cat([torch.tensor([sizes.numel()], dtype=torch.int64, device=device), nb])
    allc = torch.zeros(2 * world, dtype=torch.int64, device=device)
    dist.all_gather_into_tensor(allc, counts, group=group) if device.type == "cuda" else \
        dist.all_gather(list(allc.view(world, 2).unbind(0)), counts, group=group)
    c = allc.view(world, 2).cpu().tolist()
    nfr = [int(x[0]) for x in c]
    nby = [int(x[1]) for x in c]
    if rank == 0:
        if recv is not None:
            body, fsz = recv
        else:
            body = torch.empty(sum(nby), dtype=torch.uint8, device=device)
            fsz = torch.empty(sum(nfr), dtype=torch.int32, device=device)
        if nby[0] and frames.data_ptr() != body.data_ptr():
            body[: nby[0]].copy_(frames[: nby[0]])
        if nfr[0] and sizes.data_ptr() != fsz.data_ptr():
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
        return body[:ob], fsz[:of]
    ops = []
    if nfr[rank]:
        ops.append(dist.P2POp(dist.isend, sizes.contiguous(), 0, group=group))
    if nby[rank]:
        ops.append(dist.P2POp(dist.isend, frames[: nby[rank]].contiguous(), 0, group=group))
    for req in (dist.batch_isend_irecv(ops) if ops else []):
        req.wait()
    return None


class ShardedStream:
    """One long stream encoded window by window across the ranks of `group`: BASELINE.json
    config 4 ("blocks sharded across 8xMI355X, RCCL gather over xGMI for bitstream concat"),
    the block loop of wav2flac.zig:66-97 cut into world pieces per window.

    A window is world * F frames; rank r encodes frames [w0 + r F, w0 + (r + 1) F) of it,
    numbered from there (frame_writer.zig:235-251), and gather_frames collects every rank's
    bitstream and sizes into ONE receive buffer on rank 0, in frame order.  Rank 0 replays
    StreamInfo.updateFrameSize (metadata.zig:35-40) over the window's sizes in frame order,
    carrying {min, max} from window to window.

    GPU encoder (flacgpu.Encoder): step(d_pcm) takes this rank's shard as a device address;
    one plan is built once and moved on by world * F frames per window
    (flacgpu_plan_advance); rank 0 encodes straight into the head of its receive buffer and
    replays on the device (flacgpu_streaminfo_replay_device); nothing crosses PCIe.  Work is
    queued on torch's current stream, which the process group orders its collectives
    against.  Any other encoder (encode_frames(pcm, first_frame) -> (bytes, sizes), e.g. the
    CPU restatement in the gloo tests): step(pcm) takes this rank's shard as bytes and rank 0
    replays with flacgpu_streaminfo_update_frame_size.

    The stream's MD5 is one sequential chain over every window and does not shard (SURVEY.md
    section 8e): callers hash it beside this (host thread) and report it as the Amdahl term.
    """

    def __init__(self, encoder, frames_per_rank: int, dist=None, group=None, device="cpu", comm=None):
        import torch

        self.enc, self.F, self.dist, self.group = encoder, frames_per_rank, dist, group
        self.comm = comm  # flacgpu.Comm: the gather through the C ABI (GPU encoder only)
        self.world = dist.get_world_size(group) if dist else 1
        self.rank = dist.get_rank(group) if dist else 0
        self.device = torch.device(device)
        self.gpu = hasattr(encoder, "encode_plan_device_ex")
        self.window = 0
        self.block = encoder.block_size
        if self.gpu:
            n = frames_per_rank * self.block
            self.plan = encoder.plan([0], [n], first_frames=[self.rank * frames_per_rank], final=[False])
            self.cap = int(self.plan.out_bound)
            dev = self.device
            if self.rank == 0:
                self.body = torch.empty(self.cap * self.world, dtype=torch.uint8, device=dev)
                self.fsz = torch.empty(frames_per_rank * self.world, dtype=torch.int32, device=dev)
                self.out, self.fb = self.body, self.fsz[:frames_per_rank]
                self.minmax = torch.tensor([0xFFFFFF, 0], dtype=torch.int32, device=dev)
            else:
                self.out = torch.empty(self.cap, dtype=torch.uint8, device=dev)
                self.fb = torch.empty(frames_per_rank, dtype=torch.int32, device=dev)
            self.off = torch.empty(frames_per_rank, dtype=torch.int64, device=dev)
            self.tot = torch.zeros(2, dtype=torch.int64, device=dev)
        elif self.rank == 0:
            self.si = flacgpu.StreamInfo.new(encoder.sample_rate, encoder.channels, encoder.bits, 0, self.block)

    def step(self, pcm):
        """Encode this rank's shard of the next window; rank 0 returns (bitstream, sizes) of the
        whole window (tensors on the communication device), other ranks None.

        With the GPU encoder the returned tensors are VIEWS of this object's receive buffers: the
        next step() encodes and gathers into the same memory, so they are valid only until then.
        A caller that keeps a window (appends it to a list, hands it to another thread) must
        .clone() or .cpu() it first."""
        import numpy as np
        import torch

        first = (self.window * self.world + self.rank) * self.F
        if self.gpu:
            st = torch.cuda.current_stream(self.device).cuda_stream
            if self.window:
                self.plan.advance(self.world * self.F, st)
            self.enc.encode_plan_device_ex(self.plan, pcm, self.out.data_ptr(), self.cap, self.fb.data_ptr(),
                                           self.off.data_ptr(), self.tot.data_ptr(), stream=st)
            frames, sizes, nbytes = self.out, self.fb, self.tot[0]
        else:
            fr, sz = self.enc.encode_frames(pcm, first_frame=first)
            frames = torch.from_numpy(np.frombuffer(fr, dtype=np.uint8).copy()).to(self.device)
            sizes = torch.tensor(sz, dtype=torch.int32, device=self.device)
            nbytes = None
        if self.gpu and self.comm is not None:
            st = torch.cuda.current_stream(self.device).cuda_stream
            r0 = self.rank == 0
            tb, tf = self.comm.gather_device(frames.data_ptr(), 0, sizes.data_ptr(), self.F,
                                             d_recv=self.body.data_ptr() if r0 else 0,
                                             recv_cap=self.body.numel() if r0 else 0,
                                             d_recv_sizes=self.fsz.data_ptr() if r0 else 0,
                                             recv_sizes_cap=self.fsz.numel() if r0 else 0,
                                             d_nbytes=nbytes.data_ptr(), stream=st)
            got = (self.body[:tb], self.fsz[:tf]) if r0 else None
        elif self.dist:
            got = gather_frames(self.dist, self.group, frames, sizes, self.rank, self.world, nbytes=nbytes,
                                recv=(self.body, self.fsz) if self.gpu and self.rank == 0 else None)
        else:
            got = (frames[: int(nbytes.item())] if nbytes is not None else frames, sizes)
        self.window += 1
        if self.rank != 0:
            return None
        body, fsz = got
        if self.gpu:
            self.enc.streaminfo_replay_device(fsz.data_ptr(), fsz.numel(), self.minmax.data_ptr(),
                                              torch.cuda.current_stream(self.device).cuda_stream)
        else:
            for v in fsz.cpu().tolist():
                self.si.update_frame_size(v)
        return body, fsz

    def frame_size_minmax(self):
        """Rank 0: STREAMINFO (min_frame_size, max_frame_size) after the windows so far."""
        if self.gpu:
            m = self.minmax.cpu().tolist()
            return m[0] & 0xFFFFFFFF, m[1] & 0xFFFFFFFF
        return self.si.min_frame_size, self.si.max_frame_size

    def close(self):
        if self.gpu and getattr(self, "plan", None):
            self.plan.close()
            self.plan = None


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


def gather_comm(comm, frames, sizes, rank: int):
    """gather_frames over a flacgpu.Comm (C ABI, RCCL inside libflacgpu.so): device tensors of this
    rank's frames/sizes -> rank 0 gets (bitstream, sizes) device tensors, others None.  Two gathers:
    first every rank's (frames, bytes) counts, so that rank 0 can size its receive buffers."""
    import torch

    st = torch.cuda.current_stream(frames.device).cuda_stream
    cnt = torch.tensor([sizes.numel(), frames.numel()], dtype=torch.int64, device=frames.device)
    allc = torch.empty(2 * comm.world, dtype=torch.int64, device=frames.device)
    comm.gather_device(cnt.data_ptr(), 16, 0, 0, d_recv=allc.data_ptr() if rank == 0 else 0,
                       recv_cap=16 * comm.world if rank == 0 else 0, stream=st)
    if rank == 0:
        c = allc.view(-1, 2).cpu().tolist()
        body = torch.empty(max(1, sum(x[1] for x in c)), dtype=torch.uint8, device=frames.device)
        fsz = torch.empty(max(1, sum(x[0] for x in c)), dtype=torch.int32, device=frames.device)
        tb, tf = comm.gather_device(frames.data_ptr(), frames.numel(), sizes.data_ptr(), sizes.numel(),
                                    d_recv=body.data_ptr(), recv_cap=body.numel(), d_recv_sizes=fsz.data_ptr(),
                                    recv_sizes_cap=fsz.numel(), stream=st)
        return body[:tb], fsz[:tf]
    comm.gather_device(frames.data_ptr(), frames.numel(), sizes.data_ptr(), sizes.numel(), stream=st)
    return None


def encode_sharded(encoder, pcm: bytes, dist=None, group=None, device="cpu", md5: str = "host",
                   comm=None) -> Optional[bytes]:
    """Encode one stream (interleaved LE PCM, identical on every rank) across the ranks of
    `group`; returns the whole .flac file on rank 0 and None elsewhere.

    `encoder` provides channels, bits, sample_rate, bytes_per_sample, block_size and either
    encode_frames_device(d_pcm, n, first_frame) -> (uint8 tensor, int32 tensor) on a GPU
    (flacgpu.Encoder; frames stay in HBM) or encode_frames(pcm, first_frame) -> (bytes,
    sizes).  `device` is where the gather's tensors live ("cuda:k" for RCCL, "cpu" for gloo).  `comm` (flacgpu.Comm,
    GPU encoder): the gather runs through the C ABI instead of torch.distributed.
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
        # the context's GPU lane (its default engine is a host core): switched for this hash only
        prev = encoder.md5_engine()
        encoder.set_md5_engine(flacgpu.MD5_DEVICE)
        try:
            digest["md5"] = encoder.md5(pcm)
        finally:
            encoder.set_md5_engine(prev)
    if comm is not None:
        got = gather_comm(comm, frames, sizes, rank)
    else:
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
