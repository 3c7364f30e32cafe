#!/usr/bin/env python3
"""Benchmark: FLAC block encode on MI355X (BASELINE.json metric).

metric : MSamples/s encoded (whole node), 44.1kHz/16-bit stereo, blocksize 4096
unit   : 1 sample = one interchannel sample (STREAMINFO unit, metadata.zig:24)

Workload (config 2).  S independent long streams (files) per GPU, encoded F
4096-sample blocks of each per step (16384 streams x 16 blocks = 262144 blocks =
4 GiB of PCM per step by default -- since round 3: per step the persistent grids' ramp-down and
the MD5 chains' tail cost ~0.3 ms, amortised over more frames: 65536-block steps measured 6 %
below 131072 (profiles/r3r_shape.txt), 131072 3.8 % below 262144 (profiles/r3x_shape.txt);
the stream_curve field shows 8 .. 65536 streams at the same blocks per step): the reference's per-file block loop
(wav2flac.zig:66-97) run for S files at once.  A step is one pass of the hot
path over its batch: analysis (mid/side, wasted bits, fixed-order analysis,
Rice search, subframe choice, exact frame sizes), frame-size scan, pack (bit
packing, CRC-8/16, frames at their final offsets) and the MD5 of every
stream's PCM.  Streams continue from step to step: frame numbers move on by F
(flacgpu_plan_advance) and every stream's MD5 state is carried on the device
(flacgpu_encode_plan_device_ex), so step k's MD5 chains follow step k-1's; the
MD5 runs on its own HIP stream beside the next step's encode.  PCM is resident
in HBM before the timed region (the same bytes each step); outputs stay in HBM.

After the timed region the output is PROVED, not assumed: the device error word
is checked (flacgpu_sync_check), a sample of streams' last-step frames is
compared byte for byte with the CPU restatement (oracle/, with the same frame
numbers), and their carried MD5 states are finalised on the device and compared
with hashlib over the bytes they absorbed.  `output_ok` is that comparison.

One process per GPU.  `bench.py --gpus N` without WORLD_SIZE in the environment
starts N fresh child processes itself (RANK / LOCAL_RANK / WORLD_SIZE /
MASTER_ADDR=127.0.0.1 / MASTER_PORT; the parent never touches the GPU and
prints nothing: rank 0's JSON line is the only stdout line); under torchrun
(WORLD_SIZE set) the process is one rank.  Streams are independent files, so
ranks shard streams with no data-path collective (weak scaling); a barrier and
a max-over-ranks reduction bracket the timed region.

After the headline (config 2) the default run times BASELINE configs 3, 4 and
5 as their own lines (`configs`: 65536-block steps, the same barrier + max over
ranks, output compared with the oracle, CPU port per config at N = 1).

The JSON line also carries:
  roofline      -- the dominant kernel (analysis, pack or MD5: the longest mean
                   launch), its algorithmic bytes per launch / its mean launch time
                   from HIP events on its stream, against 8 TB/s; `traffic` from the
                   committed rocprofv3 PMC summary of the same workload and kernel
                   (profiles/), else null; `limiter` = what DESIGN.md measures binds;
  stream_curve  -- the same blocks per step at 8 .. 65536 concurrent streams, each
                   stream's MD5 on the engine the plan picks (host pool below the
                   crossover, one GPU lane per stream above), verified; both
                   engines timed near the crossover (rank 0, N = 1);
  end_to_end    -- BASELINE.md's host-buffer contract: 8 .. 64 ten-minute WAV-sized PCM
                   buffers in host memory -> .flac files in host memory (H2D,
                   kernels, D2H, MD5 on the host pool, 73-byte header), per file
                   (flacgpu_encode_file, one context + thread each) and as one
                   flacgpu_encode_files call; bounds: the files' MD5 alone on the
                   pool, the frames path alone (rank 0, N = 1);
  cpu_baseline  -- the CPU restatement (oracle/, "port", -O3) on P pinned host
                   threads over a bounded sample of the same workload.
"""
from __future__ import annotations

import argparse
import ctypes
import glob
import hashlib
import json
import os
import subprocess
import sys
import threading
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "zig-flac_amd"))

METRIC = "MSamples/s encoded (whole node), 44.1kHz/16-bit stereo, blocksize 4096"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
HBM_COPY_GBS = 6290.0  # MI355X_MICROARCH.md: measured float4 copy; BASELINE.md asks for the fraction of both
# BASELINE.json configs (channels, bits, rate, LPC max order); c2 is the headline metric's
PRESETS = {"c2": (2, 16, 44100, 0), "c3": (2, 24, 96000, 8), "c4": (8, 24, 96000, 0), "c5": (2, 32, 192000, 12)}
# CPU-baseline input per config (blocks, 512 MiB-1.5 GiB of PCM; the fixed-time runs cycle over it)
CPU_FRAMES = {"c2": 32768, "c3": 16384, "c4": 4096, "c5": 8192}
LIMITER = {  # what binds each kernel (measured, not the roofline it is priced on)
    "analyze": "VALU issue/latency (integer dependent chains per lane), not HBM",
    "pack": "LDS atomics + dependent bit-offset chains, not HBM",
    "md5": "per-stream dependent chain (one lane per stream, 64 sequential steps per 64-B block) on issue slots shared with the encode waves",
}


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--frames", type=int, default=262144, help="4096-sample blocks per GPU per step")
    p.add_argument("--streams", type=int, default=16384, help="concurrent streams (files) per GPU")
    p.add_argument("--config", choices=sorted(PRESETS), default=None,
                   help="BASELINE.json config preset (overrides --channels/--bits/--rate/--lpc); default c2")
    p.add_argument("--channels", type=int, default=2)
    p.add_argument("--bits", type=int, default=16)
    p.add_argument("--rate", type=int, default=44100)
    p.add_argument("--lpc", type=int, default=0, help="LPC max order (0 = fixed prediction, the reference)")
    p.add_argument("--no-md5", action="store_true", help="skip the per-stream GPU MD5 (diagnostics only)")
    p.add_argument("--verify-streams", type=int, default=64, help="streams compared with the oracle after timing")
    p.add_argument("--no-curve", action="store_true")
    p.add_argument("--curve", default="8,64,256,1024,8192,16384,65536")
    p.add_argument("--no-e2e", action="store_true")
    p.add_argument("--e2e-files", default="8,16,32,64", help="file counts of the end-to-end curve")
    p.add_argument("--e2e-minutes", type=float, default=10.0)
    p.add_argument("--e2e-many", type=int, default=256,
                   help="one more end-to-end point: this many files holding the largest point's samples (0: off)")
    p.add_argument("--e2e-node-files", type=int, default=32,
                   help="files per rank of the every-rank end-to-end run (N > 1)")
    p.add_argument("--e2e-max-frames", type=int, default=6144,
                   help="frames per context of the end-to-end encoders (three pipelined chunk sets)")
    p.add_argument("--e2e-numa", choices=["local", "off"], default="local",
                   help="local: every thread of the process on the GPU's NUMA node before the e2e buffers "
                        "are allocated (pinned pages and the MD5 pool's reads on the GPU's side of the fabric)")
    p.add_argument("--no-sharded", action="store_true", help="skip the sharded single-stream line")
    p.add_argument("--sharded-config", choices=sorted(PRESETS), default="c4")
    p.add_argument("--sharded-frames", type=int, default=32768,
                   help="frames per rank per window (sharded mode; SURVEY 8(d): 32768 blocks per GPU for C4)")
    p.add_argument("--sharded-steps", type=int, default=10)
    p.add_argument("--no-cpu", action="store_true")
    p.add_argument("--cpu-frames", type=int, default=32768, help="blocks of the CPU-baseline input (cycled)")
    p.add_argument("--cpu-seconds", type=float, default=1.0,
                   help="seconds per P-thread CPU-baseline run (the single-core run takes 1.5x)")
    p.add_argument("--cpu-threads", type=int, default=0, help="0: the CPU share (OMP_NUM_THREADS), capped at a socket")
    p.add_argument("--cpu-reps", type=int, default=3, help="CPU-baseline runs per leg (best, median and spread reported)")
    p.add_argument("--cpu-place", choices=["idle", "socket0", "none"], default="idle",
                   help="CPU-baseline thread placement: least busy physical cores / first socket-0 CPUs / unpinned")
    p.add_argument("--cpu-only", action="store_true", help="run only the CPU-baseline legs (no torch, no GPU) and "
                                                           "print them as one JSON line")
    p.add_argument("--configs", default="c3,c4,c5",
                   help="other BASELINE configs timed as their own lines after the headline ('' = none)")
    p.add_argument("--cfg-frames", type=int, default=65536, help="blocks per GPU per step of each --configs line")
    p.add_argument("--cfg-steps", type=int, default=20)
    a = p.parse_args()
    if a.config:
        a.channels, a.bits, a.rate, a.lpc = PRESETS[a.config]
    return a


def workload_key(a) -> str:
    # the fused single-pass schedule (FLACGPU_FUSED=1) runs other kernels: its own PMC summaries
    fused = os.environ.get("FLACGPU_FUSED", "0") == "1"
    # the one-wave-per-frame C2 analysis (FLACGPU_ANA1=1 / 2, fg_ana1.hpp) likewise
    ana1 = os.environ.get("FLACGPU_ANA1", "0")
    return (f"{a.config or 'c2'}:{a.frames}x{a.streams}" + ("+fused" if fused else "") +
            (f"+ana1v{ana1}" if ana1 in ("1", "2") and (a.config or "c2") == "c2" else ""))


def build_input(args, rank):
    """S streams of F blocks, contiguous, cut from a seeded pool (SURVEY.md 8(d) signal mix)."""
    import numpy as np
    import synth

    S, F = args.streams, args.frames // args.streams
    ch, bits = args.channels, args.bits
    n_per = F * 4096
    pool_n = max(8 * 4096 * 64, min(n_per, 4096 * 4096) + 4096 * 64)
    pool = synth.synth_samples(pool_n, ch, bits, args.rate, stream=0)
    pcm_pool = np.frombuffer(synth.to_pcm_bytes(pool, bits), dtype=np.uint8)
    fb = ch * (bits // 8)
    rng = np.random.Generator(np.random.PCG64(20260821 + 7919 * rank))
    buf = np.empty(args.frames * 4096 * fb, dtype=np.uint8)
    blocks = (pool_n - 4096) // 4096
    # each stream: a run of pool windows (4096-block windows at random starts)
    for s in range(S):
        done = 0
        while done < n_per:
            take = min(n_per - done, 4096 * 4096, (pool_n // 4096 - 1) * 4096)
            a = int(rng.integers(0, blocks - take // 4096 + 1)) * 4096 * fb
            o = (s * n_per + done) * fb
            buf[o:o + take * fb] = pcm_pool[a:a + take * fb]
            done += take
    return buf


# ---------------------------------------------------------------------------------------------
# the GPU step loop (one plan = S streams x F blocks at fixed device offsets)
class Workload:
    """md5: True / "device" (carried per-stream state on the GPU, one lane per stream), "host"
    (flacgpu_md5_plan_host on a host thread beside the encode, from the host copy h_pcm), False."""

    def __init__(self, enc, d_pcm, S, F, fb, dev, md5=True, h_pcm=None):
        import flacgpu
        import numpy as np
        import torch

        self.enc, self.S, self.F = enc, S, F
        n_per = F * 4096
        self.offsets = [s * n_per * fb for s in range(S)]
        self.plan = enc.plan(self.offsets, [n_per] * S, first_frames=[0] * S, final=[False] * S)
        self.d_pcm = d_pcm
        self.out_cap = int(self.plan.out_bound)
        self.d_out = torch.empty(self.out_cap, dtype=torch.uint8, device=dev)
        self.d_fb = torch.empty(self.plan.n_frames, dtype=torch.int32, device=dev)
        self.d_off = torch.empty(self.plan.n_frames, dtype=torch.int64, device=dev)
        self.d_tot = torch.zeros(2, dtype=torch.int64, device=dev)
        self.md5 = "device" if md5 is True else md5
        if self.md5 == "host":
            assert h_pcm is not None
            self.h_pcm = h_pcm
            self.h_state = (flacgpu.Md5State * S)()
            flacgpu.load_library().flacgpu_md5_state_init(self.h_state, S)
            self.d_state = None
        else:
            self.d_state = torch.from_numpy(np.frombuffer(flacgpu.md5_states(S), dtype=np.uint8).copy()).to(dev)
        self.stream = torch.cuda.Stream(dev)  # the encode's own stream (not the legacy null stream)
        self.md5_stream = torch.cuda.Stream(dev)  # in order: each stream's MD5 chain follows the last step's
        self.steps_done = 0
        torch.cuda.synchronize()  # the buffers above were filled on the default stream

    def step(self):
        hasher = None
        if self.md5 == "host":
            # the segments' MD5 on the library's host pool, beside this step's GPU encode (ctypes
            # releases the GIL for the call); the step ends when both have
            hasher = threading.Thread(target=self.plan.md5_host,
                                      args=(self.h_pcm.ctypes.data, self.h_state, None))
            hasher.start()
        if self.steps_done:
            self.plan.advance(self.F, self.stream.cuda_stream)
        self.enc.encode_plan_device_ex(self.plan, self.d_pcm.data_ptr(), self.d_out.data_ptr(), self.out_cap,
                                       self.d_fb.data_ptr(), self.d_off.data_ptr(), self.d_tot.data_ptr(),
                                       self.d_state.data_ptr() if self.md5 == "device" else None, None,
                                       stream=self.stream.cuda_stream, md5_stream=self.md5_stream.cuda_stream)
        if hasher:
            hasher.join()
        self.steps_done += 1

    def close(self):
        self.plan.close()
        self.d_pcm = self.d_out = self.d_fb = self.d_off = self.d_tot = self.d_state = None


def run_timed(w, steps, warmup, dist=None):
    import torch

    for _ in range(warmup):
        w.step()
    torch.cuda.synchronize()
    w.enc.reset_timing()
    w.enc.set_timing(True)
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        w.step()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    if dist:
        dist.barrier()
    w.enc.set_timing(False)
    return t1 - t0


def verify(args, w, buf, fb, n_verify, dev, frames=True):
    """Last step's frames of a sample of streams == the oracle's (frames=False: skipped); their
    carried MD5 == hashlib."""
    import numpy as np
    import torch

    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_ref

    enc = w.enc
    enc.sync_check(w.stream.cuda_stream)
    enc.sync_check(w.md5_stream.cuda_stream)
    total = int(w.d_tot[0].item())
    sizes = w.d_fb.cpu().numpy()
    offs = w.d_off.cpu().numpy()
    ok = total == int(sizes.astype(np.int64).sum()) and total > 0
    first_number = (w.steps_done - 1) * w.F
    picks = sorted(set(int(x) for x in np.linspace(0, w.S - 1, min(n_verify, w.S))))
    n_per = w.F * 4096
    for s in picks if frames else []:
        f0 = w.plan.first_frame[s]
        f1 = w.plan.first_frame[s + 1] if s + 1 < w.S else int(w.plan.n_frames)
        a = int(offs[f0])
        b = int(offs[f1]) if f1 < int(w.plan.n_frames) else total
        pcm = bytes(buf[w.offsets[s]:w.offsets[s] + n_per * fb])
        ref, ref_sizes, _ = oracle_ref.encode_stream(pcm, args.channels, args.bits, args.rate, lpc=args.lpc,
                                                     first_frame=first_number)
        got = w.d_out[a:b].cpu().numpy().tobytes()
        ok &= got == ref and [int(x) for x in sizes[f0:f1]] == ref_sizes
    md5_ok = None
    if w.md5:
        if w.md5 == "host":
            # finalise the carried host states with an empty final segment
            dig = np.frombuffer(b"".join(flacgpu_md5_many([b""] * w.S, [True] * w.S, w.h_state)),
                                dtype=np.uint8).reshape(-1, 16)
        else:
            # finalise every stream's carried state with an empty final segment, on the device
            fin = enc.plan(w.offsets, [0] * w.S, final=[True] * w.S)
            d_md5 = torch.zeros(16 * w.S, dtype=torch.uint8, device=dev)
            d_tot = torch.zeros(2, dtype=torch.int64, device=dev)
            dummy = torch.zeros(16, dtype=torch.uint8, device=dev)
            enc.encode_plan_device_ex(fin, w.d_pcm.data_ptr(), dummy.data_ptr(), 16, dummy.data_ptr(),
                                      dummy.data_ptr(), d_tot.data_ptr(), w.d_state.data_ptr(), d_md5.data_ptr(),
                                      stream=w.stream.cuda_stream)
            enc.sync_check(w.stream.cuda_stream)
            fin.close()
            dig = d_md5.cpu().numpy().reshape(-1, 16)
        md5_ok = True
        for s in picks[:16]:
            pcm = bytes(buf[w.offsets[s]:w.offsets[s] + n_per * fb])
            h = hashlib.md5()
            for _ in range(w.steps_done):
                h.update(pcm)
            md5_ok &= dig[s].tobytes() == h.digest()
        ok &= md5_ok
    return bool(ok), {"streams_compared": len(picks), "frame_numbers_from": first_number,
                      "md5_streams_compared": min(16, len(picks)) if w.md5 else 0}


def flacgpu_md5_many(chunks, final, states):
    import flacgpu

    return flacgpu.md5_many(chunks, final, states)


def kernel_times(enc):
    import flacgpu

    return {name: enc.kernel_time(k) for k, name in enumerate(flacgpu.KERNEL_NAMES)}


def read_valu_mix(cfg, kernel):
    """SIMD-cycles per VALU instruction of `kernel` in config `cfg` from the committed static-mix
    summary (tools/valu_mix.sh -> profiles/<tag>_valu_mix.json, priced with the measured issue rates
    of profiles/r5_issue_micro.txt), else None."""
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "*valu_mix*.json")), reverse=True):
        try:
            d = json.load(open(f))
        except Exception:
            continue
        v = (d.get(cfg) or {}).get(kernel)
        if v:
            return v.get("cycles_per_instr"), os.path.basename(f)
    return None, None


def read_pmc(key, kernel):
    """(HBM bytes per launch, counters) of `kernel` in the committed PMC summary of workload `key`."""
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "*pmc*.json")), reverse=True):
        try:
            d = json.load(open(f))
        except Exception:
            continue
        if d.get("workload") != key:
            continue
        return (d.get("hbm_bytes_per_launch", {}).get(kernel),
                d.get("counters_per_dispatch", {}).get(kernel, {}), os.path.basename(f))
    return None, {}, None


# ---------------------------------------------------------------------------------------------
def sharded_stream(args, rank, world, dist_mod, dev):
    """BASELINE config 4's data path: ONE long stream, each window's frames sharded over the ranks
    (rank r: frames [w0 + r F, w0 + (r + 1) F)), every rank's bitstream + sizes gathered by RCCL
    into one receive buffer on rank 0, STREAMINFO frame-size replay on rank 0's device, all inside
    the timed region (parallel.ShardedStream).  N = 1 runs the same code as a one-rank RCCL
    communicator.  The stream's MD5 is one sequential chain and does not shard: it is timed
    separately on a host core and reported as the Amdahl term, not inside `value`."""
    import numpy as np
    import torch

    import flacgpu
    import parallel

    ch, bits, rate, lpc = PRESETS[args.sharded_config]
    F = args.sharded_frames
    fb = ch * (bits // 8)
    own_group = False
    if dist_mod is None:
        import socket

        import torch.distributed as dist_mod

        sk = socket.socket()
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
        sk.close()
        dist_mod.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1,
                                    device_id=dev)
        own_group = True
    sub = argparse.Namespace(streams=1, frames=F, channels=ch, bits=bits, rate=rate)
    shard = build_input(sub, rank)  # this rank's shard of every window (frame numbers move on)
    enc = flacgpu.Encoder(ch, bits, rate, device=torch.cuda.current_device(), max_frames=F, lpc_order=lpc)
    d_pcm = torch.from_numpy(shard).to(dev)
    cstream = torch.cuda.Stream(dev)
    # the gather through the C ABI: libflacgpu.so's own RCCL communicator (flacgpu_gather_frames_device),
    # its id handed out over the torch process group
    comm = flacgpu.Comm.from_process_group(dist_mod, None, torch.cuda.current_device())
    with torch.cuda.stream(cstream):
        ss = parallel.ShardedStream(enc, F, dist=dist_mod, device=dev, comm=comm)
        for _ in range(2):
            ss.step(d_pcm.data_ptr())
        torch.cuda.synchronize()
        enc.reset_timing()
        enc.set_timing(True)
        dist_mod.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.sharded_steps):
            got = ss.step(d_pcm.data_ptr())
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        dist_mod.barrier()
        enc.set_timing(False)
    t = torch.tensor([dt], dtype=torch.float64, device=dev)
    dist_mod.all_reduce(t, op=dist_mod.ReduceOp.MAX)
    dt = float(t.item())
    kt = kernel_times(enc)
    res = None
    if rank == 0:
        # proof: rank 0's frames of the last window == the restatement's at the same frame numbers;
        # the window's device replay == the host replay of its sizes (metadata.zig:35-40)
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        import oracle_ref

        body, fsz = got
        sizes = fsz.cpu().numpy().astype(np.int64)
        nb0 = int(sizes[:F].sum())
        last_first = (ss.window - 1) * world * F
        k = min(F, 64)
        ref, ref_sizes, _ = oracle_ref.encode_stream(bytes(shard[: k * 4096 * fb]), ch, bits, rate, lpc=lpc,
                                                     first_frame=last_first)
        ok = body[: len(ref)].cpu().numpy().tobytes() == ref and [int(x) for x in sizes[:k]] == ref_sizes
        ok &= int(body.numel()) == int(sizes.sum()) and nb0 > 0
        mm = torch.tensor([0xFFFFFF, 0], dtype=torch.int32, device=dev)
        enc.streaminfo_replay_device(fsz.data_ptr(), fsz.numel(), mm.data_ptr())
        lo, hi = 0xFFFFFF, 0
        for v in sizes.tolist():
            if v > hi:
                hi = v
            elif v < lo:
                lo = v
        ok &= mm.cpu().tolist() == [lo, hi]
        # the Amdahl term: one stream's MD5 over a window's bytes on one host core
        sample = shard[: min(len(shard), 64 << 20)].tobytes()
        t1 = time.perf_counter()
        hashlib.md5(sample).digest()
        md5_s = (time.perf_counter() - t1) * (world * len(shard) / len(sample))
        samples = world * F * 4096 * args.sharded_steps
        per = {n: round(v[1] / max(v[0], 1), 4) for n, v in kt.items() if v[0]}
        res = {"workload": f"{args.sharded_config.upper()}: {rate/1000:g}kHz {bits}-bit {ch}ch, ONE stream, "
                           f"windows of {world} x {F} frames (rank r encodes the r-th {F}), RCCL gather of "
                           "bitstream + sizes into one rank-0 buffer, STREAMINFO replay on rank 0's device",
               "ranks": world, "frames_per_rank": F, "windows": args.sharded_steps,
               "value": round(samples / dt / 1e6, 2), "unit": "MSamples/s",
               "ms_per_window": round(dt / args.sharded_steps * 1e3, 4),
               "kernel_ms_per_window": per,
               "gather": "flacgpu_gather_frames_device (C ABI, libflacgpu.so's own RCCL communicator): "
                         "all_gather of (frames, bytes) counts, then grouped point-to-point RCCL transfers into "
                         "slices of one receive buffer (rank 0 encodes into its head in place)",
               "md5_amdahl": {"ms_per_window_one_host_core": round(md5_s * 1e3, 2),
                              "stream_cap_msamples_per_s": round(world * F * 4096 / md5_s / 1e6, 1),
                              "note": "one stream's MD5 is a serial chain over every window (wav_reader.zig:66): "
                                      "it does not shard and is not in `value`"},
               "output_ok": bool(ok),
               "verified": f"rank 0's first {k} frames of the last window (frame numbers from {last_first}) vs "
                           "the restatement; device STREAMINFO replay of the window vs the host replay"}
    ss.close()
    comm.close()
    enc.close()
    del d_pcm
    if own_group:
        dist_mod.destroy_process_group()
    return res


def stream_curve(args, enc, d_pcm, buf, fb, dev):
    """Same blocks per step at S concurrent streams: the encode beside the per-stream MD5 chains,
    on the engine the plan picks (flacgpu_plan_md5_engine: the host pool for a few long chains, one
    GPU lane per stream above the crossover), MD5 verified at every point.  Near the crossover the
    other engine is timed too (`other`), which is how DESIGN.md section 5.2's crossover is measured."""
    import flacgpu

    out = []
    for S in [int(x) for x in args.curve.split(",") if x]:
        if args.frames % S:
            continue
        F = args.frames // S
        probe = enc.plan([0] * S, [F * 4096] * S, final=[False] * S)
        pick = "host" if probe.md5_engine() == flacgpu.MD5_HOST else "device"
        probe.close()
        engines = [pick] + ([{"host": "device", "device": "host"}[pick]] if 64 <= S <= 1024 else [])
        point = {"streams": S, "blocks_per_stream_per_step": F, "md5_engine": pick}
        for eng in engines:
            w = Workload(enc, d_pcm, S, F, fb, dev, md5=eng, h_pcm=buf)
            steps = 2 if F <= 64 else 1
            dt = run_timed(w, steps, 1)
            kt = kernel_times(enc)
            ok, _ = verify(args, w, buf, fb, 2, dev, frames=False)
            per = {k: round(v[1] / v[0], 3) for k, v in kt.items() if v[0]}
            samples = S * F * 4096 * steps
            res = {"value": round(samples / dt / 1e6, 1), "ms_per_step": round(dt / steps * 1e3, 3),
                   "kernel_ms": per, "md5_ok": ok}
            if eng == pick:
                point.update(res)
            else:
                point["other"] = dict(engine=eng, **res)
            w.close()
        out.append(point)
    return out


def _timed(fn):
    t0 = time.perf_counter()
    fn()
    return time.perf_counter() - t0


def gpu_local_cpus(device=0):
    """CPUs of the GPU's NUMA node (sysfs local_cpulist of the device's PCI function) that this process
    may use, or None."""
    import torch

    try:
        pr = torch.cuda.get_device_properties(device)
        bdf = f"{pr.pci_domain_id:04x}:{pr.pci_bus_id:02x}:{pr.pci_device_id:02x}.0"
        txt = open(f"/sys/bus/pci/devices/{bdf}/local_cpulist").read().strip()
        cpus = set()
        for part in txt.split(","):
            a, _, b = part.partition("-")
            cpus.update(range(int(a), int(b or a) + 1))
        cpus &= os.sched_getaffinity(0)
        return sorted(cpus) or None
    except Exception:
        return None


def move_process(cpus):
    """Every thread of this process onto `cpus` (sched_setaffinity acts per thread)."""
    for tid in os.listdir("/proc/self/task"):
        try:
            os.sched_setaffinity(int(tid), cpus)
        except OSError:
            pass


def e2e_files(n_files, n, fb, ch, bits, rate, stream=11):
    """n_files ten-minute-sized PCM buffers in pinned host memory, cut from one seeded pool."""
    import numpy as np
    import torch

    import synth

    pool_n = 4096 * 1024
    pool = np.frombuffer(synth.to_pcm_bytes(synth.synth_samples(pool_n, ch, bits, rate, stream=stream), bits),
                         dtype=np.uint8)
    files = []
    for i in range(n_files):
        buf = torch.empty(n * fb, dtype=torch.uint8, pin_memory=True).numpy()
        pos, k = 0, i
        while pos < n:
            take = min(n - pos, pool_n - 4096 * (k % 64))
            a = 4096 * (k % 64) * fb
            buf[pos * fb:(pos + take) * fb] = pool[a:a + take * fb]
            pos += take
            k += 7
        files.append(buf)
    return files


def end_to_end_node(args, rank, world, dist, dev):
    """The end-to-end contract on EVERY rank at once (N > 1): each rank encodes its own files
    (host PCM -> .flac in host memory, one flacgpu_encode_files call on its GPU, MD5s on its share of
    the host pool), the calls bracketed by barriers; node value = every rank's samples / the slowest
    rank's wall.  File 0 of every rank is compared with the restatement's whole-file encode."""
    import torch

    import flacgpu

    ch, bits, rate = 2, 16, 44100
    n = int(args.e2e_minutes * 60 * rate)
    fb = ch * 2
    nf = args.e2e_node_files
    local = gpu_local_cpus(torch.cuda.current_device()) if args.e2e_numa == "local" else None
    saved_aff = os.sched_getaffinity(0)
    if local:
        move_process(local)
    files = e2e_files(nf, n, fb, ch, bits, rate, stream=11 + rank)
    L = flacgpu.load_library()
    enc = flacgpu.Encoder(ch, bits, rate, device=torch.cuda.current_device(), max_frames=args.e2e_max_frames)
    cap = 200 + ((n + 4095) // 4096 + 1) * enc.frame_bound()
    outs = [torch.empty(cap, dtype=torch.uint8, pin_memory=True).numpy() for _ in files]
    fp = (ctypes.c_void_p * nf)(*[f.ctypes.data for f in files])
    op = (ctypes.c_void_p * nf)(*[o.ctypes.data for o in outs])
    ns = (ctypes.c_uint64 * nf)(*([n] * nf))
    caps = (ctypes.c_size_t * nf)(*([cap] * nf))
    bl = (ctypes.c_size_t * nf)()

    def call():
        return L.flacgpu_encode_files(enc.ctx, nf, fp, 2, ns, op, caps, bl)

    rc = call()  # warm-up (pool threads, pinned mappings)
    walls = []
    for _ in range(2):
        dist.barrier()
        t0 = time.perf_counter()
        rc |= call()
        dt = time.perf_counter() - t0
        dist.barrier()
        walls.append(dt)
    wall = min(walls)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_ref

    ok = rc == 0 and outs[0][: bl[0]].tobytes() == oracle_ref.encode_file(files[0].tobytes(), ch, bits, rate)
    t = torch.tensor([wall, float(nf * n), 0.0 if ok else 1.0], dtype=torch.float64, device=dev)
    tmax = t.clone()
    dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    enc.close()
    if local:
        move_process(saved_aff)
    max_wall, samples, bad = float(tmax[0].item()), float(t[1].item()), float(t[2].item())
    return {"value": round(samples / max_wall / 1e6, 1), "unit": "MSamples/s", "ranks": world,
            "files": nf * world, "files_per_rank": nf, "mode": "batch", "minutes_per_file": args.e2e_minutes,
            "wall_ms": round(max_wall * 1e3, 2), "rank0_wall_ms": round(wall * 1e3, 2),
            "path": "every rank at once: pinned host PCM -> .flac in pinned host memory, one flacgpu_encode_files "
                    "call per rank on its own GPU (MD5s on that rank's share of the host pool); node value = "
                    "sum of every rank's samples / the slowest rank's wall (barrier before and after)",
            "output_ok": bad == 0}


def e2e_many_point(args, nmax, n, ch, bits, rate, fb):
    """One flacgpu_encode_files batch of args.e2e_many files holding the same total samples as nmax
    files of n (shorter files), with its host-MD5 bound; file 0 checked against the restatement."""
    import torch

    import flacgpu

    nm = args.e2e_many
    nn = (n * nmax // nm) // 4096 * 4096 + 1234  # ragged last frame, as the full-length files
    files = e2e_files(nm, nn, fb, ch, bits, rate, stream=23)
    L = flacgpu.load_library()
    enc = flacgpu.Encoder(ch, bits, rate, device=torch.cuda.current_device(), max_frames=args.e2e_max_frames)
    cap = 200 + ((nn + 4095) // 4096 + 1) * enc.frame_bound()
    outs = [torch.empty(cap, dtype=torch.uint8, pin_memory=True).numpy() for _ in files]
    fp = (ctypes.c_void_p * nm)(*[f.ctypes.data for f in files])
    op = (ctypes.c_void_p * nm)(*[o.ctypes.data for o in outs])
    ns = (ctypes.c_uint64 * nm)(*([nn] * nm))
    caps = (ctypes.c_size_t * nm)(*([cap] * nm))
    bl = (ctypes.c_size_t * nm)()
    rc = L.flacgpu_encode_files(enc.ctx, nm, fp, 2, ns, op, caps, bl)  # warm-up
    best = None
    for _ in range(2):
        t0 = time.perf_counter()
        rc |= L.flacgpu_encode_files(enc.ctx, nm, fp, 2, ns, op, caps, bl)
        dt = time.perf_counter() - t0
        best = dt if best is None else min(best, dt)
    md5_alone = min(_timed(lambda: flacgpu.md5_many(files)) for _ in range(2))
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_ref

    ok = rc == 0 and outs[0][: bl[0]].tobytes() == oracle_ref.encode_file(files[0].tobytes(), ch, bits, rate)
    out_b = sum(bl[i] for i in range(nm))
    enc.close()
    return {"files": nm, "minutes_per_file": round(nn / rate / 60, 3), "value": round(nm * nn / best / 1e6, 1),
            "wall_ms": round(best * 1e3, 2), "md5_pool_alone_ms": round(md5_alone * 1e3, 2),
            "frac_of_md5_bound": round(md5_alone / best, 3),
            "h2d_gbs": round(nm * nn * fb / best / 1e9, 2), "d2h_gbs": round(out_b / best / 1e9, 2), "ok": bool(ok)}


def end_to_end(args):
    """BASELINE.md end-to-end contract: host PCM buffers -> .flac files in host memory, as a curve
    over the number of files encoded at once, per file (one context + host thread each) and as one
    batch call (flacgpu_encode_files), every MD5 on the host pool beside the GPU encode; bounds per
    point: the same files' MD5 alone on the pool, and (per file) the frames path alone."""
    import numpy as np
    import torch

    import flacgpu
    import synth

    ch, bits, rate = 2, 16, 44100
    n = int(args.e2e_minutes * 60 * rate)
    fb = ch * 2
    counts = sorted({int(x) for x in str(args.e2e_files).split(",") if x})
    saved_aff = os.sched_getaffinity(0)
    local = gpu_local_cpus(torch.cuda.current_device()) if args.e2e_numa == "local" else None
    if local:
        move_process(local)  # before the buffers are allocated and first touched
    nmax = max(counts)

    def pinned(nbytes):
        return torch.empty(nbytes, dtype=torch.uint8, pin_memory=True).numpy()

    files = e2e_files(nmax, n, fb, ch, bits, rate)
    L = flacgpu.load_library()
    # 6144 frames (default): three chunk sets of 2048 frames (32 MiB of PCM) for the pipelined schedule
    encs = [flacgpu.Encoder(ch, bits, rate, device=torch.cuda.current_device(), max_frames=args.e2e_max_frames)
            for _ in files]
    cap = 200 + ((n + 4095) // 4096 + 1) * encs[0].frame_bound()
    outs = [pinned(cap) for _ in files]
    lens = [ctypes.c_size_t(0) for _ in files]
    rcs = [0] * nmax

    def one(i):
        rcs[i] = L.flacgpu_encode_file(encs[i].ctx, files[i].ctypes.data_as(ctypes.c_void_p), 2, n,
                                       outs[i].ctypes.data_as(ctypes.c_void_p), cap, ctypes.byref(lens[i]))

    def frames_only(i):
        # the same path without the MD5 and header: flacgpu_encode_frames (H2D, kernels, D2H)
        n_out = ctypes.c_size_t(0)
        rcs[i] = L.flacgpu_encode_frames(encs[i].ctx, files[i].ctypes.data_as(ctypes.c_void_p), 2, n, 0,
                                         outs[i].ctypes.data_as(ctypes.c_void_p), cap, ctypes.byref(n_out), None)

    def batch(nf):
        # one context, one call: flacgpu_encode_files (one pipelined schedule, MD5s batched)
        fp = (ctypes.c_void_p * nf)(*[f.ctypes.data for f in files[:nf]])
        op = (ctypes.c_void_p * nf)(*[o.ctypes.data for o in outs[:nf]])
        ns = (ctypes.c_uint64 * nf)(*([n] * nf))
        caps = (ctypes.c_size_t * nf)(*([cap] * nf))
        bl = (ctypes.c_size_t * nf)()
        t0 = time.perf_counter()
        rc = L.flacgpu_encode_files(encs[0].ctx, nf, fp, 2, ns, op, caps, bl)
        dt = time.perf_counter() - t0
        for i in range(nf):
            lens[i].value = bl[i]
        return dt, rc

    def run_all(nf, fn=one):
        th = [threading.Thread(target=fn, args=(i,)) for i in range(nf)]
        t0 = time.perf_counter()
        for t in th:
            t.start()
        for t in th:
            t.join()
        return time.perf_counter() - t0

    run_all(min(nmax, 8))
    curve = []
    for nf in counts:
        best = min(run_all(nf) for _ in range(2))
        # the host-MD5 bound at this file count: the same files' MD5 alone on the library's pool
        # (flacgpu_md5_many: what the encode's hashing does, with no GPU work or other threads)
        md5_alone = min(_timed(lambda: flacgpu.md5_many(files[:nf])) for _ in range(2))
        ok_nf = all(r == 0 for r in rcs[:nf])
        # ... and the GPU + PCIe path alone (frames only, no MD5): the other bound
        frames_alone = min(run_all(nf, frames_only) for _ in range(2))
        ok_nf &= all(r == 0 for r in rcs[:nf])
        bound = max(md5_alone, frames_alone)
        # the batch API on one context (flacgpu_encode_files)
        bt = [batch(nf) for _ in range(2)]
        bbest = min(t for t, _ in bt)
        ok_b = all(rc == 0 for _, rc in bt)
        out_b = sum(lens[i].value for i in range(nf))
        curve.append({"files": nf, "value": round(nf * n / best / 1e6, 1), "wall_ms": round(best * 1e3, 2),
                      "md5_pool_alone_ms": round(md5_alone * 1e3, 2),
                      "frames_alone_ms": round(frames_alone * 1e3, 2),
                      "frac_of_md5_bound": round(md5_alone / best, 3),
                      "frac_of_bound": round(bound / best, 3),
                      "binding": "host_md5" if md5_alone >= frames_alone else "gpu_pcie_frames",
                      "batch": {"value": round(nf * n / bbest / 1e6, 1), "wall_ms": round(bbest * 1e3, 2),
                                "frac_of_md5_bound": round(md5_alone / bbest, 3), "ok": ok_b,
                                # the schedule's PCIe traffic: PCM up + frames down over the batch's wall
                                "h2d_gbs": round(nf * n * fb / bbest / 1e9, 2), "d2h_gbs": round(out_b / bbest / 1e9, 2)},
                      "ok": ok_nf and ok_b})
    ok = all(c["ok"] for c in curve)
    # bounds: one file's MD5 on one host core; pinned H2D bandwidth
    t0 = time.perf_counter()
    hashlib.md5(files[0]).digest()
    md5_s = time.perf_counter() - t0
    d = torch.empty(len(files[0]), dtype=torch.uint8, device=torch.cuda.current_device())
    src = torch.from_numpy(files[0])
    d.copy_(src, non_blocking=True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(4):
        d.copy_(src, non_blocking=True)
    torch.cuda.synchronize()
    h2d_gbs = 4 * len(files[0]) / (time.perf_counter() - t0) / 1e9
    del d
    share = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or len(os.sched_getaffinity(0))
    md5_gbs = len(files[0]) / md5_s / 1e9
    # proof: file 0 is byte-identical to the restatement's whole-file encode (header, MD5, frames)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_ref

    ref = oracle_ref.encode_file(files[0].tobytes(), ch, bits, rate)
    ok &= outs[0][: lens[0].value].tobytes() == ref  # the batch call's file 0 (the last run)
    one(0)
    ok &= rcs[0] == 0 and outs[0][: lens[0].value].tobytes() == ref  # and the per-file call's
    for e in encs:
        e.close()
    many = None
    if args.e2e_many > nmax:
        # the same bytes as the largest point, cut into more, shorter files: more MD5 chains per pool
        # worker (the AVX-512 sixteen-chain path takes over past six), so the host-MD5 bound moves up
        # and the PCIe schedule is what is left
        del files, outs
        try:
            torch._C._host_emptyCache()  # the cached pinned blocks of the curve's buffers
        except Exception:
            pass
        many = e2e_many_point(args, nmax, n, ch, bits, rate, fb)
        ok &= many["ok"]
    if local:
        move_process(saved_aff)
    runs = [(c["value"], c["files"], c["wall_ms"], "per_file", args.e2e_minutes) for c in curve] + \
           [(c["batch"]["value"], c["files"], c["batch"]["wall_ms"], "batch", args.e2e_minutes) for c in curve]
    if many:
        runs.append((many["value"], many["files"], many["wall_ms"], "batch", many["minutes_per_file"]))
    top = max(runs)
    big = max(curve, key=lambda c: c["files"])
    return {"files": top[1], "mode": top[3], "minutes_per_file": top[4], "samples": int(top[1] * top[4] * 60 * rate),
            "many_files": many,
            "batch_gbs": [big["batch"]["h2d_gbs"], big["batch"]["d2h_gbs"]],
            "value": top[0], "unit": "MSamples/s", "wall_ms": top[2], "curve": curve,
            "md5_one_file_host_core_ms": round(md5_s * 1e3, 2),
            "bounds_msamples_per_s": {
                "pcie_h2d_pinned": round(h2d_gbs * 1e3 / fb, 1), "h2d_gbs": round(h2d_gbs, 2),
                "host_md5_cores_x_rate": round(share * md5_gbs * 1e3 / fb, 1), "cores": share,
                "one_file_md5_floor_ms": round(md5_s * 1e3, 2)},
            "path": "pinned host PCM -> .flac in pinned host memory (73-byte header + frames), two ways: "
                    "per_file = flacgpu_encode_file per file (one context + host thread each), batch = ONE "
                    "flacgpu_encode_files call on one context (one pipelined H2D / kernels / D2H schedule in "
                    "2048-frame chunks running on from file to file); every file's MD5 on the library's host "
                    "hashing pool beside the encode (up to 8 chains interleaved per core, fg_md5_host.cpp)",
            "md5_pool_threads": os.environ.get("FLACGPU_MD5_THREADS", "default (CPUs of the affinity mask)"),
            "numa": {"mode": args.e2e_numa, "gpu_local_cpus": len(local) if local else None},
            "output_ok": bool(ok)}


# ---------------------------------------------------------------------------------------------
def cpu_facts():
    facts = {"model": None, "cores_per_socket": None, "sockets": None}
    try:
        for line in subprocess.run(["lscpu"], capture_output=True, text=True).stdout.splitlines():
            k, _, v = line.partition(":")
            v = v.strip()
            if k == "Model name":
                facts["model"] = v
            elif k == "Core(s) per socket":
                facts["cores_per_socket"] = int(v)
            elif k == "Socket(s)":
                facts["sockets"] = int(v)
    except Exception:
        pass
    return facts


def _cpulist(txt):
    cpus = []
    for part in txt.strip().split(","):
        if part:
            a, _, b = part.partition("-")
            cpus += list(range(int(a), int(b or a) + 1))
    return cpus


def socket0_cpus():
    try:
        avail = os.sched_getaffinity(0)
        return [c for c in _cpulist(open("/sys/devices/system/node/node0/cpulist").read()) if c in avail]
    except Exception:
        return sorted(os.sched_getaffinity(0))


def cpu_busy(interval=0.3):
    """Busy fraction of every CPU of this process's mask over `interval` seconds (/proc/stat), or {}."""
    def snap():
        d = {}
        for line in open("/proc/stat"):
            if line.startswith("cpu") and line[3:4].isdigit():
                f = line.split()
                v = [int(x) for x in f[1:]]
                idle = v[3] + (v[4] if len(v) > 4 else 0)
                d[int(f[0][3:])] = (sum(v), idle)
        return d
    try:
        s0 = snap()
        time.sleep(interval)
        s1 = snap()
    except Exception:
        return {}
    avail = os.sched_getaffinity(0)
    out = {}
    for c, (t1, i1) in s1.items():
        if c in avail and c in s0:
            dt = t1 - s0[c][0]
            out[c] = 1.0 - (i1 - s0[c][1]) / dt if dt > 0 else 0.0
    return out


def pick_cores(P, place="idle"):
    """P CPUs for the CPU-baseline threads, one per physical core.
    idle    -- the least busy physical cores of the process's mask (/proc/stat over 0.3 s; a core's
               load = its busiest SMT sibling), so that the sample does not share cores with other
               work on the machine (the GPU box is one slice of a shared host: the first cores of
               socket 0 are the ones everybody else's pinned threads land on too);
    socket0 -- the first P CPUs of NUMA node 0 (rounds 1-5);
    none    -- no pinning (the threads float)."""
    if place == "none":
        return None, {}
    if place == "socket0":
        return socket0_cpus(), {}
    avail = sorted(os.sched_getaffinity(0))
    busy = cpu_busy()
    seen, cores = set(), []
    for c in avail:
        if c in seen:
            continue
        try:
            sib = [x for x in _cpulist(open(f"/sys/devices/system/cpu/cpu{c}/topology/thread_siblings_list").read())
                   if x in avail]
        except Exception:
            sib = [c]
        seen.update(sib)
        cores.append((max(busy.get(x, 0.0) for x in sib), c))
    cores.sort()
    chosen = [c for _, c in cores[:P]]
    load = [round(b, 3) for b, _ in cores[:P]]
    return chosen, {"physical_cores_in_mask": len(cores), "chosen_busy_max": max(load) if load else None,
                    "chosen_busy_mean": round(sum(load) / len(load), 3) if load else None}


def _cpu_run(L, oracle_ref, buf, args, P, seconds, cpus, lpc):
    """P threads (thread t pinned to cpus[t], or floating if cpus is None), each encoding whole
    8-block streams (incl. MD5) of `buf` one after another until `seconds` have passed: a fixed-time
    throughput sample (no tail of one late thread); -> (samples, s) where s = the time the last
    thread finished its last stream."""
    ch, bits = args.channels, args.bits
    fb = ch * (bits // 8)
    per_stream = 8 * 4096  # 8-block streams, the headline's shape
    n_streams_buf = len(buf) // (per_stream * fb)
    cfg = oracle_ref.config(ch, bits, args.rate, lpc=lpc)
    res = [0] * P
    fin = [0.0] * P
    cap = 8 * L.oracle_max_frame_bytes(4096, bits, ch) + 64
    go = threading.Barrier(P)
    beg = [0.0] * P

    def run(t):
        if cpus:
            try:
                os.sched_setaffinity(0, {cpus[t % len(cpus)]})  # this thread only
            except Exception:
                pass
        out = ctypes.create_string_buffer(cap)
        sizes = (ctypes.c_uint32 * 8)()
        md5 = ctypes.create_string_buffer(16)
        done, j = 0, 0
        go.wait()  # threads placed and buffers allocated: the clock starts with the first encode
        beg[t] = t0 = time.perf_counter()
        while True:
            s = (t + j * P) % n_streams_buf
            base = buf.ctypes.data + s * per_stream * fb
            r = L.oracle_encode_stream(ctypes.byref(cfg), ctypes.c_void_p(base), bits // 8, ctypes.c_uint64(per_stream),
                                       ctypes.c_uint64(0), out, ctypes.c_size_t(cap), sizes, md5)
            done += per_stream if r > 0 else 0
            j += 1
            now = time.perf_counter()
            if now - t0 >= seconds:
                break
        res[t], fin[t] = done, now

    th = [threading.Thread(target=run, args=(t,)) for t in range(P)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    return sum(res), max(fin) - min(beg)


def _best_of(fn, reps):
    """reps runs of fn() -> (samples, s); -> (best rate, [every rate]) in MSamples/s."""
    rates = []
    for _ in range(reps):
        tot, dt = fn()
        rates.append(tot / dt / 1e6)
    return max(rates), rates


def _spread(rates):
    rs = sorted(rates)
    return {"best": round(rs[-1], 3), "median": round(rs[len(rs) // 2], 3), "worst": round(rs[0], 3),
            "spread": round((rs[-1] - rs[0]) / rs[-1], 4) if rs[-1] else None, "runs": [round(r, 3) for r in rates]}


HEALTH_MIN = 0.9  # per-core rate at P threads / single-core rate below this: the sample was disturbed


def cpu_baseline(buf, args, reps=None, place=None):
    """The CPU restatement (oracle/, built -O3 -march=x86-64-v4 as liboracle_fast.so): one thread
    (one core, the reference's own shape: wav2flac is single-threaded) and P threads on P distinct
    physical cores, each encoding whole streams (incl. MD5); best of `reps` runs of each.  LPC
    configs are also run fixed-only, which is what the reference (no LPC, readme.md:27) does on the
    same input.  main() runs this BEFORE torch is imported or any HIP call is made (no GPU runtime
    threads, no host MD5 pool, no pinned buffers yet), so the sample has the host to itself.
    `health` = (P-thread rate / P) / single-core rate: below HEALTH_MIN the P-thread sample did not
    scale (shared cores, clock drop) and the line says so."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_ref

    reps = reps or args.cpu_reps
    place = place or args.cpu_place
    L = oracle_ref.lib(fast=True)
    facts = cpu_facts()
    share = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or len(os.sched_getaffinity(0))
    P = args.cpu_threads or min(share, facts["cores_per_socket"] or share)
    try:
        main_aff = os.sched_getaffinity(0)
    except Exception:
        main_aff = None
    cpus, pinfo = pick_cores(P, place)
    if cpus is not None and len(cpus) < P:
        P = len(cpus)  # fewer physical cores in the mask than the share: one thread per core
    one_cpu = cpus[:1] if cpus else None
    sec = args.cpu_seconds
    best1, r1 = _best_of(lambda: _cpu_run(L, oracle_ref, buf, args, 1, 1.5 * sec, one_cpu, args.lpc), reps)
    bestP, rP = _best_of(lambda: _cpu_run(L, oracle_ref, buf, args, P, sec, cpus, args.lpc), reps)
    fixed_only = None
    if args.lpc:
        bestf, rf = _best_of(lambda: _cpu_run(L, oracle_ref, buf, args, P, sec, cpus, 0), reps)
        fixed_only = {"value": round(bestf, 3), "cores": P, **{k: v for k, v in _spread(rf).items() if k != "best"},
                      "note": "LPC off: the reference's own encoding of this input (it has no LPC)"}
    if main_aff:
        try:
            os.sched_setaffinity(0, main_aff)
        except Exception:
            pass
    cps = facts["cores_per_socket"]
    health = bestP / P / best1 if best1 else None
    return {
        "value": round(bestP, 3),
        "unit": "MSamples/s",
        "cores": P,
        "kind": "port",
        "sample": f"{P} threads on {P} physical cores ({place}) encoding 8-block streams (incl. MD5) of a "
                  f"{len(buf) >> 20}-MiB input for {sec:g} s per run, best of {reps}, before any GPU/torch init",
        "reps": reps,
        "spread": _spread(rP),
        "single_core": {"value": round(best1, 3), "cores": 1, **{k: v for k, v in _spread(r1).items() if k != "best"},
                        "sample": f"one thread on one core for {1.5 * sec:g} s per run"},
        "health": round(health, 4) if health else None,
        "health_ok": bool(health and health >= HEALTH_MIN),
        "health_note": (f"per-core rate at {P} threads / single-core rate (best samples); >= {HEALTH_MIN}: the "
                        "P-thread sample scaled" if health and health >= HEALTH_MIN else
                        f"per-core rate at {P} threads is {health:.2f} of single-core (< {HEALTH_MIN}): the "
                        "P-thread sample did NOT scale linearly on this host (shared cores or all-core clock drop); "
                        "the socket estimate below uses the measured per-core rate at P threads") if health else None,
        "placement": {"mode": place, "cpus": cpus, **pinfo},
        "fixed_only": fixed_only,
        "lpc": args.lpc,
        "cpu_model": facts["model"],
        "cores_per_socket": cps,
        "sockets": facts["sockets"],
        "build": "oracle/flac_oracle.c -O3 -march=x86-64-v4 (C restatement, CRC-16 by slicing-by-8 tables "
                 "since r3w where the reference folds with PCLMUL; the Zig reference is unbuildable here: no "
                 "Zig 0.16 on the box)",
        "per_core": round(bestP / P, 3),
        "single_socket_estimate": round(bestP / P * cps, 1) if cps else None,
        "single_socket_note": f"measured at P = {P} threads (the box's CPU share for one GPU) of {cps} cores per "
                              "socket; the socket figure scales the best P-thread sample's per-core rate linearly "
                              "(an ESTIMATE, an upper bound: memory bandwidth and clocks are shared)",
    }


def cpu_input(args, cfg, rank=0):
    """The CPU legs' input: the same generator as the GPU step (build_input) for `cfg`, sized to the
    CPU sample (CPU_FRAMES blocks), not to the GPU step."""
    sub = argparse.Namespace(**vars(args))
    sub.config = cfg
    sub.channels, sub.bits, sub.rate, sub.lpc = PRESETS[cfg]
    sub.cpu_frames = args.cpu_frames if cfg == (args.config or "c2") else CPU_FRAMES[cfg]
    F = 16 if cfg == "c2" else 4  # blocks per stream of the GPU step (headline / --configs lines)
    sub.frames = -(-sub.cpu_frames // F) * F
    sub.streams = sub.frames // F
    return sub, build_input(sub, rank)


def cpu_legs(args, cfgs):
    """Every CPU-baseline leg of the run, measured first (main() calls this before torch)."""
    out = {}
    for cfg in cfgs:
        sub, buf = cpu_input(args, cfg)
        out[cfg] = cpu_baseline(buf, sub)
        del buf
    return out


# ---------------------------------------------------------------------------------------------
# roofline of one configuration's step, from HIP events (bench) + the committed PMC summary
VALU_PEAK = 1024 * 0.5 * 2.4e9  # wave64 VALU instructions/s: 1024 SIMD-32s x 1 per 2 cycles x 2.4 GHz
SIMD_CYCLES_PER_S = 1024 * 2.4e9  # SIMD-cycles per second over the chip (weighted issue: tools/valu_rates.py)


def roofline_of(args, kt, steps, pcm_bytes, out_bytes, ms_per_step, key):
    """The step's roofline.  `bound` is the resource that binds (VALU issue: Sigma SQ_INSTS_VALU of
    every kernel of the step / (VALU peak x step time), from the committed PMC of this workload);
    achieved / peak / frac price the dominant kernel against HBM (the contract's figure, kept
    beside it).  Every kernel's own figures are in `kernels`."""
    per_launch = {name: (v[1] / v[0]) / 1e3 for name, v in kt.items() if v[0]}
    # launches per step: 1, or the range count of the overlapped schedule (FLACGPU_OVERLAP)
    lps = {name: max(1, round(v[0] / steps)) for name, v in kt.items() if v[0]}
    # The encode kernels run in sequence on the step's stream (analysis -> scan -> pack), the MD5
    # beside them on its own stream: while the MD5's chain is shorter than the encode path the
    # dominant kernel is the longest encode kernel, otherwise the MD5.
    path_s = sum(per_launch.get(k, 0.0) * lps.get(k, 1) for k in ("analyze", "analyze_tail", "scan", "pack"))
    fused = "pack" not in per_launch and "analyze" in per_launch  # FLACGPU_FUSED: no pack launch
    algo = {"analyze": pcm_bytes + (out_bytes if fused else 0), "pack": pcm_bytes + out_bytes, "md5": pcm_bytes}
    algo = {k: v // lps.get(k, 1) for k, v in algo.items()}
    valu_step, valu_src, valu_missing = 0.0, None, []

    def kernel_roofline(k):
        avg = per_launch[k]
        ach = algo[k] / avg / 1e9
        traffic, counters, src = read_pmc(key, k)
        issue = None
        if counters.get("SQ_INSTS_VALU"):
            cpi, msrc = read_valu_mix(args.config or "c2", k)
            issue = {"valu_wave_instr_per_launch": counters["SQ_INSTS_VALU"], "peak_valu_wave_instr_per_s": VALU_PEAK,
                     "valu_issue_frac": round(counters["SQ_INSTS_VALU"] / avg / VALU_PEAK, 4),
                     # SIMD-cycles the mix needs at the measured per-opcode rates / SIMD-cycles available
                     "weighted_issue_frac": round(counters["SQ_INSTS_VALU"] * cpi / avg / SIMD_CYCLES_PER_S, 4)
                     if cpi else None, "cycles_per_instr": cpi, "mix_source": msrc,
                     "waves_per_launch": counters.get("SQ_WAVES"), "source": src}
        return {"achieved": round(ach, 2), "frac": round(ach / HBM_PEAK_GBS, 5),
                "frac_vs_6p29": round(ach / HBM_COPY_GBS, 5), "avg_launch_ms": round(avg * 1e3, 4),
                "algorithmic_bytes_per_launch": algo[k], "traffic": traffic, "traffic_source": src,
                "traffic_ratio": round(traffic / algo[k], 3) if traffic else None, "issue": issue}

    wcyc_step, wcyc_ok = 0.0, True
    for k in per_launch:
        _, counters, src = read_pmc(key, k)
        if counters.get("SQ_INSTS_VALU"):
            valu_step += counters["SQ_INSTS_VALU"] * lps[k]
            valu_src = src
            cpi, _ = read_valu_mix(args.config or "c2", k)
            if cpi:
                wcyc_step += counters["SQ_INSTS_VALU"] * lps[k] * cpi
            elif k in ("analyze", "pack", "md5"):
                wcyc_ok = False
        elif k in ("analyze", "pack", "md5"):
            valu_missing.append(k)
    enc_k = [k for k in ("analyze", "pack") if k in per_launch]
    md5_off_path = "md5" not in per_launch or per_launch["md5"] < path_s
    dom = max(enc_k, key=lambda k: per_launch[k] * lps[k]) if md5_off_path else "md5"
    rk = {k: kernel_roofline(k) for k in ("analyze", "pack", "md5") if k in per_launch}
    achieved = algo[dom] / per_launch[dom] / 1e9
    step_issue = round(valu_step / (VALU_PEAK * ms_per_step / 1e3), 4) if valu_step and not valu_missing else None
    weighted = (round(wcyc_step / (SIMD_CYCLES_PER_S * ms_per_step / 1e3), 4)
                if valu_step and not valu_missing and wcyc_ok and wcyc_step else None)
    return {
        "bound": "valu-issue",
        "step_issue_frac": step_issue,
        "weighted_issue_frac": weighted,
        "weighted_issue_note": "Sigma SQ_INSTS_VALU x SIMD-cycles per instruction of each kernel's mix (measured "
                               "per-opcode rates, profiles/r5_issue_micro.txt; static mix, tools/valu_rates.py) / "
                               "(1024 SIMDs x 2.4 GHz x ms_per_step)",
        "step_issue_note": ("Sigma SQ_INSTS_VALU per launch x launches per step over every kernel of the step "
                            f"({valu_src}) / ({VALU_PEAK:.4g} wave-instr/s x ms_per_step)" if step_issue is not None
                            else f"no committed PMC summary for workload {key} (kernels {valu_missing})"),
        "limiter": LIMITER[dom],
        "kernel": {"analyze": "k_analyze<..., FP> (fused analysis + pack, 4096-sample frames)" if fused
                   else "k_analyze (4096-sample frames)", "pack": "k_pack4 / k_packw / k_pack",
                   "md5": "k_md5_streams_lds"}[dom],
        "achieved": round(achieved, 2),
        "peak": HBM_PEAK_GBS,
        "unit": "GB/s",
        "frac": round(achieved / HBM_PEAK_GBS, 5),
        "frac_vs_6p29": round(achieved / HBM_COPY_GBS, 5),
        "hbm_frac": round(achieved / HBM_PEAK_GBS, 5),
        "traffic": rk[dom]["traffic"],
        "traffic_source": rk[dom]["traffic_source"],
        "algorithmic_bytes_per_launch": algo[dom],
        "avg_launch_ms": round(per_launch[dom] * 1e3, 4),
        "launches": kt[dom][0],
        "launches_per_step": lps[dom],
        "encode_path_gbs": round((pcm_bytes + out_bytes) / path_s / 1e9, 2) if path_s > 0 else None,
        "issue": rk[dom]["issue"],
        "selection": "longest encode kernel on the step's critical path (the MD5 chain, "
                     f"{per_launch.get('md5', 0) * 1e3:.3f} ms, runs beside the {path_s * 1e3:.3f}-ms encode path)"
                     if md5_off_path else "the MD5 chain is longer than the encode path: it bounds the step",
        "kernels": rk,
    }


def workload_text(args, F):
    cfg = (args.config or "c2").upper()
    return (f"{cfg}: {args.rate/1000:g}kHz {args.bits}-bit {args.channels}ch, blocksize 4096, "
            f"{args.streams} concurrent streams/GPU x {F} blocks each per step "
            f"({args.frames} blocks/step), frame numbers + per-stream MD5 state carried across "
            "steps, " + (f"LPC orders 1..{args.lpc} + full subframe-type search" if args.lpc else "fixed prediction") +
            (", MD5 off (diagnostic)" if args.no_md5 else ", MD5 on its own HIP stream beside the next step's encode"))


def rate_units(value, channels, rate):
    """SURVEY §8(d)'s companions of the interchannel-sample metric: channel samples per second and
    the multiple of real time (seconds of audio encoded per second) for the same throughput."""
    return {"channel_msamples_per_s": round(value * channels, 1), "x_realtime": round(value * 1e6 / rate, 1)}


def config_line(args, cfg, dist, rank, world, dev, cpu=None):
    """One BASELINE config (c3 / c4 / c5) as its own timed line inside the default run: its preset,
    65536-block steps, barrier + max over ranks, output compared with the oracle after timing, the
    CPU port timed on rank 0 at N = 1 (one core, P cores, and fixed-only for the LPC configs)."""
    import numpy as np
    import torch

    import flacgpu

    sub = argparse.Namespace(**vars(args))
    sub.config = cfg
    sub.channels, sub.bits, sub.rate, sub.lpc = PRESETS[cfg]
    sub.frames, sub.streams = args.cfg_frames, args.streams
    sub.cpu_frames = CPU_FRAMES[cfg]
    buf = build_input(sub, rank)
    fb = sub.channels * (sub.bits // 8)
    enc = flacgpu.Encoder(sub.channels, sub.bits, sub.rate, device=torch.cuda.current_device(),
                          max_frames=sub.frames, lpc_order=sub.lpc)
    d_pcm = torch.from_numpy(buf).to(dev)
    F = sub.frames // sub.streams
    w = Workload(enc, d_pcm, sub.streams, F, fb, dev, md5=not args.no_md5)
    elapsed = run_timed(w, args.cfg_steps, args.warmup, dist)
    if dist:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    kt = kernel_times(enc)
    pcm_bytes = sub.frames * 4096 * fb
    out_bytes = int(w.d_fb.cpu().numpy().astype(np.int64).sum())
    ms = elapsed / args.cfg_steps * 1e3
    ok, vinfo = verify(sub, w, buf, fb, min(args.verify_streams, 32), dev) if rank == 0 else (True, {})
    w.close()
    enc.close()
    del d_pcm
    torch.cuda.empty_cache()
    line = None
    if rank == 0:
        line = {"config": cfg, "workload": workload_text(sub, F), "workload_key": workload_key(sub),
                "value": round(sub.frames * 4096 * world * args.cfg_steps / elapsed / 1e6, 2), "unit": "MSamples/s",
                "n_gpus": world, "steps": args.cfg_steps, "ms_per_step": round(ms, 4),
                "kernel_ms_per_step": {k: round(v[1] / args.cfg_steps, 4) for k, v in kt.items() if v[0]},
                "compression_ratio": round(out_bytes / pcm_bytes, 4),
                "roofline": roofline_of(sub, kt, args.cfg_steps, pcm_bytes, out_bytes, ms, workload_key(sub)),
                "output_ok": ok, "verified": vinfo, "cpu_baseline": None}
        line["units"] = rate_units(line["value"], sub.channels, sub.rate)
        if cpu:  # measured before torch (main(), cpu_legs)
            line["cpu_baseline"] = cpu
            line["vs_cpu_single_socket_estimate"] = (round(line["value"] / line["cpu_baseline"]["single_socket_estimate"], 1)
                                                     if line["cpu_baseline"].get("single_socket_estimate") else None)
    return line


# ---------------------------------------------------------------------------------------------
# the stdout line: the driver keeps only the tail of stdout (about 8 KB), so the line it parses is a
# compact summary of at most LINE_MAX bytes; the full record goes to a sidecar file (`detail`)
LINE_MAX = 4096


def _r(x, nd=4):
    return round(x, nd) if isinstance(x, float) else x


def _compact_roofline(r):
    if not r:
        return None
    ks = {}
    for k, v in (r.get("kernels") or {}).items():
        ks[k] = {"ms": v.get("avg_launch_ms"), "frac": _r(v.get("frac")), "traffic_ratio": v.get("traffic_ratio"),
                 "issue": (v.get("issue") or {}).get("valu_issue_frac"),
                 "w_issue": (v.get("issue") or {}).get("weighted_issue_frac")}
    out = {"bound": r.get("bound"), "kernel": r.get("kernel"), "achieved": r.get("achieved"), "peak": r.get("peak"),
           "unit": r.get("unit"), "frac": r.get("frac"), "frac_vs_6p29": r.get("frac_vs_6p29"),
           "peak_measured_copy": HBM_COPY_GBS, "traffic": r.get("traffic"),
           "traffic_ratio": (r.get("kernels") or {}).get(_dom_name(r), {}).get("traffic_ratio"),
           "algorithmic_bytes_per_launch": r.get("algorithmic_bytes_per_launch"),
           "avg_launch_ms": r.get("avg_launch_ms"), "step_issue_frac": r.get("step_issue_frac"),
           "kernels": ks}
    if r.get("weighted_issue_frac") is not None:
        out["weighted_issue_frac"] = r["weighted_issue_frac"]
    return out


def _dom_name(r):
    kern = r.get("kernel") or ""
    return "md5" if "md5" in kern else ("pack" if "pack" in kern and "analyze" not in kern else "analyze")


def _compact_cpu(c):
    if not c:
        return None
    sp = c.get("spread") or {}
    return {"value": c.get("value"), "unit": c.get("unit"), "cores": c.get("cores"), "kind": c.get("kind"),
            "sample": c.get("sample", "")[:120],
            "reps": c.get("reps"), "median": sp.get("median"), "spread": sp.get("spread"),
            "single_core": (c.get("single_core") or {}).get("value"),
            "health": c.get("health"), "health_ok": c.get("health_ok"),
            "single_socket_estimate": c.get("single_socket_estimate"),
            "fixed_only": (c.get("fixed_only") or {}).get("value"), "cpu_model": c.get("cpu_model")}


def compact_line(full: dict, detail_path: str | None = None) -> dict:
    """The driver-parsed stdout line built from the full record: the contract keys, a compact
    roofline and CPU baseline, one summary per BASELINE config and one-number summaries of the
    stream curve, the end-to-end path and the sharded stream.  len(json.dumps(...)) <= LINE_MAX
    (tests/test_bench_line.py); everything else is in the sidecar named by `detail`."""
    keep = ("metric", "value", "unit", "units", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
            "vs_baseline", "dtype", "data")
    line = {k: full.get(k) for k in keep}
    cfg = full.get("config") or {}
    line["config"] = {"workload": cfg.get("workload_key"), "blocks_per_gpu_per_step": cfg.get("blocks_per_gpu_per_step"),
                      "streams_per_gpu": cfg.get("streams_per_gpu"), "channels_bits_rate": cfg.get("channels_bits_rate"),
                      "compression_ratio": cfg.get("compression_ratio"), "parallelism": cfg.get("parallelism")}
    line["roofline"] = _compact_roofline(full.get("roofline"))
    line["kernel_ms_per_step"] = full.get("kernel_ms_per_step")
    line["output_ok"] = full.get("output_ok")
    line["cpu_baseline"] = _compact_cpu(full.get("cpu_baseline"))
    cs = {}
    for c in full.get("configs") or []:
        if not c:
            continue
        r = c.get("roofline") or {}
        cb = c.get("cpu_baseline") or {}
        cs[c["config"]] = {"value": c.get("value"), "ms_per_step": c.get("ms_per_step"),
                           "kernel_ms": c.get("kernel_ms_per_step"), "frac": r.get("frac"),
                           "frac_vs_6p29": r.get("frac_vs_6p29"),
                           "step_issue_frac": r.get("step_issue_frac"),
                           "weighted_issue_frac": r.get("weighted_issue_frac"),
                           "traffic_ratio": (r.get("kernels") or {}).get(_dom_name(r), {}).get("traffic_ratio"),
                           "x_realtime": (c.get("units") or {}).get("x_realtime"),
                           "output_ok": c.get("output_ok"), "cpu": cb.get("value"),
                           "cpu_single_core": (cb.get("single_core") or {}).get("value"),
                           "cpu_health": cb.get("health")}
    line["configs"] = cs or None
    sc = full.get("stream_curve")
    if sc:
        line["stream_curve"] = {str(p["streams"]): [p.get("value"), p.get("md5_engine"),
                                                    (p.get("other") or {}).get("value")] for p in sc}
        line["stream_curve_ok"] = all(p.get("md5_ok") and (p.get("other") or {}).get("md5_ok", True) for p in sc)
    e = full.get("end_to_end")
    if e:
        top = max(e.get("curve") or [{}], key=lambda c: c.get("files", 0))
        line["end_to_end"] = {"value": e.get("value"), "files": e.get("files"), "mode": e.get("mode"),
                              "ranks": e.get("ranks", 1),
                              "batch_frac_of_md5_bound": {str(c["files"]): c["batch"]["frac_of_md5_bound"]
                                                          for c in e.get("curve") or []},
                              "batch_h2d_d2h_gbs": e.get("batch_gbs"),
                              "largest_batch": (top.get("batch") or {}).get("value"),
                              "many_files": ({k: (e.get("many_files") or {}).get(k) for k in
                                              ("files", "minutes_per_file", "value", "frac_of_md5_bound", "h2d_gbs")}
                                             if e.get("many_files") else None),
                              "vs_cpu_single_socket_estimate": e.get("vs_cpu_single_socket_estimate"),
                              "output_ok": e.get("output_ok")}
        if e.get("error"):
            line["end_to_end"]["error"] = e["error"]
    s = full.get("sharded_stream")
    if s:
        line["sharded_stream"] = {"value": s.get("value"), "ranks": s.get("ranks"), "ms_per_window": s.get("ms_per_window"),
                                  "output_ok": s.get("output_ok")}
        if s.get("error"):
            line["sharded_stream"]["error"] = s["error"]
    line["detail"] = detail_path
    # last resort, never expected: drop the largest optional blocks until the line fits
    for k in ("stream_curve", "end_to_end", "kernel_ms_per_step", "configs"):
        if len(json.dumps(line)) <= LINE_MAX:
            break
        line.pop(k, None)
    return line


def write_detail(full: dict) -> str | None:
    """The full record as a sidecar JSON file (FLACGPU_BENCH_DETAIL, default gpurun_out/bench_detail.json
    under the repo root); returns its path relative to the repo root, None if it cannot be written."""
    path = os.environ.get("FLACGPU_BENCH_DETAIL") or os.path.join(ROOT, "gpurun_out", "bench_detail.json")
    try:
        os.makedirs(os.path.dirname(path), exist_ok=True)
        with open(path, "w") as f:
            json.dump(full, f, indent=1)
        return os.path.relpath(path, ROOT)
    except OSError:
        return None


def visible_gpus() -> int:
    """GPUs this process could use, counted in a child process: the launcher itself never loads
    torch or touches the GPU (FLACGPU_BENCH_FAKE_GPUS overrides the count: CPU tests)."""
    fake = os.environ.get("FLACGPU_BENCH_FAKE_GPUS")
    if fake is not None:
        return int(fake)
    r = subprocess.run([sys.executable, "-c", "import torch; print(torch.cuda.device_count())"],
                       capture_output=True, text=True, timeout=600)
    try:
        return int(r.stdout.strip().splitlines()[-1])
    except (ValueError, IndexError):
        return 0


def launch(args) -> int:
    """`bench.py --gpus N` with no WORLD_SIZE in the environment: one fresh child process per rank
    (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT set, the same argv), the torchrun
    convention without torchrun.  The parent makes no GPU call before, during or after, never execs,
    and prints nothing on stdout: rank 0's JSON line is the run's only stdout line.  Fewer visible
    GPUs than N is an error (one rank per GPU).  Returns the exit code (the first failing rank's)."""
    import socket

    n = args.gpus
    have = visible_gpus()
    if have < n:
        print(f"bench.py --gpus {n}: {have} GPU(s) visible; one rank per GPU needs {n}", file=sys.stderr)
        return 2
    sk = socket.socket()
    sk.bind(("127.0.0.1", 0))
    port = sk.getsockname()[1]
    sk.close()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__), *sys.argv[1:]], env=env))
    rc, live = 0, set(range(n))
    while live:
        for i in sorted(live):
            c = procs[i].poll()
            if c is None:
                continue
            live.discard(i)
            if c != 0 and rc == 0:
                rc = c if c > 0 else 128 - c  # killed by signal -c
                for j in live:  # a rank failed: the others would wait for it forever
                    procs[j].terminate()
        time.sleep(0.1)
    return rc


def stub_worker(args):
    """FLACGPU_BENCH_STUB=1 (CPU tests of the launcher): the rank plumbing of main() -- gloo process
    group from the launcher's environment, barrier, max-over-ranks, rank 0's one JSON line -- with
    no GPU and no encode."""
    sys.stdout.flush()
    json_fd = os.dup(1)
    os.dup2(2, 1)  # as in main(): gloo / RCCL banners go to stderr
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if os.environ.get("FLACGPU_BENCH_STUB_FAIL") == str(rank):
        raise SystemExit(7)  # a rank that dies before the rendezvous (launcher test)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    ids = [None] * world
    dist.all_gather_object(ids, {"rank": rank, "local_rank": int(os.environ.get("LOCAL_RANK", "-1")),
                                 "pid": os.getpid(), "ppid": os.getppid()})
    dist.barrier()
    t = torch.tensor([float(rank)], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    if rank == 0:
        os.write(json_fd, (json.dumps({"metric": METRIC, "stub": True, "n_gpus": world, "ranks": ids,
                                       "max_over_ranks": t.item(), "steps": args.steps,
                                       "warmup": args.warmup}) + "\n").encode())
    dist.destroy_process_group()


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        raise SystemExit(launch(args))
    if os.environ.get("FLACGPU_BENCH_STUB") == "1":
        return stub_worker(args)
    # the contract is ONE JSON line on stdout: libraries that print banners there (RCCL prints
    # its version at communicator init, on every rank) are moved to stderr at the fd level
    sys.stdout.flush()
    json_fd = os.dup(1)
    os.dup2(2, 1)
    # the host MD5 pool (end_to_end) sizes itself from FLACGPU_MD5_THREADS, else the cgroup quota /
    # affinity mask: on the GPU box that mask is the whole machine, the share is OMP_NUM_THREADS
    if "FLACGPU_MD5_THREADS" not in os.environ and os.environ.get("OMP_NUM_THREADS", "1") not in ("", "1"):
        os.environ["FLACGPU_MD5_THREADS"] = os.environ["OMP_NUM_THREADS"]
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # the CPU baseline first (N = 1, or --cpu-only): before torch is imported and before any HIP call,
    # host MD5 pool or pinned buffer exists, so its sample has the host to itself
    headline = args.config or "c2"
    other_cfgs = [c for c in (args.configs or "").split(",") if c] if not args.config else []
    cpu_pre = {}
    if args.cpu_only or (world == 1 and not args.no_cpu):
        t0 = time.perf_counter()
        cpu_pre = cpu_legs(args, [headline] + other_cfgs)
        print(f"bench.py: CPU legs {time.perf_counter() - t0:.1f}s", file=sys.stderr)
        if args.cpu_only:
            os.write(json_fd, (json.dumps({"cpu_only": True, "legs": cpu_pre}) + "\n").encode())
            return
    import numpy as np
    import torch

    if world > 1 and args.gpus not in (1, world):
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}: running {world} ranks", file=sys.stderr)
    dist = None
    if world > 1:
        import torch.distributed as dist_mod

        dist = dist_mod
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(0)
    dev = torch.device("cuda", torch.cuda.current_device())

    import flacgpu

    if args.frames % args.streams:
        raise SystemExit("--frames must be a multiple of --streams")
    buf = build_input(args, rank)
    fb = args.channels * (args.bits // 8)
    enc = flacgpu.Encoder(args.channels, args.bits, args.rate, device=torch.cuda.current_device(),
                          max_frames=args.frames, lpc_order=args.lpc)
    d_pcm = torch.from_numpy(buf).to(dev)
    F = args.frames // args.streams
    w = Workload(enc, d_pcm, args.streams, F, fb, dev, md5=not args.no_md5)
    elapsed = run_timed(w, args.steps, args.warmup, dist)
    if dist:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    samples_per_rank = args.frames * 4096
    value = samples_per_rank * world * args.steps / elapsed / 1e6
    ms_per_step = elapsed / args.steps * 1e3

    kt = kernel_times(enc)
    fbytes = w.d_fb.cpu().numpy().astype(np.int64)
    total_bytes = int(w.d_tot[0].item())
    pcm_bytes = args.frames * 4096 * fb
    key = workload_key(args)
    roof = roofline_of(args, kt, args.steps, pcm_bytes, int(fbytes.sum()), ms_per_step, key)

    ok, vinfo = verify(args, w, buf, fb, args.verify_streams, dev) if rank == 0 else (True, {})
    w.close()

    sharded = None
    if not args.no_sharded:
        del d_pcm
        torch.cuda.empty_cache()
        try:
            sharded = sharded_stream(args, rank, world, dist, dev)
        except Exception as e:
            # the C ABI agrees on errors across ranks (every rank raises alike), so the headline
            # measured above still reaches the line; the failure is reported in it
            print(f"bench.py: sharded stream failed: {e!r}", file=sys.stderr)
            sharded = {"error": f"{type(e).__name__}: {e}"[:300], "output_ok": False, "ranks": world}
        d_pcm = torch.from_numpy(buf).to(dev) if (rank == 0 and world == 1 and not args.no_curve
                                                  and not args.no_md5) else None

    curve = e2e = cpu = md5_rates = None
    if world > 1 and not args.no_e2e and headline == "c2":
        del d_pcm
        d_pcm = None
        torch.cuda.empty_cache()
        try:
            e2e = end_to_end_node(args, rank, world, dist, dev)
        except Exception as e:  # as the sharded leg: the headline still reaches the line
            print(f"bench.py: end-to-end (node) failed: {e!r}", file=sys.stderr)
            e2e = {"error": f"{type(e).__name__}: {e}"[:300], "output_ok": False, "ranks": world}
    if rank == 0 and world == 1:
        if not args.no_curve and not args.no_md5:
            curve = stream_curve(args, enc, d_pcm, buf, fb, dev)
            md5_rates = flacgpu.md5_rates().as_dict()
        if not args.no_e2e and (args.config or "c2") == "c2":
            del d_pcm
            torch.cuda.empty_cache()
            e2e = end_to_end(args)
        cpu = cpu_pre.get(headline)
    d_pcm = None
    enc.close()
    torch.cuda.empty_cache()

    # the other BASELINE configs, each its own timed line (every rank: streams sharded as above)
    configs = None
    if args.configs and not args.config:
        del buf
        configs = [config_line(args, c, dist, rank, world, dev, cpu_pre.get(c)) for c in other_cfgs]

    if e2e and cpu:
        e2e["vs_cpu_measured_P_cores"] = round(e2e["value"] / cpu["value"], 2)
        if cpu.get("single_socket_estimate"):
            e2e["vs_cpu_single_socket_estimate"] = round(e2e["value"] / cpu["single_socket_estimate"], 2)

    if rank == 0:
        line = {
            "metric": METRIC,
            "value": round(value, 2),
            "unit": "MSamples/s",
            "units": rate_units(value, args.channels, args.rate),
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "int32",
            "data": "synthetic",
            "config": {
                "workload": workload_text(args, F),
                "workload_key": key,
                "blocks_per_gpu_per_step": args.frames,
                "streams_per_gpu": args.streams,
                "channels_bits_rate": f"{args.channels}ch/{args.bits}-bit/{args.rate}Hz",
                "samples_per_gpu_per_step": samples_per_rank,
                "compression_ratio": round(total_bytes / pcm_bytes, 4),
                "parallelism": f"streams sharded over {world} GPU(s), no collective on the data path",
                "launcher": "torchrun / bench.py --gpus N (one fresh process per rank)" if world > 1 else "one process",
            },
            "roofline": roof,
            "kernel_ms_per_step": {k: round(v[1] / args.steps, 4) for k, v in kt.items() if v[0]},
            "output_ok": ok,
            "verified": vinfo,
            "configs": configs,
            "stream_curve": curve,
            "md5_rates": md5_rates,
            "sharded_stream": sharded,
            "end_to_end": e2e,
            "cpu_baseline": cpu,
        }
        detail = write_detail(line)
        print("bench.py full record: " + json.dumps(line), file=sys.stderr)
        sys.stdout.flush()
        os.write(json_fd, (json.dumps(compact_line(line, detail)) + "\n").encode())
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
