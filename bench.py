#!/usr/bin/env python3
"""Benchmark: FLAC block encode on MI355X (BASELINE.json metric).

metric : MSamples/s encoded (whole node), 44.1kHz/16-bit stereo, blocksize 4096
unit   : 1 sample = one interchannel sample (STREAMINFO unit, metadata.zig:24)

A "step" is one pass of the hot path over one batch: every 4096-sample block
of S independent streams (8192 streams x 8 blocks = 65536 blocks per GPU by
default, BASELINE config 2)
goes through the gfx950 kernels of libflacgpu.so -- analysis (mid/side, wasted
bits, fixed-order analysis, Rice search, subframe choice, exact frame sizes),
frame-size scan, pack (bit packing, CRC-8/16, frames written at their final
offsets: one contiguous bitstream per stream) -- and the MD5 of every stream's
raw PCM is computed on the GPU concurrently.  Inputs are resident in
HBM before the timed region; outputs stay in HBM.  The MD5 is sequential
within a stream (one lane per stream), so its rate grows with the number of
streams in flight: 8192 streams keep it under the encode.

One process per GPU (torchrun for N > 1).  Streams are independent files, so
ranks shard streams with no data-path collective (weak scaling); a barrier and
a max-over-ranks reduction bracket the timed region.

The JSON line also carries:
  roofline     -- the dominant kernel (analysis or pack, whichever takes
                  longer): its algorithmic bytes per launch (analysis: PCM
                  read; pack: PCM read + frame bytes written) / its mean launch
                  time, measured with HIP events on the launch stream during
                  the timed steps, against 8 TB/s; `traffic` from the
                  committed rocprofv3 PMC profile (profiles/), else null;
  cpu_baseline -- the CPU restatement (oracle/, "port") timed on host
                  threads over a bounded sample of the same workload.
"""
from __future__ import annotations

import argparse
import ctypes
import glob
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "zig-flac_amd"))

METRIC = "MSamples/s encoded (whole node), 44.1kHz/16-bit stereo, blocksize 4096"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
# BASELINE.json configs (channels, bits, rate, LPC max order); c2 is the headline metric's
PRESETS = {"c2": (2, 16, 44100, 0), "c3": (2, 24, 96000, 8), "c4": (8, 24, 96000, 0), "c5": (2, 32, 192000, 12)}


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--frames", type=int, default=65536, help="4096-sample blocks per GPU")
    p.add_argument("--streams", type=int, default=8192, help="independent streams (files) per GPU")
    p.add_argument("--channels", type=int, default=2)
    p.add_argument("--bits", type=int, default=16)
    p.add_argument("--rate", type=int, default=44100)
    p.add_argument("--lpc", type=int, default=0, help="LPC max order (0 = fixed prediction, the reference)")
    p.add_argument("--config", choices=sorted(PRESETS), default=None,
                   help="BASELINE.json config preset (overrides --channels/--bits/--rate/--lpc); default c2")
    p.add_argument("--no-md5", action="store_true", help="skip the per-stream GPU MD5 (diagnostics only)")
    p.add_argument("--md5-join", action="store_true",
                   help="join each step's MD5 back into the encode stream (no overlap of consecutive steps)")
    p.add_argument("--stream-pad", type=int, default=0,
                   help="bytes of gap between consecutive streams in HBM (multiple of 4; layout diagnostics)")
    p.add_argument("--cpu-frames", type=int, default=32768, help="blocks in the CPU-baseline sample")
    p.add_argument("--cpu-threads", type=int, default=16)
    p.add_argument("--no-cpu", action="store_true")
    p.add_argument("--verify", action="store_true", help="decode + check a sample of streams after timing")
    a = p.parse_args()
    if a.config:
        a.channels, a.bits, a.rate, a.lpc = PRESETS[a.config]
    return a


def make_pool(n, ch, bits, rate):
    import synth

    return synth.synth_samples(n, ch, bits, rate, stream=0)


def build_input(args, rank):
    """Synthetic PCM for S streams: windows of a seeded pool (SURVEY.md 8(d) signal)."""
    import numpy as np
    import synth

    S, F = args.streams, args.frames // args.streams
    ch, bits = args.channels, args.bits
    n_per = F * 4096
    pool_n = max(8 * 4096 * 64, n_per + 4096 * 64)
    pool = make_pool(pool_n, ch, bits, args.rate)
    pcm_pool = np.frombuffer(synth.to_pcm_bytes(pool, bits), dtype=np.uint8)
    fb = ch * (bits // 8)
    rng = np.random.Generator(np.random.PCG64(20260821 + 7919 * rank))
    starts = rng.integers(0, (pool_n - n_per) // 4096 + 1, size=S) * 4096
    stream_bytes = n_per * fb
    pitch = stream_bytes + args.stream_pad
    buf = np.zeros(S * pitch, dtype=np.uint8)
    for s in range(S):
        a = int(starts[s]) * fb
        buf[s * pitch:s * pitch + stream_bytes] = pcm_pool[a:a + stream_bytes]
    offsets = [s * pitch for s in range(S)]
    samples = [n_per] * S
    return buf, offsets, samples


def cpu_baseline(buf, offsets, samples, args):
    """Oracle (scalar C restatement) on host threads over a bounded sample."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_ref

    L = oracle_ref.lib()
    ch, bits = args.channels, args.bits
    fb = ch * (bits // 8)
    # each thread encodes whole streams (thread t: streams t, t+T, ...) until it has its share of blocks
    per_thread = max(1, args.cpu_frames // args.cpu_threads)
    jobs = []
    for t in range(args.cpu_threads):
        mine, blocks, s = [], 0, t
        while blocks < per_thread and s < len(offsets):
            nb = (samples[s] + 4095) // 4096
            mine.append(bytes(buf[offsets[s]:offsets[s] + samples[s] * fb]))
            blocks += nb
            s += args.cpu_threads
        jobs.append(mine)
    cfg = oracle_ref.config(ch, bits, args.rate, lpc=args.lpc)
    res = [0] * len(jobs)

    def run(i):
        done = 0
        for pcm in jobs[i]:
            n = len(pcm) // fb
            nf = (n + 4095) // 4096
            cap = nf * L.oracle_max_frame_bytes(4096, bits, ch) + 64
            out = ctypes.create_string_buffer(cap)
            sizes = (ctypes.c_uint32 * nf)()
            md5 = ctypes.create_string_buffer(16)
            r = L.oracle_encode_stream(ctypes.byref(cfg), pcm, bits // 8, ctypes.c_uint64(n), ctypes.c_uint64(0),
                                       out, ctypes.c_size_t(cap), sizes, md5)
            done += n if r > 0 else 0
        res[i] = done

    th = [threading.Thread(target=run, args=(i,)) for i in range(len(jobs))]
    t0 = time.perf_counter()
    for t in th:
        t.start()
    for t in th:
        t.join()
    dt = time.perf_counter() - t0
    tot = sum(res)
    return {
        "value": round(tot / dt / 1e6, 3),
        "unit": "MSamples/s",
        "cores": args.cpu_threads,
        "kind": "port",
        "sample": f"{tot} samples ({sum(len(j) for j in jobs)} whole streams, {tot // 4096} blocks, incl. MD5) on "
                  f"{args.cpu_threads} host threads (one oracle encode per stream), {dt:.2f}s wall",
    }


def read_traffic(kernel, frames_per_launch):
    """HBM bytes per launch of `kernel` from the committed rocprofv3 PMC summary (profiles/*pmc*.json)."""
    cands = sorted(glob.glob(os.path.join(ROOT, "profiles", "*pmc*.json")))
    if not cands:
        return None
    try:
        d = json.load(open(cands[-1]))
        if d.get("frames_per_launch") != frames_per_launch:
            return None
        return d.get("hbm_bytes_per_launch", {}).get(kernel)
    except Exception:
        return None


def read_issue(kernel, frames_per_launch, avg_s):
    """VALU issue load of `kernel` from the committed PMC summary: wave-instructions per launch
    against 1024 SIMDs x 0.5 wave64 VALU instructions/clock (SIMD-32, 2 passes; MI355X_MICROARCH.md)
    at 2.4 GHz.  A lower bound on VALU busy (64-bit and transcendental ops take more passes)."""
    cands = sorted(glob.glob(os.path.join(ROOT, "profiles", "*pmc*.json")))
    if not cands or avg_s <= 0:
        return None
    try:
        d = json.load(open(cands[-1]))
        if d.get("frames_per_launch") != frames_per_launch:
            return None
        c = d.get("counters_per_dispatch", {}).get(kernel, {})
        valu, salu = c.get("SQ_INSTS_VALU"), c.get("SQ_INSTS_SALU")
        if not valu:
            return None
        peak = 1024 * 0.5 * 2.4e9
        return {"valu_wave_instr_per_launch": valu, "salu_wave_instr_per_launch": salu,
                "peak_valu_wave_instr_per_s": peak, "valu_issue_frac": round(valu / avg_s / peak, 4),
                "source": os.path.basename(cands[-1])}
    except Exception:
        return None


def main():
    args = parse()
    import numpy as np
    import torch

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
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
    buf, offsets, samples = build_input(args, rank)
    enc = flacgpu.Encoder(args.channels, args.bits, args.rate, device=torch.cuda.current_device(),
                          max_frames=args.frames, lpc_order=args.lpc)
    plan = enc.plan(offsets, samples)
    d_pcm = torch.from_numpy(buf).to(dev)
    out_cap = int(plan.out_bound)
    d_out = torch.empty(out_cap, dtype=torch.uint8, device=dev)
    d_fb = torch.empty(plan.n_frames, dtype=torch.int32, device=dev)
    d_off = torch.empty(plan.n_frames, dtype=torch.int64, device=dev)
    d_tot = torch.zeros(2, dtype=torch.int64, device=dev)
    d_md5 = torch.zeros(args.streams * 16, dtype=torch.uint8, device=dev)
    stream = torch.cuda.current_stream(dev)
    # The MD5 is per-stream sequential (latency-bound), the encode throughput-bound: step k's MD5
    # runs on its own HIP stream (two alternate) and overlaps step k+1's encode.  Every step's MD5
    # and frames are complete at the synchronize that closes the timed region.
    md5_streams = [torch.cuda.Stream(dev), torch.cuda.Stream(dev)]
    n_step = [0]

    def step():
        ms = None if args.md5_join else md5_streams[n_step[0] % 2].cuda_stream
        n_step[0] += 1
        enc.encode_plan_device(plan, d_pcm.data_ptr(), d_out.data_ptr(), out_cap, d_fb.data_ptr(),
                               d_off.data_ptr(), d_tot.data_ptr(), None if args.no_md5 else d_md5.data_ptr(),
                               stream.cuda_stream, md5_stream=ms)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    enc.reset_timing()
    enc.set_timing(True)
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    if dist:
        dist.barrier()
    enc.set_timing(False)
    elapsed = t1 - t0
    if dist:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    samples_per_rank = sum(samples)
    value = samples_per_rank * world * args.steps / elapsed / 1e6

    # roofline of the dominant kernel, from HIP events on its stream
    kt = {name: enc.kernel_time(k) for k, name in enumerate(flacgpu.KERNEL_NAMES)}
    fb = d_fb.cpu().numpy().astype(np.int64)
    total_bytes = int(d_tot[0].item())
    frame_in = 4096 * args.channels * (args.bits // 8)
    n_frames = int(plan.n_frames)
    per_launch = {name: (v[1] / v[0]) / 1e3 for name, v in kt.items() if v[0]}
    dom = "pack" if per_launch.get("pack", 0) > per_launch.get("analyze", 0) else "analyze"
    algo_bytes = n_frames * frame_in + (int(fb.sum()) if dom == "pack" else 0)
    n_launch = kt[dom][0]
    avg_s = per_launch.get(dom, 0.0)
    achieved = algo_bytes / avg_s / 1e9 if avg_s > 0 else 0.0
    traffic = read_traffic(dom, n_frames)
    path_s = sum(per_launch.get(k, 0.0) for k in ("analyze", "analyze_tail", "scan", "pack"))
    path_bytes = n_frames * frame_in + int(fb.sum())

    # validity checks on the last step's output
    ok = bool(total_bytes == int(fb.sum()) and total_bytes > 0)
    if args.verify and rank == 0:
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        import hashlib
        import oracle_ref

        out = d_out[:total_bytes].cpu().numpy().tobytes()
        offs = d_off.cpu().numpy()
        md5s = d_md5.cpu().numpy().reshape(-1, 16)
        for s in list(range(0, args.streams, max(1, args.streams // 8))):
            f0 = plan.first_frame[s]
            f1 = plan.first_frame[s + 1] if s + 1 < args.streams else plan.n_frames
            a = int(offs[f0])
            b = int(offs[f1]) if f1 < plan.n_frames else total_bytes
            pcm = bytes(buf[offsets[s]:offsets[s] + samples[s] * frame_in // 4096])
            dec, _ = oracle_ref.decode_frames(out[a:b], args.channels, args.bits, args.rate, samples[s])
            ok &= dec == pcm
            if not args.no_md5:
                ok &= md5s[s].tobytes() == hashlib.md5(pcm).digest()

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu:
        cpu = cpu_baseline(buf, offsets, samples, args)

    if rank == 0:
        line = {
            "metric": METRIC,
            "value": round(value, 2),
            "unit": "MSamples/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "int32",
            "data": "synthetic",
            "config": {
                "workload": f"{(args.config or 'c2').upper()}: {args.rate/1000:g}kHz {args.bits}-bit "
                            f"{args.channels}ch, blocksize 4096, "
                            f"{args.frames} blocks/GPU as {args.streams} streams x {args.frames // args.streams} "
                            f"blocks, " + (f"LPC orders 1..{args.lpc} + full subframe-type search"
                                           if args.lpc else "fixed prediction") +
                            f", per-stream GPU MD5" + (" (off)" if args.no_md5 else
                                                          (" joined per step" if args.md5_join else
                                                           " overlapping the next step's encode")),
                "blocks_per_gpu": args.frames,
                "streams_per_gpu": args.streams,
                "samples_per_gpu": samples_per_rank,
                "compression_ratio": round(total_bytes / (samples_per_rank * frame_in / 4096), 4),
                "parallelism": f"streams sharded over {world} GPU(s), no collective on the data path",
            },
            "roofline": {
                "bound": "hbm",
                "kernel": "k_analyze (4096-sample frames)" if dom == "analyze" else "k_pack",
                "achieved": round(achieved, 2),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 5),
                "traffic": traffic,
                "algorithmic_bytes_per_launch": algo_bytes,
                "avg_launch_ms": round(avg_s * 1e3, 4),
                "launches": n_launch,
                "encode_path_gbs": round(path_bytes / path_s / 1e9, 2) if path_s > 0 else None,
                "issue": read_issue(dom, n_frames, avg_s),
            },
            "kernel_ms_per_step": {k: round(v[1] / max(v[0], 1), 4) for k, v in kt.items() if v[0]},
            "output_ok": ok,
            "cpu_baseline": cpu,
        }
        print(json.dumps(line))
    plan.close()
    enc.close()
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
