"""PCIe-inclusive rate of the host-buffer boundary (flacgpu_encode_frames), for DESIGN.md §5.

Host PCM (interleaved LE 16-bit stereo, 44.1 kHz, blocksize 4096) in pageable memory ->
frames in pageable memory, through the C ABI exactly as the reference's Zig host would call
it (one call per buffer; the library chunks by max_frames).  Not the bench `value` (that is
HBM-resident input).  Usage: python tools/host_rate.py [frames] [reps]
"""
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "zig-flac_amd"))
import flacgpu  # noqa: E402


def main():
    frames = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    n = frames * 4096
    rng = np.random.default_rng(20260821)
    t = np.arange(n, dtype=np.float64)
    sig = 6000 * np.sin(t * 0.031) + 2500 * np.sin(t * 0.0071) + rng.normal(0, 300, n)
    pcm = np.empty((n, 2), dtype=np.int16)
    pcm[:, 0] = np.clip(sig, -32768, 32767).astype(np.int16)
    pcm[:, 1] = np.clip(0.7 * sig + rng.normal(0, 200, n), -32768, 32767).astype(np.int16)
    pcm = np.ascontiguousarray(pcm)
    res = {"frames": frames, "samples": n, "pcm_bytes": pcm.nbytes}
    for mf in (8192, 32768):
        with flacgpu.Encoder(2, 16, 44100, device=0, max_frames=mf) as enc:
            cap = frames * enc.frame_bound() + 64
            out = np.empty(cap, dtype=np.uint8)
            sizes = np.empty(frames, dtype=np.uint32)
            out_len = ctypes.c_size_t(0)

            def run():
                rc = enc.lib.flacgpu_encode_frames(enc.ctx, pcm.ctypes.data_as(ctypes.c_void_p), 2, n, 0,
                                                   out.ctypes.data_as(ctypes.c_void_p), cap, ctypes.byref(out_len),
                                                   sizes.ctypes.data_as(ctypes.c_void_p))
                assert rc == 0, rc

            run()
            best = 1e9
            for _ in range(reps):
                t0 = time.perf_counter()
                run()
                best = min(best, time.perf_counter() - t0)
            res[f"max_frames_{mf}"] = {"seconds": round(best, 5), "MSamples_per_s": round(n / best / 1e6, 1),
                                       "out_bytes": int(out_len.value),
                                       "pcm_GB_per_s": round(pcm.nbytes / best / 1e9, 2)}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
