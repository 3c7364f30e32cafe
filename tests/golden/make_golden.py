#!/usr/bin/env python3
"""Generate the golden vectors in tests/golden/ (committed with this script).

Each case is a deterministic synthetic input (zig-flac_amd/synth.py: numpy PCG64,
seed 20260821 + stream) encoded by the CPU restatement (oracle/) and verified by
the independent decoder before it is written.  The reference itself (Zig 0.16)
cannot be built here or on the GPU box, so these vectors pin the restatement's
bytes across changes and give the GPU path fixed targets; they are not
reference-produced.

Files: <name>.flac (frames only, or a whole file for kind == "file"),
manifest.json (inputs, sizes, MD5, sha256 of input PCM and output).
Run: python tests/golden/make_golden.py
"""
import hashlib
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "zig-flac_amd"))

# name, kind, channels, bits, rate, n_samples, stream seed, first frame, block
CASES = [
    ("c1_44k16_stereo", "frames", 2, 16, 44100, 3 * 4096 + 1000, 0, 0, 4096),
    ("c1_44k16_stereo_file", "file", 2, 16, 44100, 2 * 4096 + 333, 1, 0, 4096),
    ("mono_44k16", "frames", 1, 16, 44100, 2 * 4096 + 5, 2, 0, 4096),
    ("c3_96k24_stereo", "frames", 2, 24, 96000, 2 * 4096 + 576, 3, 0, 4096),
    ("c5_192k32_stereo", "frames", 2, 32, 192000, 2 * 4096 + 255, 4, 0, 4096),
    ("c4_96k24_8ch", "frames", 8, 24, 96000, 4096 + 192, 5, 0, 4096),
    ("3ch_8bit", "frames", 3, 8, 22050, 4096 + 24, 6, 0, 4096),
    ("utf8_widths", "frames", 2, 16, 48000, 4 * 4096, 7, 2046, 4096),
    ("block1152", "frames", 2, 16, 44100, 5 * 1152 + 4, 8, 0, 1152),
    ("specials", "frames", 2, 16, 44100, 5 * 4096, 9, 0, 4096),
]


def make_pcm(name, ch, bits, rate, n, seed):
    import numpy as np
    import synth

    x = synth.synth_samples(n, ch, bits, rate, stream=seed)
    if name == "specials":  # the special block kinds of SURVEY.md 8(d), one per frame
        lo, hi = -(1 << (bits - 1)), (1 << (bits - 1)) - 1
        rng = np.random.default_rng(seed)
        x[0:4096] = 0
        x[4096:8192] = 1234
        x[8192:12288] = rng.integers(lo, hi + 1, size=(4096, ch))
        x[12288:16384] = (x[12288:16384] >> 3) << 3
        x[16384:20480] = np.where(np.arange(4096) % 2 == 0, hi, lo)[:, None]
    return synth.to_pcm_bytes(x, bits)


def main():
    import oracle_ref

    manifest = []
    for name, kind, ch, bits, rate, n, seed, first, block in CASES:
        pcm = make_pcm(name, ch, bits, rate, n, seed)
        if kind == "file":
            out = oracle_ref.encode_file(pcm, ch, bits, rate, block)
            sizes, md5 = None, hashlib.md5(pcm).hexdigest()
            dec, _ = oracle_ref.decode_frames(out[73:], ch, bits, rate, n)
        else:
            out, sizes, md5b = oracle_ref.encode_stream(pcm, ch, bits, rate, block, first_frame=first)
            md5 = md5b.hex()
            dec, _ = oracle_ref.decode_frames(out, ch, bits, rate, n, first_number=first)
        assert dec == pcm, name
        assert md5 == hashlib.md5(pcm).hexdigest(), name
        open(os.path.join(HERE, name + ".flac"), "wb").write(out)
        manifest.append({"name": name, "kind": kind, "channels": ch, "bits": bits, "rate": rate, "n_samples": n,
                         "stream_seed": seed, "first_frame": first, "block": block,
                         "pcm_sha256": hashlib.sha256(pcm).hexdigest(),
                         "out_sha256": hashlib.sha256(out).hexdigest(), "out_bytes": len(out),
                         "frame_bytes": sizes, "md5": md5})
        print(f"{name}: {len(pcm)} B PCM -> {len(out)} B")
    json.dump({"generator": "tests/golden/make_golden.py", "cases": manifest},
              open(os.path.join(HERE, "manifest.json"), "w"), indent=1)


if __name__ == "__main__":
    main()
