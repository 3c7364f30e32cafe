#!/usr/bin/env python3
"""What the build-defined LPC buys, and what its single-order choice costs.

Compressed bytes of the bench's synthetic signal mix (synth.py, special blocks included) for the
LPC configs, through the CPU restatement (oracle/): fixed prediction only (the reference's
encoder), the LPC contract the GPU implements (one order, picked by the Levinson-Durbin error;
oracle/flac_oracle.c:447-475) and, as an analysis mode outside the contract, an exhaustive search
that runs the Rice search for every order 1..Q and keeps the smallest (oracle_set_lpc_exhaustive,
libFLAC's -e).  Every stream is decoded back to the PCM (lossless).  Prints one JSON line."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "zig-flac_amd")]
import oracle_ref  # noqa: E402
import synth  # noqa: E402

CONFIGS = {"c3": (2, 24, 96000, 8), "c5": (2, 32, 192000, 12), "c2_lpc12": (2, 16, 44100, 12)}


def main(frames=192):
    L = oracle_ref.lib()
    out = {"frames_per_config": frames, "signal": "synth.synth_pcm (bench mix, special blocks every 64th)"}
    for name, (ch, bits, rate, q) in CONFIGS.items():
        n = frames * 4096
        pcm = synth.synth_pcm(n, ch, bits, rate, stream=5)
        row = {"pcm_bytes": len(pcm), "lpc_order_max": q}
        for mode, lpc, exh in (("fixed", 0, 0), ("lpc_contract", q, 0), ("lpc_exhaustive", q, 1)):
            L.oracle_set_lpc_exhaustive(exh)
            try:
                fr, _, _ = oracle_ref.encode_stream(pcm, ch, bits, rate, lpc=lpc)
            finally:
                L.oracle_set_lpc_exhaustive(0)
            dec, _ = oracle_ref.decode_frames(fr, ch, bits, rate, n)
            assert dec == pcm, (name, mode)
            row[mode] = {"bytes": len(fr), "ratio": round(len(fr) / len(pcm), 5)}
        f, c, e = (row[m]["bytes"] for m in ("fixed", "lpc_contract", "lpc_exhaustive"))
        row["lpc_saves_vs_fixed"] = round(1 - c / f, 5)
        row["exhaustive_saves_vs_contract"] = round(1 - e / c, 5)
        out[name] = row
    print(json.dumps(out))


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 192)
