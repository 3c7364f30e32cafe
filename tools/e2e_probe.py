#!/usr/bin/env python3
"""The end-to-end leg of bench.py alone (host PCM -> .flac in host memory), for A/B runs of its
knobs on the GPU box (FLACGPU_MD5_THREADS, FLACGPU_FILE_SHARED, ...): prints one JSON line with
every curve point.  Usage: tools/e2e_probe.py [--e2e-files 32,64] [--e2e-many 256] [bench.py args]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def main():
    sys.argv = [sys.argv[0]] + sys.argv[1:]
    args = bench.parse()
    if "FLACGPU_MD5_THREADS" not in os.environ and os.environ.get("OMP_NUM_THREADS", "1") not in ("", "1"):
        os.environ["FLACGPU_MD5_THREADS"] = os.environ["OMP_NUM_THREADS"]
    import torch

    torch.cuda.set_device(0)
    e = bench.end_to_end(args)
    pts = [{"files": c["files"], "per_file": c["value"], "batch": c["batch"]["value"],
            "md5_frac_batch": c["batch"]["frac_of_md5_bound"], "h2d": c["batch"]["h2d_gbs"]} for c in e["curve"]]
    print(json.dumps({"threads": os.environ.get("FLACGPU_MD5_THREADS"), "value": e["value"], "points": pts,
                      "many": e.get("many_files"), "ok": e["output_ok"]}))


if __name__ == "__main__":
    main()
