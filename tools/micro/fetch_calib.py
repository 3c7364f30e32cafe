#!/usr/bin/env python3
"""Join tools/fetch_calib.sh's outputs: FETCH_SIZE (KiB, per dispatch, averaged) x 1024 / the bytes
each k_fetch<M> reads (printed by the micro), per access pattern.  The guide's 16-B case reads 0.5
(MI355X_MICROARCH.md, HBM section); the other rows calibrate the 4-B LDS-DMA staging and the c4
channel-half split that the analysis and pack kernels use."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def main():
    d, tag = sys.argv[1], sys.argv[2]
    runs = [json.loads(x) for x in open(os.path.join(d, "run.jsonl")) if x.strip()]
    stats = {}
    for f in glob.glob(os.path.join(d, "kt", "**", "*kernel_stats.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            stats[r["Name"]] = float(r["AverageNs"])
    fetch = defaultdict(list)
    for f in glob.glob(os.path.join(d, "pmc1", "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == "FETCH_SIZE":
                fetch[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    rows = []
    for r in runs:
        key = next((k for k in fetch if r["kernel"] + "(" in k), None)
        fs = sum(fetch[key]) / len(fetch[key]) * 1024 if key else None
        ns = next((v for k, v in stats.items() if r["kernel"] + "(" in k), None)
        rows.append(dict(r, fetch_bytes=fs, fetch_over_bytes=round(fs / r["bytes"], 4) if fs else None,
                         trace_avg_ms=round(ns / 1e6, 4) if ns else None))
    out = {"tag": tag, "note": "fetch_over_bytes = FETCH_SIZE KiB x 1024 / bytes the kernel reads (no x2 applied)",
           "rows": rows}
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for base in (os.path.join(root, "profiles"), os.path.join(root, "gpurun_out", "profiles")):
        os.makedirs(base, exist_ok=True)
        json.dump(out, open(os.path.join(base, f"{tag}_fetch_calib.json"), "w"), indent=1)
    for r in rows:
        print(f"{r['name']:6s} bytes={r['bytes']:>12d} fetch/bytes={r['fetch_over_bytes']} "
              f"best={r['best_ms']}ms trace={r['trace_avg_ms']}ms {r['gbs_best']} GB/s")


if __name__ == "__main__":
    main()
