#!/usr/bin/env python3
"""Copy / compute overlap from a rocprofv3 kernel + memory-copy trace (tools only).

Usage: tools/overlap.py <dir with *_kernel_trace.csv and *_memory_copy_trace.csv> [out.json]

The trace is cut into bursts at idle gaps > 20 ms (one end-to-end batch call is one burst); for
each burst of at least 50 ms: its wall time, the busy time (union of intervals) of H2D copies, D2H
copies and kernels, and the time during which each pair ran at once.  A schedule whose uploads,
kernels and downloads overlap has busy(H2D) + busy(kernels) + busy(D2H) well above the wall."""
import csv
import glob
import json
import os
import sys


def union(iv):
    out = []
    for a, b in sorted(iv):
        if out and a <= out[-1][1]:
            out[-1][1] = max(out[-1][1], b)
        else:
            out.append([a, b])
    return out


def length(u):
    return sum(b - a for a, b in u)


def inter(u, v):
    i = j = 0
    t = 0
    while i < len(u) and j < len(v):
        a, b = max(u[i][0], v[j][0]), min(u[i][1], v[j][1])
        if a < b:
            t += b - a
        if u[i][1] < v[j][1]:
            i += 1
        else:
            j += 1
    return t


def load(d):
    ev = {"kernel": [], "h2d": [], "d2h": [], "d2d": []}
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            ev["kernel"].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    for f in glob.glob(os.path.join(d, "**", "*memory_copy_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            kind = " ".join(str(v) for v in r.values()).upper()
            k = ("h2d" if "HOST_TO_DEVICE" in kind else "d2h" if "DEVICE_TO_HOST" in kind
                 else "d2d" if "DEVICE_TO_DEVICE" in kind else None)
            if k:
                ev[k].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    return ev


def bursts(ev, gap=20_000_000, min_len=50_000_000):
    allv = union([x for v in ev.values() for x in v])
    out = []
    for a, b in allv:
        if out and a - out[-1][1] <= gap:
            out[-1][1] = max(out[-1][1], b)
        else:
            out.append([a, b])
    return [(a, b) for a, b in out if b - a >= min_len]


def main():
    d = sys.argv[1]
    ev = load(d)
    res = []
    for a, b in bursts(ev):
        u = {k: union([(max(s, a), min(e, b)) for s, e in v if e > a and s < b]) for k, v in ev.items()}
        wall = b - a
        ms = lambda t: round(t / 1e6, 3)  # noqa: E731
        res.append({"wall_ms": ms(wall),
                    "busy_ms": {k: ms(length(x)) for k, x in u.items() if x},
                    "overlap_ms": {"kernel&h2d": ms(inter(u["kernel"], u["h2d"])),
                                   "kernel&d2h": ms(inter(u["kernel"], u["d2h"])),
                                   "h2d&d2h": ms(inter(u["h2d"], u["d2h"]))},
                    "sum_busy_over_wall": round((length(u["kernel"]) + length(u["h2d"]) + length(u["d2h"])) / wall, 3),
                    "launches": {k: sum(1 for s, e in v if e > a and s < b) for k, v in ev.items()}})
    out = {"trace": os.path.basename(os.path.normpath(d)), "bursts": res}
    txt = json.dumps(out, indent=1)
    if len(sys.argv) > 2:
        open(sys.argv[2], "w").write(txt + "\n")
    print(txt)


if __name__ == "__main__":
    main()
