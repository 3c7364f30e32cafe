#!/usr/bin/env python3
"""Summarise a tools/profile.sh run (rocprofv3 kernel trace + PMC passes) into
profiles/<tag>_summary.md and profiles/<tag>_pmc.json.

HBM bytes follow MI355X_MICROARCH.md (HBM / rocprofv3): FETCH_SIZE and WRITE_SIZE
are kilobytes (x1024); on gfx950 FETCH_SIZE counts half the bytes of wide
coalesced reads, so it is doubled (calibrated for the 4-B LDS-DMA staging of the wide configs too:
tools/micro/fetch_micro.hip, profiles/r4g_fetch_calib.json).  Counters are averaged per dispatch of each
kernel family.

Usage: tools/pmc_summary.py <prof_dir> <tag> <frames_per_launch> <workload key (bench.py workload_key)>
"""
import csv
import json
import os
import re
import sys
from collections import defaultdict

FAMILIES = [("analyze_tail", r"k_analyze<\d+, \d+, false"), ("analyze", r"k_analyze<\d+, \d+, true"), ("analyze", r"k_ana4<"), ("analyze", r"k_ana1<"),
            ("pack_tail", r"k_pack<\d+, \d+, false"), ("pack", r"k_pack<\d+, \d+, true"), ("pack", r"k_pack4<"), ("pack", r"k_packw<"),
            ("scan", r"k_scan"), ("md5", r"k_md5_streams"), ("md5_blocks", r"k_md5_blocks")]


def family(name):
    for fam, pat in FAMILIES:
        if re.search(pat, name):
            return fam
    return None


def main():
    d, tag, frames = sys.argv[1], sys.argv[2], int(sys.argv[3])
    workload = sys.argv[4] if len(sys.argv) > 4 else None
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    stats = {}
    ks = os.path.join(d, "kt", "kt_kernel_stats.csv")
    if os.path.exists(ks):
        for r in csv.DictReader(open(ks)):
            fam = family(r["Name"])
            if fam:
                stats[fam] = {"calls": int(r["Calls"]), "avg_ns": float(r["AverageNs"]),
                              "pct": float(r["Percentage"]), "name": r["Name"]}
    ctr = defaultdict(lambda: defaultdict(list))
    for sub in sorted(os.listdir(d)):
        f = os.path.join(d, sub, "pmc_counter_collection.csv")
        if not sub.startswith("pmc") or not os.path.exists(f):
            continue
        for r in csv.DictReader(open(f)):
            fam = family(r["Kernel_Name"])
            if fam:
                ctr[fam][r["Counter_Name"]].append(float(r["Counter_Value"]))
    avg = {fam: {c: sum(v) / len(v) for c, v in cs.items()} for fam, cs in ctr.items()}
    hbm = {}
    for fam, cs in avg.items():
        if "FETCH_SIZE" in cs and "WRITE_SIZE" in cs:
            hbm[fam] = round(cs["FETCH_SIZE"] * 1024 * 2 + cs["WRITE_SIZE"] * 1024)
    out = {"tag": tag, "workload": workload, "frames_per_launch": frames, "hbm_bytes_per_launch": hbm,
           "fetch_note": "FETCH_SIZE KiB x1024 x2 (gfx950 half-count correction: the guide's 16-B loads, and "
                         "4-B LDS-DMA calibrated in profiles/r4g_fetch_calib.json) + WRITE_SIZE KiB x1024",
           "kernel_stats": stats, "counters_per_dispatch": avg}
    os.makedirs(os.path.join(root, "profiles"), exist_ok=True)
    json.dump(out, open(os.path.join(root, "profiles", f"{tag}_pmc.json"), "w"), indent=1)
    lines = [f"# rocprofv3 summary: {tag}", "", f"workload: {workload}; frames per launch: {frames}", "",
             "| kernel | calls | avg us | % time | HBM MB/launch (corrected) |", "|---|---|---|---|---|"]
    for fam in dict.fromkeys(f for f, _ in FAMILIES if f in stats):
        s = stats[fam]
        h = hbm.get(fam)
        lines.append(f"| {fam} | {s['calls']} | {s['avg_ns']/1e3:.1f} | {s['pct']:.1f} | "
                     f"{h/1e6:.1f} |" if h else f"| {fam} | {s['calls']} | {s['avg_ns']/1e3:.1f} | {s['pct']:.1f} | - |")
    lines += ["", "## counters per dispatch", ""]
    for fam, cs in avg.items():
        lines.append(f"- **{fam}**: " + ", ".join(f"{k}={v:.4g}" for k, v in sorted(cs.items())))
    open(os.path.join(root, "profiles", f"{tag}_summary.md"), "w").write("\n".join(lines) + "\n")
    print("\n".join(lines))


if __name__ == "__main__":
    main()
