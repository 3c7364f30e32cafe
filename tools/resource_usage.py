"""Summarise `hipcc -Rpass-analysis=kernel-resource-usage` remarks: one line per kernel (tools only).
Usage: python tools/resource_usage.py remarks.txt [substring]"""
import re
import subprocess
import sys

txt = open(sys.argv[1]).read()
key = sys.argv[2] if len(sys.argv) > 2 else ""
cur, rows = None, {}
for line in txt.splitlines():
    m = re.search(r"remark: Function Name: (\S+)", line)
    if m:
        cur = m.group(1)
        rows[cur] = {}
        continue
    m = re.search(r"remark:\s+([^:]+): (\S+) \[-Rpass", line)
    if m and cur:
        rows[cur][m.group(1).strip()] = m.group(2)
names = subprocess.run(["c++filt"], input="\n".join(rows), capture_output=True, text=True).stdout.split("\n")
for (k, v), dn in zip(rows.items(), names):
    if key and key not in dn:
        continue
    print(f"{dn[:58]:58s} VGPR {v.get('VGPRs','?'):>3} spillV {v.get('VGPRs Spill','?'):>3} scratch "
          f"{v.get('ScratchSize [bytes/lane]','?'):>4} occ {v.get('Occupancy [waves/SIMD]','?')} "
          f"spillS {v.get('SGPRs Spill','?')}")
