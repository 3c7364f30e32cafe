#!/bin/bash
# Static VALU mix (SIMD-cycles per instruction at the measured gfx950 issue rates) of every bench
# config's analysis / pack / MD5 kernels -> profiles/<tag>_valu_mix.json, which bench.py reads for
# `weighted_issue_frac`.  CPU only (hipcc -S of the current sources, ~6 min on 8 cores).
# Usage: tools/valu_mix.sh <tag>
set -e
TAG=${1:-r5}
REPO=$(cd "$(dirname "$0")/.." && pwd)
OUT=$(mktemp -d)
FLAGS="-O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=off -mllvm -pragma-unroll-threshold=1000000 --cuda-device-only -S"
for v in "2 0" "3 8" "3 0" "4 12"; do
  set -- $v
  /opt/rocm/bin/hipcc $FLAGS -DFG_B=$1 -DFG_LPW=$2 -o $OUT/b$1l$2.s $REPO/zig-flac_amd/csrc/fg_enc.hip 2>/dev/null &
done
/opt/rocm/bin/hipcc $FLAGS -o $OUT/misc.s $REPO/zig-flac_amd/csrc/fg_misc.hip 2>/dev/null &
wait
V=$REPO/tools/valu_rates.py
python3 - "$OUT" "$V" "$REPO/profiles/${TAG}_valu_mix.json" <<'PY'
import json, subprocess, sys
out, v, dst = sys.argv[1:4]
K = {  # config -> kernel -> (listing, mangled-name key)
    "c2": {"analyze": ("b2l0", "9k_analyzeILi2ELi16ELb1ELi256ELi2ELi0ELb0"), "pack": ("b2l0", "7k_pack4ILi512"),
           "md5": ("misc", "17k_md5_streams_ldsILj1ELj2ELj4")},
    "c3": {"analyze": ("b3l8", "9k_analyzeILi3ELi24ELb1ELi256ELi2ELi8ELb0"),
           "pack": ("b3l8", "6k_packILi3ELi24ELb1ELi256ELi2ELi8E"), "md5": ("misc", "17k_md5_streams_ldsILj1ELj2ELj4")},
    "c4": {"analyze": ("b3l0", "9k_analyzeILi3ELi24ELb1ELi256ELi4ELi0ELb0"),
           "pack": ("b3l0", "7k_packwILi3ELi24ELi0ELi0ELi32ELb1"), "md5": ("misc", "17k_md5_streams_ldsILj1ELj2ELj4")},
    "c5": {"analyze": ("b4l12", "9k_analyzeILi4ELi32ELb1ELi256ELi2ELi12ELb0"),
           "pack": ("b4l12", "7k_packwILi4ELi32ELi2ELi12ELi16ELb0"), "md5": ("misc", "17k_md5_streams_ldsILj1ELj3ELj4")},
}
res = {"note": "static VALU mix per kernel (tools/valu_rates.py), SIMD-cycles per wave-instruction at the "
               "per-opcode issue rates measured in profiles/r5_issue_micro.txt"}
for cfg, ks in K.items():
    res[cfg] = {}
    for k, (f, key) in ks.items():
        r = subprocess.run([sys.executable, v, f"{out}/{f}.s", key, "--json"], capture_output=True, text=True)
        res[cfg][k] = json.loads(r.stdout) if r.returncode == 0 and r.stdout.strip() else None
json.dump(res, open(dst, "w"), indent=1)
print(json.dumps(res)[:600])
PY
rm -rf $OUT
