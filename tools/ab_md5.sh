#!/bin/bash
# A/B of libflacgpu.so variants (FLACGPU_LIB) on bench shapes.  Usage: tools/ab_md5.sh <tag> <variant dirs...>
set -o pipefail
TAG=$1; shift
mkdir -p gpurun_out
for V in "$@"; do
  for S in 8192 16384; do
    FLACGPU_LIB=$PWD/zig-flac_amd/$V/libflacgpu.so timeout -k 10 120 python bench.py --streams $S --steps 10 --warmup 2 --no-cpu --no-curve --no-e2e --verify-streams 8 > gpurun_out/ab_${TAG}_${V}_$S.json 2>/dev/null || { echo "FAIL $V $S"; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], sys.argv[3], d['value'], d['output_ok'], d['kernel_ms_per_step'])" gpurun_out/ab_${TAG}_${V}_$S.json $V $S
  done
done
