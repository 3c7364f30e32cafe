#!/bin/bash
# A/B of libflacgpu.so variants on BASELINE configs.  Usage: tools/ab_cfg.sh <tag> "<configs>" <variant dirs...>
set -o pipefail
TAG=$1; CFGS=$2; shift 2
mkdir -p gpurun_out
for V in "$@"; do
  for C in $CFGS; do
    FLACGPU_LIB=$PWD/zig-flac_amd/$V/libflacgpu.so timeout -k 10 200 python bench.py --config $C --steps 5 --warmup 2 --no-cpu --no-curve --no-e2e --verify-streams 8 > gpurun_out/ab_${TAG}_${V}_$C.json 2>gpurun_out/ab_${TAG}_${V}_$C.err || { echo "FAIL $V $C"; tail -3 gpurun_out/ab_${TAG}_${V}_$C.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], sys.argv[3], d['value'], d['output_ok'], d['kernel_ms_per_step'])" gpurun_out/ab_${TAG}_${V}_$C.json $V $C
  done
done
