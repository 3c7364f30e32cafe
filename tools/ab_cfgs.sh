#!/bin/bash
# Same-box A/B of libflacgpu.so builds (FLACGPU_LIB) over bench configs, alternating builds.
# Usage (GPU box, repo root): tools/ab_cfgs.sh <tag> "<configs>" <lib dir>...
#   e.g. tools/ab_cfgs.sh crc "c2 c4" zig-flac_amd/build_base zig-flac_amd/build
set -o pipefail
TAG=$1; CFGS=$2; shift 2
mkdir -p gpurun_out
REPS=${AB_REPS:-2}
for cfg in $CFGS; do
  CA=""; [ "$cfg" = c2 ] || CA="--config $cfg"
  ST=20; [ "$cfg" = c2 ] || ST=8
  for rep in $(seq $REPS); do
    for V in "$@"; do
      out=gpurun_out/ab_${TAG}_${cfg}_$(basename $V)_$rep.json
      FLACGPU_LIB=$PWD/$V/libflacgpu.so timeout -k 10 240 python bench.py $CA --steps $ST --warmup 2 --no-cpu --no-curve --no-e2e --no-sharded --verify-streams 8 > $out 2> $out.err || { echo "FAIL $cfg $V"; tail -5 $out.err; exit 1; }
      python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['ms_per_step'], d['output_ok'], d['kernel_ms_per_step'])" $out "$cfg $(basename $V)"
    done
  done
done
