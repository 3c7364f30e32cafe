#!/bin/bash
# A/B of libflacgpu.so builds (FLACGPU_LIB) on the default C2 bench line, alternating.
# Usage: tools/ab_lib.sh <tag> <lib dir>...   (e.g. zig-flac_amd/build_old zig-flac_amd/build)
set -o pipefail
TAG=$1; shift
mkdir -p gpurun_out
ARGS=${AB_ARGS:-"--steps 20 --warmup 3 --no-cpu --no-curve --no-e2e --no-sharded --verify-streams 8"}
for rep in 1 2; do
  for V in "$@"; do
    out=gpurun_out/ab_${TAG}_$(basename $V)_$rep.json
    FLACGPU_LIB=$PWD/$V/libflacgpu.so timeout -k 10 200 python bench.py $ARGS > $out 2> $out.err || { echo "FAIL $V"; tail -5 $out.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['ms_per_step'], d['output_ok'], d['kernel_ms_per_step'])" $out $V
  done
done
