#!/bin/bash
# r3x: larger steps at 16384 streams (12 and 16 blocks per stream per step) against 8 (same box, 2 reps)
set -o pipefail
mkdir -p gpurun_out
for rep in 1 2; do
  for SH in "131072 16384" "196608 16384" "262144 16384"; do
    set -- $SH
    out=gpurun_out/r3x_${1}_${2}_$rep.json
    timeout -k 10 300 python bench.py --frames $1 --streams $2 --steps 10 --warmup 2 --no-cpu --no-curve --no-e2e --no-sharded --verify-streams 4 > $out 2> $out.err || { echo "FAIL $SH"; tail -5 $out.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['ms_per_step'], d['output_ok'], d['kernel_ms_per_step'])" $out "$1x$2"
  done
done
