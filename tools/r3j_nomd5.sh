#!/bin/bash
# r3j: what the stream MD5 costs the step, per config: bench lines with and without it (same box)
set -o pipefail
mkdir -p gpurun_out
for cfg in c2 c3 c4 c5; do
  CA=""; [ "$cfg" = c2 ] || CA="--config $cfg"
  ST=20; [ "$cfg" = c2 ] || ST=8
  for M in md5 nomd5; do
    X=""; [ $M = nomd5 ] && X="--no-md5"
    out=gpurun_out/r3j_${cfg}_$M.json
    timeout -k 10 240 python bench.py $CA $X --steps $ST --warmup 2 --no-cpu --no-curve --no-e2e --no-sharded --verify-streams 8 > $out 2> $out.err || { echo "FAIL $cfg $M"; tail -5 $out.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['ms_per_step'], d['output_ok'], d['kernel_ms_per_step'])" $out "$cfg $M"
  done
done
