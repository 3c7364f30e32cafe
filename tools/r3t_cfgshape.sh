#!/bin/bash
# r3t: batch shape of the c3/c4/c5 lines (65536 vs 131072 frames per step, 16384 streams; same box, 2 reps)
set -o pipefail
mkdir -p gpurun_out
for rep in 1 2; do
  for C in c3 c4 c5; do
    for F in 65536 131072; do
      out=gpurun_out/r3t_${C}_${F}_$rep.json
      timeout -k 10 300 python bench.py --config $C --frames $F --steps 10 --warmup 2 --no-cpu --no-curve --no-e2e --no-sharded --verify-streams 4 > $out 2> $out.err || { echo "FAIL $C $F"; tail -5 $out.err; exit 1; }
      python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['ms_per_step'], d['output_ok'], d['kernel_ms_per_step'])" $out "$C:$F"
    done
  done
done
