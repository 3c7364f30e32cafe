#!/bin/bash
# r3z: the C2 encode waves at issue priority 1 (FLACGPU_ENC_PRIO=1), above the MD5 waves' 0: at the
# 262144-block step the MD5 (6.7 ms) has ~1 ms of slack under the encode (7.75 ms); same box, 3 reps
set -o pipefail
mkdir -p gpurun_out
for rep in 1 2 3; do
  for P in 0 1; do
    out=gpurun_out/r3z_p${P}_$rep.json
    FLACGPU_ENC_PRIO=$P timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu --no-curve --no-e2e --no-sharded --verify-streams 8 > $out 2> $out.err || { echo "FAIL $P"; tail -5 $out.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['ms_per_step'], d['output_ok'], d['kernel_ms_per_step'])" $out "prio$P"
  done
done
