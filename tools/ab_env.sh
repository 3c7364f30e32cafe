#!/bin/bash
# A/B of env knobs on the default C2 bench line (no CPU baseline / curve / e2e).
# Usage: tools/ab_env.sh "<VAR=val ...>" "<VAR=val ...>" ...   (each argument one variant; "" = defaults)
set -o pipefail
mkdir -p gpurun_out
ARGS=${AB_ARGS:-"--steps 20 --warmup 3 --no-cpu --no-curve --no-e2e --verify-streams 8"}
for rep in 1 2; do
  for V in "$@"; do
    env $V timeout -k 10 200 python bench.py $ARGS > gpurun_out/ab.json 2> gpurun_out/ab.err || { echo "FAIL [$V]"; tail -5 gpurun_out/ab.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open('gpurun_out/ab.json')); print(sys.argv[1], d['value'], d['ms_per_step'], d['output_ok'], d['kernel_ms_per_step'])" "[$V]"
  done
done
