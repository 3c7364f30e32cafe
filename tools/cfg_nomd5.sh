#!/bin/bash
# Config bench lines without the MD5 (encode kernels alone).  Usage: tools/cfg_nomd5.sh <tag> "<configs>" [extra bench args]
set -o pipefail
TAG=$1; CFGS=$2; shift 2
mkdir -p gpurun_out
for C in $CFGS; do
  timeout -k 10 200 python bench.py --config $C --steps 5 --warmup 2 --no-cpu --no-curve --no-e2e --verify-streams 4 --no-md5 "$@" > gpurun_out/nm_${TAG}_$C.json 2> gpurun_out/nm_${TAG}_$C.err || { echo "FAIL $C"; tail -3 gpurun_out/nm_${TAG}_$C.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['output_ok'], d['kernel_ms_per_step'])" gpurun_out/nm_${TAG}_$C.json $C
done
