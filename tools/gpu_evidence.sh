#!/bin/bash
# Round evidence: full GPU suite, c2-c5 lines, the default
# bench line (CPU baseline, stream curve, end-to-end).  GPU box, repo root.
set -o pipefail
TAG=${1:-r2f}
mkdir -p gpurun_out
bash tools/gpu_cfgs.sh $TAG "c3 c4 c5" || exit 1
timeout -k 10 600 python -u bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { echo BENCH_FAIL; tail -20 gpurun_out/bench_$TAG.err; exit 1; }
tail -1 gpurun_out/bench_$TAG.json | cut -c1-600
