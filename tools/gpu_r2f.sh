#!/bin/bash
# Round-2 evidence after the LPC order-selection change: full GPU suite, c2-c5 lines, the default
# bench line (CPU baseline, stream curve, end-to-end).  GPU box, repo root.
set -o pipefail
mkdir -p gpurun_out
bash tools/gpu_cfgs.sh r2f "c3 c4 c5" || exit 1
timeout -k 10 600 python -u bench.py > gpurun_out/bench_r2f.json 2> gpurun_out/bench_r2f.err || { echo BENCH_FAIL; tail -20 gpurun_out/bench_r2f.err; exit 1; }
tail -1 gpurun_out/bench_r2f.json | cut -c1-600
