#!/bin/bash
# Round evidence on one GPU box: the default bench line (with the CPU baseline), then the
# rocprofv3 kernel-trace + PMC profile of the same command -> profiles/<tag>_*.
# Usage: tools/round_evidence.sh <tag>
set -o pipefail
TAG=${1:-r1}
mkdir -p gpurun_out
timeout -k 10 400 python bench.py > gpurun_out/bench_default.log 2>&1 || { echo BENCH_FAIL; tail -5 gpurun_out/bench_default.log; exit 1; }
tail -1 gpurun_out/bench_default.log | tee gpurun_out/${TAG}_bench.json
bash tools/profile.sh $TAG 65536
