#!/bin/bash
# GPU-box check: parity tests, a verified short bench, then the default bench line.
# Usage (from the repo root, on the GPU box): tools/gpu_check.sh [tag]
set -o pipefail
TAG=${1:-run}
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/pytest_$TAG.log; exit 1; }
tail -2 gpurun_out/pytest_$TAG.log
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu --verify > gpurun_out/bench_verify_$TAG.log 2>&1 || { echo BENCH_FAIL; tail -5 gpurun_out/bench_verify_$TAG.log; exit 1; }
tail -1 gpurun_out/bench_verify_$TAG.log
timeout -k 10 300 python bench.py --no-cpu --no-md5 --steps 10 --warmup 2 > gpurun_out/bench_nomd5_$TAG.log 2>&1 || { echo BENCH2_FAIL; tail -5 gpurun_out/bench_nomd5_$TAG.log; exit 1; }
tail -1 gpurun_out/bench_nomd5_$TAG.log
