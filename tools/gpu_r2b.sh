#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
bash tools/gpu_tests.sh r2b tests/test_file_host.py tests/test_parallel.py tests/test_gpu_plan.py || exit 1
timeout -k 10 400 python bench.py > gpurun_out/bench_r2b.json 2> gpurun_out/bench_r2b.err || { echo BENCH_FAIL; tail -20 gpurun_out/bench_r2b.err; exit 1; }
cat gpurun_out/bench_r2b.json
timeout -k 10 200 python bench.py --streams 16384 --no-cpu --no-curve --no-e2e > gpurun_out/bench_r2b_16k.json 2>> gpurun_out/bench_r2b.err && cut -c1-400 gpurun_out/bench_r2b_16k.json
timeout -k 10 200 python bench.py --no-md5 --no-cpu --no-curve --no-e2e > gpurun_out/bench_r2b_nomd5.json 2>> gpurun_out/bench_r2b.err && cut -c1-400 gpurun_out/bench_r2b_nomd5.json
