#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
for v in build build_p0 build_p1; do
  FLACGPU_LIB=$PWD/zig-flac_amd/$v/libflacgpu.so timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu > gpurun_out/bench_p.log 2>&1 || { echo BENCH_FAIL $v; tail -5 gpurun_out/bench_p.log; exit 1; }
  tail -1 gpurun_out/bench_p.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', d['value'], d['ms_per_step'], d['kernel_ms_per_step'])"
done
