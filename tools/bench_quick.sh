#!/bin/bash
# Quick c2 bench lines: pipelined MD5 (default), joined MD5, no MD5.
set -o pipefail
mkdir -p gpurun_out
for mode in "" "--md5-join" "--no-md5"; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu --verify $mode > gpurun_out/bench_q.log 2>&1 || { echo BENCH_FAIL $mode; tail -5 gpurun_out/bench_q.log; exit 1; }
  tail -1 gpurun_out/bench_q.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$mode', d['value'], d['ms_per_step'], d['kernel_ms_per_step'], d['output_ok'], d['roofline']['kernel'], d['roofline']['frac'])"
done
