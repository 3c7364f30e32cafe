#!/bin/bash
# Bench lines for the BASELINE configs (c2 headline; c3/c4/c5 parity configs), verified output.
set -o pipefail
mkdir -p gpurun_out
for c in c2 c3 c4 c5; do
  timeout -k 10 300 python bench.py --config $c --steps 5 --warmup 2 --no-cpu --verify > gpurun_out/bench_$c.log 2>&1 || { echo BENCH_FAIL $c; tail -5 gpurun_out/bench_$c.log; exit 1; }
  tail -1 gpurun_out/bench_$c.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$c', d['value'], d['kernel_ms_per_step'], d['output_ok'], d['config']['compression_ratio'])"
done
