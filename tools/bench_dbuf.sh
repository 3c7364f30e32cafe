#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "stream_parity or tail_lengths" --timeout 120 --timeout-method thread > gpurun_out/pytest_db.log 2>&1 || { echo PYTEST_FAIL; tail -30 gpurun_out/pytest_db.log; exit 1; }
tail -1 gpurun_out/pytest_db.log
for v in 1 0; do
  for mode in "--no-md5" ""; do
    FLACGPU_PACK_DBUF=$v timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu $mode > gpurun_out/bench_db.log 2>&1 || { echo BENCH_FAIL; tail -5 gpurun_out/bench_db.log; exit 1; }
    tail -1 gpurun_out/bench_db.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('dbuf=$v $mode', d['value'], d['kernel_ms_per_step'])"
  done
done
