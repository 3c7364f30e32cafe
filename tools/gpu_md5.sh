#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "md5" --timeout 120 --timeout-method thread > gpurun_out/pytest_md5.log 2>&1 || { echo MD5_FAIL; tail -30 gpurun_out/pytest_md5.log; exit 1; }
tail -1 gpurun_out/pytest_md5.log
bash tools/bench_configs.sh
