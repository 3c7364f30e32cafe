#!/bin/bash
# GPU-box check of the LPC path, the whole GPU suite, then the config bench lines.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_lpc.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_lpc.log 2>&1 || { echo LPC_FAIL; tail -60 gpurun_out/pytest_lpc.log; exit 1; }
tail -2 gpurun_out/pytest_lpc.log
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_all.log 2>&1 || { echo ALL_FAIL; tail -60 gpurun_out/pytest_all.log; exit 1; }
tail -2 gpurun_out/pytest_all.log
bash tools/bench_configs.sh
