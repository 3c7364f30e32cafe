#!/bin/bash
# Fast GPU check: C2 parity tests (+ LPC subset), then the quick c2 bench lines.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_all.log 2>&1 || { echo TEST_FAIL; tail -40 gpurun_out/pytest_all.log; exit 1; }
tail -2 gpurun_out/pytest_all.log
bash tools/bench_quick.sh
