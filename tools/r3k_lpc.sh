#!/bin/bash
# r3k: Levinson-Durbin coefficients through LDS (in-place pair update): LPC GPU tests, A/B c3/c5.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_lpc.py tests/test_gpu_plan.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r3k_pytest_lpc.log 2>&1
rc=$?; tail -3 gpurun_out/r3k_pytest_lpc.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/r3k_pytest_lpc.log | head; exit $rc; }
bash tools/ab_cfgs.sh r3k "c3 c5" zig-flac_amd/build_prev zig-flac_amd/build || exit 1
