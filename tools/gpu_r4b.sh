#!/bin/bash
# r4b: k_ana1 (one wave per C2 frame) parity, then same-box A/B against k_analyze (tools/ab.sh)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_plan.py -q --timeout 120 --timeout-method thread > gpurun_out/r4b_parity.log 2>&1
rc=$?
echo "parity rc=$rc"; tail -3 gpurun_out/r4b_parity.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
AB_REPS=2 tools/ab.sh r4b c2 v1:FLACGPU_ANA1=1 v2:FLACGPU_ANA1=2 four:FLACGPU_ANA1=0
