#!/bin/bash
# r3p: every candidate wave measures its exact segment bits before the estimate barrier: parity with
# that build (stereo configs), then same-box A/B.
set -o pipefail
mkdir -p gpurun_out
FLACGPU_LIB=$PWD/zig-flac_amd/build_new/libflacgpu.so timeout -k 10 400 python -u -m pytest tests/test_gpu_plan.py tests/test_gpu_parity.py tests/test_gpu_lpc.py tests/test_gpu_fuzz.py tests/test_gpu_fused.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r3p_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/r3p_pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/r3p_pytest.log | head; exit $rc; }
AB_REPS=2 bash tools/ab_cfgs.sh r3p "c2 c3 c5" zig-flac_amd/build zig-flac_amd/build_new || exit 1
