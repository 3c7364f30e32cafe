#!/bin/bash
# r3o: k_pack4 ORs the CRC into its stores (one barrier less per frame): parity with that build, A/B.
set -o pipefail
mkdir -p gpurun_out
FLACGPU_LIB=$PWD/zig-flac_amd/build_new/libflacgpu.so timeout -k 10 400 python -u -m pytest tests/test_gpu_plan.py tests/test_gpu_parity.py tests/test_gpu_fuzz.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r3o_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/r3o_pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/r3o_pytest.log | head; exit $rc; }
AB_REPS=3 bash tools/ab_cfgs.sh r3o "c2" zig-flac_amd/build zig-flac_amd/build_new || exit 1
