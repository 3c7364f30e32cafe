#!/bin/bash
# r4zc: the C2 build (fg_enc_b2_l0) scheduled with -mllvm -amdgpu-sched-strategy=max-ilp (build_x;
# k_analyze 13 spilled VGPRs, k_pack4 2): GPU suite on it, then the same-box A/B
set -o pipefail
mkdir -p gpurun_out
FLACGPU_LIB=$PWD/zig-flac_amd/build_x/libflacgpu.so timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r4zc_pytest.log 2>&1 || { tail -30 gpurun_out/r4zc_pytest.log; exit 1; }
tail -2 gpurun_out/r4zc_pytest.log
AB_REPS=3 tools/ab.sh r4zc "c2" base:- ilp:lib=zig-flac_amd/build_x
