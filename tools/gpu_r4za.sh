#!/bin/bash
# r4za: phase stamps of the C2 analysis and pack kernels at the final code (build_st = -DFG_STAMPS)
set -o pipefail
mkdir -p gpurun_out
FLACGPU_LIB=$PWD/zig-flac_amd/build_st/libflacgpu.so timeout -k 10 200 python tools/stamps.py > gpurun_out/r4za_stamps_c2_16.log 2>&1 || { tail -20 gpurun_out/r4za_stamps_c2_16.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r4za_stamps_c2_16.log
