#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
FLACGPU_LIB=$PWD/zig-flac_amd/build_st/libflacgpu.so timeout -k 10 200 python tools/stamps.py > gpurun_out/stamps.log 2>&1 || { echo STAMPS_FAIL; tail -20 gpurun_out/stamps.log; exit 1; }
grep -v amdgpu.ids gpurun_out/stamps.log
