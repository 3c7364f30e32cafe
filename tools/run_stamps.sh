#!/bin/bash
# Phase stamps (-DFG_STAMPS build in zig-flac_amd/build_st) for C2 and the wide configs.
set -o pipefail
mkdir -p gpurun_out
for cfg in "2 16 44100 0" "8 24 96000 0" "2 24 96000 8" "2 32 192000 12"; do
  set -- $cfg
  tag=c${1}_${2}
  CH=$1 BITS=$2 RATE=$3 LPC=$4 FLACGPU_LIB=$PWD/zig-flac_amd/build_st/libflacgpu.so timeout -k 10 200 python tools/stamps.py > gpurun_out/stamps_$tag.log 2>&1 || { echo STAMPS_FAIL $tag; tail -20 gpurun_out/stamps_$tag.log; exit 1; }
  echo "== $tag"; grep -v amdgpu.ids gpurun_out/stamps_$tag.log
done
