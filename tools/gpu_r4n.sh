#!/bin/bash
# r4n: LPC sub-phase stamps (c3, c5 shapes), then rocprofv3 kernel stats + PMC for c4 (65536,
# split items just in time) and C2 (262144, the headline shape) at this round's code
set -o pipefail
mkdir -p gpurun_out
for cfg in "2 24 96000 8" "2 32 192000 12"; do
  set -- $cfg
  tag=c${1}_${2}
  CH=$1 BITS=$2 RATE=$3 LPC=$4 FLACGPU_LIB=$PWD/zig-flac_amd/build_st/libflacgpu.so timeout -k 10 200 python tools/stamps.py > gpurun_out/r4n_stamps_$tag.log 2>&1 || { echo STAMPS_FAIL $tag; tail -20 gpurun_out/r4n_stamps_$tag.log; exit 1; }
  echo "== $tag"; grep -v amdgpu.ids gpurun_out/r4n_stamps_$tag.log | head -20
done
tools/profile.sh r4n_c4 c4 65536 16384 || exit 1
tools/profile.sh r4n_c2 c2 262144 16384 || exit 1
cat profiles/r4n_c4_summary.md profiles/r4n_c2_summary.md
