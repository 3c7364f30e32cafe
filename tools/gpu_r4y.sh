#!/bin/bash
# r4y: MD5 schedule knobs at the current code: c4 with the three-chunk ring (kernel 2), C2 without
# the reserved MD5 slots (FLACGPU_MD5_RESERVE=0; auto reserves them at 16 blocks per stream)
set -o pipefail
mkdir -p gpurun_out
AB_REPS=2 AB_ARGS="--frames 65536" tools/ab.sh r4y "c4" base:- k2:FLACGPU_MD5_KERNEL=2 || exit 1
AB_REPS=2 tools/ab.sh r4y "c2" base:- rsv0:FLACGPU_MD5_RESERVE=0
