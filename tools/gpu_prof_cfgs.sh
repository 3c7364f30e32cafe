#!/bin/bash
# Keyed rocprofv3 kernel trace + PMC at the bench shape for the given configs.
# Usage: tools/gpu_prof_cfgs.sh <tag> <configs...>
set -o pipefail
TAG=$1; shift
mkdir -p gpurun_out
for C in "$@"; do
  S=16384
  bash tools/profile.sh ${TAG}_$C $C 65536 $S || { echo PROFILE_FAIL $C; exit 1; }
  head -12 profiles/${TAG}_${C}_summary.md
done
