#!/bin/bash
# Keyed rocprofv3 kernel trace + PMC of the LPC configs (c3, c5) and c4 at the bench shape.
set -o pipefail
mkdir -p gpurun_out
for C in c3 c5 c4; do
  bash tools/profile.sh r2f_$C $C 65536 16384 || { echo PROFILE_FAIL $C; exit 1; }
  head -12 profiles/r2f_${C}_summary.md
done
