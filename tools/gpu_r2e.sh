#!/bin/bash
# Phase stamps (build_st) for the four configs, then the keyed C2 profile at the bench default.
set -o pipefail
mkdir -p gpurun_out
bash tools/run_stamps.sh || exit 1
bash tools/profile.sh r2e_c2 c2 65536 16384 || { echo PROFILE_FAIL; exit 1; }
cat profiles/r2e_c2_summary.md
