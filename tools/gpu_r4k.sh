#!/bin/bash
# r4k: r4j (encode_files tests + e2e per-file vs batch), then c5 MD5 scheduling A/B at the
# configs-block shape (65536 frames): priority, kernel variant, reserved slots
set -o pipefail
bash tools/gpu_r4j.sh || exit 1
AB_REPS=1 AB_ARGS="--frames 65536" tools/ab.sh r4k "c5" base:- prio1:FLACGPU_MD5_PRIO=1 prio3:FLACGPU_MD5_PRIO=3 k2:FLACGPU_MD5_KERNEL=2 rsv:FLACGPU_MD5_RESERVE=1
