#!/bin/bash
# r3i profiles: the C2 line at defaults (split encode: roofline.traffic for the bench) and the fused
# schedule (FLACGPU_FUSED=1) for its counters.
set -o pipefail
bash tools/profile.sh r3i_c2 c2 65536 16384 && head -12 profiles/r3i_c2_summary.md || exit 1
FLACGPU_FUSED=1 bash tools/profile.sh r3i_c2fused c2 65536 16384 && head -12 profiles/r3i_c2fused_summary.md
