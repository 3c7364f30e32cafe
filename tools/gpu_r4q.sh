#!/bin/bash
# r4q: GPU tests; C2 A/B with the bestOrder LDS stash + late subframe-header bits vs the previous
# commit (build_ab); C2 profile (analysis WRITE_SIZE)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r4q_parity.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; tail -2 gpurun_out/r4q_parity.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/r4q_parity.log | head; exit $rc; }
AB_REPS=2 tools/ab.sh r4q "c2" new:- old:lib=zig-flac_amd/build_ab || exit 1
tools/profile.sh r4q_c2 c2 262144 16384 > gpurun_out/r4q_prof.log 2>&1 || { echo profile failed; tail -5 gpurun_out/r4q_prof.log; exit 1; }
head -12 profiles/r4q_c2_summary.md
