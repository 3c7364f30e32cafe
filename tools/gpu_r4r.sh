#!/bin/bash
# r4r: GPU tests; A/B vs the previous commit (build_ab) at C2 and c3/c4/c5 (65536): C2 analysis with
# no in-loop spill stores (bestOrder LDS stash, late subframe-header bits, coalesced descriptor
# headers); C2 profile
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r4r_parity.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; tail -2 gpurun_out/r4r_parity.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/r4r_parity.log | head; exit $rc; }
AB_REPS=2 tools/ab.sh r4r "c2" new:- old:lib=zig-flac_amd/build_ab || exit 1
AB_REPS=1 AB_ARGS="--frames 65536" tools/ab.sh r4r "c3 c4 c5" new:- old:lib=zig-flac_amd/build_ab || exit 1
tools/profile.sh r4r_c2 c2 262144 16384 > gpurun_out/r4r_prof.log 2>&1 || { echo profile failed; tail -5 gpurun_out/r4r_prof.log; exit 1; }
head -12 profiles/r4r_c2_summary.md
