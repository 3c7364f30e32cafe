#!/bin/bash
# r4u: GPU tests; A/B of the LDS job ring (next job records by LDS-DMA instead of registers) vs
# the previous commit (build_ab) at C2 and c3/c4/c5 (65536 frames)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r4u_parity.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; tail -2 gpurun_out/r4u_parity.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/r4u_parity.log | head; exit $rc; }
AB_REPS=2 AB_ARGS="--frames 65536" tools/ab.sh r4u "c4 c5 c3" new:- old:lib=zig-flac_amd/build_ab || exit 1
AB_REPS=2 tools/ab.sh r4u "c2" new:- old:lib=zig-flac_amd/build_ab
