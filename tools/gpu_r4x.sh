#!/bin/bash
# r4x: the C2 analysis's exact pass split between a written FIXED subframe's wave and an unwritten
# candidate's wave (FG_XSPLIT) vs the previous commit (build_ab): all GPU tests, C2 A/B, 3 reps
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r4x_parity.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; tail -2 gpurun_out/r4x_parity.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/r4x_parity.log | head; exit $rc; }
AB_REPS=3 tools/ab.sh r4x "c2" new:- old:lib=zig-flac_amd/build_ab
