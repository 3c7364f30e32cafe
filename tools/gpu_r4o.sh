#!/bin/bash
# r4o: GPU tests, then c4 A/B: the NC=4 analysis build vs the runtime-channel one, and just-in-time
# tickets for the split pack too (FLACGPU_SPLIT_JIT=3)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r4o_parity.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; tail -2 gpurun_out/r4o_parity.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/r4o_parity.log | head; exit $rc; }
AB_REPS=2 AB_ARGS="--frames 65536" tools/ab.sh r4o "c4" nc4:- rt:FLACGPU_NC4=0 jit3:FLACGPU_SPLIT_JIT=3
AB_REPS=2 tools/ab.sh r4o "c2" fused:- unfused:lib=zig-flac_amd/build_x
