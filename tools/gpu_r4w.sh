#!/bin/bash
# r4w: k_pack4 drains its DMAs and takes its ticket before the output stores, so the next frame's
# top waits for LDS only (FG_P4_EARLYWAIT) vs the previous commit (build_ab): C2 A/B + pack4 tests
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_plan.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r4w_parity.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; tail -2 gpurun_out/r4w_parity.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/r4w_parity.log | head; exit $rc; }
AB_REPS=3 tools/ab.sh r4w "c2" new:- old:lib=zig-flac_amd/build_ab
