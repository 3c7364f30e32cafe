#!/bin/bash
# r3f: table-free CRC-16 + b128 frame stores: GPU suite, same-box A/B vs the HEAD build, PMC.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r3f_pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/r3f_pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
bash tools/ab_cfgs.sh r3f "c2 c4 c3 c5" zig-flac_amd/build_base zig-flac_amd/build || exit 1
bash tools/profile.sh r3f_c2 c2 65536 16384 && head -12 profiles/r3f_c2_summary.md
