#!/bin/bash
# r3m: LDS-only descriptor barrier + dword parameter stores in the analysis: GPU suite, A/B.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r3m_pytest_gpu.log 2>&1
rc=$?; tail -2 gpurun_out/r3m_pytest_gpu.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/r3m_pytest_gpu.log | head; exit $rc; }
bash tools/ab_cfgs.sh r3m "c2 c4 c3" zig-flac_amd/build_prev zig-flac_amd/build || exit 1
