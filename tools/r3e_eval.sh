#!/bin/bash
# Round-3 re-entry check on the GPU box: full GPU suite at defaults, then the overlap and
# per-XCD queue A/Bs (tools/ab_ovl.sh, tools/ab_xcd.sh).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r3e_pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/r3e_pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
bash tools/ab_ovl.sh r3e || exit 1
bash tools/ab_xcd.sh r3e || exit 1
