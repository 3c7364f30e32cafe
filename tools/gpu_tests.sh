#!/bin/bash
# GPU parity tests only (one pytest process), log under gpurun_out/.
# Usage (GPU box, repo root): tools/gpu_tests.sh <tag> [pytest selection...]
set -o pipefail
TAG=${1:-run}; shift || true
SEL=${@:-tests}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest $SEL -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
rc=$?
grep -E "passed|failed|error" gpurun_out/pytest_$TAG.log | tail -3
[ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/pytest_$TAG.log | head -30; exit $rc; }
