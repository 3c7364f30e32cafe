#!/bin/bash
# Quick GPU iteration: selected parity tests, then short C2 lines (default streams, and encode alone).
# Usage: tools/gpu_quick.sh <tag> [bench args...]
set -o pipefail
TAG=${1:-q}; shift || true
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_plan.py tests/test_gpu_fuzz.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_$TAG.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/pytest_$TAG.log | head -20; exit $rc; }
for mode in md5 nomd5; do
  extra=""; [ $mode = nomd5 ] && extra="--no-md5"
  timeout -k 10 200 python bench.py --no-cpu --no-curve --no-e2e --verify-streams 16 $extra "$@" > gpurun_out/q_${TAG}_$mode.json 2> gpurun_out/q_${TAG}_$mode.err || { echo FAIL $mode; tail -5 gpurun_out/q_${TAG}_$mode.err; exit 1; }
  python3 -c "import json;d=json.loads(open('gpurun_out/q_${TAG}_$mode.json').read().strip().splitlines()[-1]);print('$mode',d['value'],d['kernel_ms_per_step'],d['output_ok'])"
done
