#!/bin/bash
# r4g: plan tests (host MD5 engine vs device state), FETCH_SIZE calibration, curve + e2e bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_plan.py -q --timeout 120 --timeout-method thread > gpurun_out/r4g_parity.log 2>&1
rc=$?
echo "parity rc=$rc"; tail -3 gpurun_out/r4g_parity.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/r4g_parity.log | head; exit $rc; }
tools/fetch_calib.sh r4g || { echo "fetch calib failed"; exit 1; }
timeout -k 10 400 python -u bench.py --steps 3 --warmup 1 --configs= --no-sharded --no-cpu > gpurun_out/r4g_bench.json 2> gpurun_out/r4g_bench.err
rc=$?; echo "bench rc=$rc"; tail -3 gpurun_out/r4g_bench.err; exit $rc
