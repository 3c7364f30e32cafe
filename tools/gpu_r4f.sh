#!/bin/bash
# r4f: parity (k_ana1 variants, k_analyze power-of-two Rice search), same-box A/B vs the previous
# build, then the stream curve (MD5 engine picked per plan) and the end-to-end curve
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_plan.py -q --timeout 120 --timeout-method thread > gpurun_out/r4f_parity.log 2>&1
rc=$?
echo "parity rc=$rc"; tail -3 gpurun_out/r4f_parity.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/r4f_parity.log | head; exit $rc; }
AB_REPS=2 tools/ab.sh r4f "c2" new:- old:lib=zig-flac_amd/build_ab0 || exit 1
timeout -k 10 400 python -u bench.py --steps 3 --warmup 1 --configs= --no-sharded --no-cpu > gpurun_out/r4f_bench.json 2> gpurun_out/r4f_bench.err
rc=$?; echo "bench rc=$rc"; tail -3 gpurun_out/r4f_bench.err; exit $rc
