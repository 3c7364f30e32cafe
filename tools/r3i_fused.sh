#!/bin/bash
# r3i: the fused single-pass encode (FLACGPU_FUSED=1): its tests, the whole GPU suite with it on,
# the suite at defaults, then same-box bench A/B of the two schedules on the C2 line.
set -o pipefail
mkdir -p gpurun_out
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
timeout -k 10 300 $T tests/test_gpu_fused.py > gpurun_out/r3i_fused_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r3i_fused_tests.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/r3i_fused_tests.log | head -20; exit $rc; }
FLACGPU_FUSED=1 timeout -k 10 400 $T tests -m gpu > gpurun_out/r3i_pytest_gpu_fused.log 2>&1
rc=$?; tail -3 gpurun_out/r3i_pytest_gpu_fused.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/r3i_pytest_gpu_fused.log | head -20; exit $rc; }
ARGS="--steps 20 --warmup 3 --no-cpu --no-curve --no-e2e --no-sharded --verify-streams 8"
for rep in 1 2; do
  for F in 0 1; do
    out=gpurun_out/ab_r3i_f${F}_$rep.json
    FLACGPU_FUSED=$F timeout -k 10 200 python bench.py $ARGS > $out 2> $out.err || { echo "FAIL f$F"; tail -5 $out.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['ms_per_step'], d['output_ok'], d['kernel_ms_per_step'])" $out f$F
  done
done
