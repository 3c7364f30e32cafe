#!/bin/bash
# LPC parity tests then c3/c5 bench lines (new k_ana4 vs FLACGPU_ANA4=0).
set -o pipefail
mkdir -p gpurun_out
bash tools/gpu_tests.sh lpc tests/test_gpu_lpc.py tests/test_gpu_plan.py || exit 1
for C in c3 c5; do
  for A in 1 0; do
    FLACGPU_ANA4=$A timeout -k 10 200 python bench.py --config $C --steps 5 --warmup 2 --no-cpu --no-curve --no-e2e --verify-streams 8 > gpurun_out/lpcab_${C}_$A.json 2> gpurun_out/lpcab_${C}_$A.err || { echo "FAIL $C $A"; tail -3 gpurun_out/lpcab_${C}_$A.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], 'ana4', sys.argv[3], d['value'], d['output_ok'], d['kernel_ms_per_step'])" gpurun_out/lpcab_${C}_$A.json $C $A
  done
done
