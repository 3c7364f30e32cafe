#!/bin/bash
# r3v: c4 split pack with 4 waves per subframe of the half (16 samples per lane) in one
# double-buffered 1024-thread workgroup per CU (FLACGPU_PSPLIT_WPS=4) against 2 waves per subframe
# in two single-buffered 512-thread workgroups: GPU suite with the knob on, then the c4 line, 3 reps
set -o pipefail
mkdir -p gpurun_out
FLACGPU_PSPLIT_WPS=4 timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r3v_pytest_gpu.log 2>&1 || { tail -30 gpurun_out/r3v_pytest_gpu.log; exit 1; }
tail -1 gpurun_out/r3v_pytest_gpu.log
for rep in 1 2 3; do
  for W in 2 4; do
    out=gpurun_out/r3v_c4_w${W}_$rep.json
    FLACGPU_PSPLIT_WPS=$W timeout -k 10 300 python bench.py --config c4 --frames 65536 --steps 10 --warmup 2 --no-cpu --no-curve --no-e2e --no-sharded --verify-streams 16 > $out 2> $out.err || { echo "FAIL $W"; tail -5 $out.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['ms_per_step'], d['output_ok'], d['kernel_ms_per_step'])" $out "c4:wps$W"
  done
done
