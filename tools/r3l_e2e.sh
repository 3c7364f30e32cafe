#!/bin/bash
# r3l: end-to-end curve with the host hashing pool (default) vs one plain MD5 chain per file
# (FLACGPU_MD5_THREADS=-1), same box; then the file-path GPU tests.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_file_host.py tests/test_gpu_fused.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r3l_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/r3l_pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/r3l_pytest.log | head; exit $rc; }
ARGS="--steps 3 --warmup 1 --no-cpu --no-curve --no-sharded --verify-streams 2"
for M in -1 0 16 8; do
  out=gpurun_out/r3l_e2e_t$M.json
  FLACGPU_MD5_THREADS=$M timeout -k 10 400 python bench.py $ARGS > $out 2> $out.err || { echo "FAIL $M"; tail -5 $out.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1]))['end_to_end']; print(sys.argv[2], [(c['files'], c['value'], c['wall_ms']) for c in d['curve']], d['bounds_msamples_per_s'], d['output_ok'])" $out t$M
done
