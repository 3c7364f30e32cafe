#!/bin/bash
# r3n: evidence at HEAD -- GPU suite, the full default bench line (CPU baseline, stream curve,
# end-to-end curve, sharded stream), then one line per other BASELINE config with its CPU baselines.
set -o pipefail
mkdir -p gpurun_out
STEP=${1:-all}
if [ "$STEP" = all ] || [ "$STEP" = a ]; then
  timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r3n_pytest_gpu.log 2>&1
  rc=$?; tail -2 gpurun_out/r3n_pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
  echo "bench (default line) ..."
  timeout -k 10 900 python bench.py > gpurun_out/r3n_bench.json 2> gpurun_out/r3n_bench.err || { tail -5 gpurun_out/r3n_bench.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r3n_bench.json')); print('C2', d['value'], d['ms_per_step'], d['output_ok'], d['kernel_ms_per_step'], (d.get('end_to_end') or {}).get('value'), (d.get('cpu_baseline') or {}).get('value'))"
fi
if [ "$STEP" = all ] || [ "$STEP" = b ]; then
  for C in c3 c4 c5; do
    echo "bench $C ..."
    timeout -k 10 600 python bench.py --config $C --steps 8 --warmup 2 --no-curve --no-e2e > gpurun_out/r3n_cfg_$C.json 2> gpurun_out/r3n_cfg_$C.err || { tail -5 gpurun_out/r3n_cfg_$C.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['output_ok'], d['kernel_ms_per_step'], (d.get('cpu_baseline') or {}).get('value'))" gpurun_out/r3n_cfg_$C.json $C
  done
fi
if [ "$STEP" = c ]; then
  for C in c3 c4 c5; do
    echo "profile $C ..."
    bash tools/profile.sh r3n_$C $C 65536 16384 || { echo PROFILE_FAIL $C; exit 1; }
    head -10 profiles/r3n_${C}_summary.md
  done
fi
