#!/bin/bash
# A/B of the overlapped encode schedule (fg_api.cpp encode_core) on the default C2 bench line:
# parity of the plan path with the schedule forced on small plans, then bench lines per setting.
# Usage (GPU box, repo root): tools/ab_ovl.sh <tag> [bench args...]
set -o pipefail
TAG=${1:-ovl}; shift || true
mkdir -p gpurun_out
FLACGPU_OVERLAP=4 FLACGPU_OVL_MIN=8 timeout -k 10 600 python -u -m pytest tests/test_gpu_plan.py tests/test_gpu_parity.py \
  -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_${TAG}_ovl.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_${TAG}_ovl.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/pytest_${TAG}_ovl.log | head -20; exit $rc; }
ARGS="--steps 20 --warmup 3 --no-cpu --no-curve --no-e2e --no-sharded --verify-streams 8 $*"
run() {
  local name=$1; shift
  env "$@" timeout -k 10 200 python bench.py $ARGS > gpurun_out/ab_${TAG}_$name.json 2> gpurun_out/ab_${TAG}_$name.err ||
    { echo "FAIL $name"; tail -5 gpurun_out/ab_${TAG}_$name.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'], d['output_ok'], d['kernel_ms_per_step'])" gpurun_out/ab_${TAG}_$name.json $name
}
for rep in 1 2; do
  run base$rep FLACGPU_OVERLAP=0 || exit 1
  run k4_22_$rep FLACGPU_OVERLAP=4 || exit 1
  run k8_22_$rep FLACGPU_OVERLAP=8 || exit 1
done
run k8_31 FLACGPU_OVERLAP=8 FLACGPU_OVL_ANA=3 FLACGPU_OVL_PACK=1 || exit 1
run k8_13 FLACGPU_OVERLAP=8 FLACGPU_OVL_ANA=1 FLACGPU_OVL_PACK=3 || exit 1
run k16_22 FLACGPU_OVERLAP=16 || exit 1
run k8_40 FLACGPU_OVERLAP=8 FLACGPU_OVL_ANA=0 FLACGPU_OVL_PACK=0 || exit 1
