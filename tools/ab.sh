#!/bin/bash
# The one A/B harness: same-box bench.py lines for every (config, variant), variants alternating
# within each rep, one summary row per run.
# Usage (GPU box, repo root):
#   tools/ab.sh <tag> "<configs>" <variant>...
#     config  : c2 (the headline line) | c3 | c4 | c5
#     variant : name:SPEC, SPEC = comma-separated ENV=VALUE assignments (FLACGPU_* knobs), or
#               lib=<build dir> for another libflacgpu.so build (FLACGPU_LIB), or "-" for none
#   e.g. tools/ab.sh ana1 "c2 c3" one:FLACGPU_ANA1=1 four:FLACGPU_ANA1=0
# Env: AB_REPS (2), AB_STEPS (20; 10 for c3-c5), AB_ARGS (extra bench.py arguments)
# Rows: tag config variant rep MS/s ms/step output_ok kernel_ms/step -> gpurun_out/ab_<tag>.txt
# (JSON lines in gpurun_out/ab_<tag>_<config>_<variant>_<rep>.json)
set -o pipefail
TAG=$1; CFGS=$2; shift 2
mkdir -p gpurun_out
SUM=gpurun_out/ab_$TAG.txt
REPS=${AB_REPS:-2}
for cfg in $CFGS; do
  CA="--configs="; ST=${AB_STEPS:-20}
  if [ "$cfg" != c2 ]; then CA="--config $cfg"; ST=${AB_STEPS:-10}; fi
  for rep in $(seq $REPS); do
    for V in "$@"; do
      name=${V%%:*}; spec=${V#*:}
      envs=()
      if [ "$spec" != "-" ]; then
        IFS=',' read -ra kv <<< "$spec"
        for a in "${kv[@]}"; do
          case $a in
            lib=*) envs+=("FLACGPU_LIB=$PWD/${a#lib=}/libflacgpu.so") ;;
            *) envs+=("$a") ;;
          esac
        done
      fi
      out=gpurun_out/ab_${TAG}_${cfg}_${name}_$rep.json
      eval env "${envs[@]}" timeout -k 10 300 python bench.py $CA --steps $ST --warmup 3 --no-cpu --no-curve \
        --no-e2e --no-sharded --verify-streams 8 $AB_ARGS > $out 2> $out.err || { echo "FAIL $cfg $name"; tail -5 $out.err; exit 1; }
      python3 -c "
import json, sys
d = json.load(open(sys.argv[1]))
print(*sys.argv[2:], d['value'], d['ms_per_step'], d['output_ok'], json.dumps(d['kernel_ms_per_step']))" \
        $out $TAG $cfg $name $rep | tee -a $SUM
    done
  done
done
