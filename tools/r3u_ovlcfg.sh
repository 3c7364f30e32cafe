#!/bin/bash
# r3u: overlapped schedule (FLACGPU_OVERLAP=4: analysis of range i+1 beside scan + pack of range i) at
# c3 / c4 / c5, where the pack is a larger share of the step than at C2 (same box, 2 reps)
set -o pipefail
mkdir -p gpurun_out
F=${R3U_FRAMES:-65536}
for rep in 1 2; do
  for C in c4 c3 c5; do
    for V in 0:2:2 4:2:2 4:1:1; do
      IFS=: read OV OA OP <<< "$V"
      out=gpurun_out/r3u_${C}_ov${OV}_${OA}${OP}_$rep.json
      FLACGPU_OVERLAP=$OV FLACGPU_OVL_ANA=$OA FLACGPU_OVL_PACK=$OP timeout -k 10 300 python bench.py --config $C --frames $F --steps 10 --warmup 2 --no-cpu --no-curve --no-e2e --no-sharded --verify-streams 8 > $out 2> $out.err || { echo "FAIL $C $OV"; tail -5 $out.err; exit 1; }
      python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['ms_per_step'], d['output_ok'], d['kernel_ms_per_step'])" $out "$C:ov$V"
    done
  done
done
