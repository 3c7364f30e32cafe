#!/bin/bash
# r4i: GPU tests; e2e blocking-sync host waits vs spinning (FLACGPU_SPIN_SYNC=1); c4 pack split
# on per-XCD queues vs the global ticket (FLACGPU_PACK_XCDQ=0)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r4i_parity.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; tail -2 gpurun_out/r4i_parity.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/r4i_parity.log | head; exit $rc; }
for v in block spin block2; do
  E=""; [ $v = spin ] && E="FLACGPU_SPIN_SYNC=1"
  env $E timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --configs= --no-sharded --no-cpu --no-curve > gpurun_out/r4i_$v.json 2> gpurun_out/r4i_$v.err || { echo "bench $v failed"; tail -5 gpurun_out/r4i_$v.err; exit 1; }
  python3 -c "
import json,sys; d=json.load(open(sys.argv[1])); e=d['end_to_end']
print(sys.argv[2], [(c['files'], c['value'], c['wall_ms'], c['md5_pool_alone_ms'], c['frames_alone_ms'], c['frac_of_bound']) for c in e['curve']])" gpurun_out/r4i_$v.json $v
done
AB_REPS=2 tools/ab.sh r4i "c4" xq:- noxq:FLACGPU_PACK_XCDQ=0
