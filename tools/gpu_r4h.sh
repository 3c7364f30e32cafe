#!/bin/bash
# r4h: e2e with blocking-sync host waits vs spinning (FLACGPU_SPIN_SYNC=1), same box
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_file_host.py tests/test_golden.py -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/r4h_parity.log 2>&1
rc=$?; echo "parity rc=$rc"; tail -2 gpurun_out/r4h_parity.log; [ $rc -eq 0 ] || exit $rc
for v in block spin block2; do
  E=""; [ $v = spin ] && E="FLACGPU_SPIN_SYNC=1"
  env $E timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --configs= --no-sharded --no-cpu --no-curve > gpurun_out/r4h_$v.json 2> gpurun_out/r4h_$v.err || { echo "bench $v failed"; tail -5 gpurun_out/r4h_$v.err; exit 1; }
  python3 -c "
import json,sys; d=json.load(open(sys.argv[1])); e=d['end_to_end']
print(sys.argv[2], [(c['files'], c['value'], c['wall_ms'], c['md5_pool_alone_ms'], c['frames_alone_ms'], c['frac_of_bound']) for c in e['curve']])" gpurun_out/r4h_$v.json $v
done
