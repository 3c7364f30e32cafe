#!/bin/bash
# r4ze: MD5 pool with up to eight chains per worker (in-tree build) against HEAD's four (build_ab):
# GPU suite on the new build, then end-to-end batches of 64 / 72 files at 16 and 15 workers
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r4ze_pytest.log 2>&1 || { tail -30 gpurun_out/r4ze_pytest.log; exit 1; }
tail -2 gpurun_out/r4ze_pytest.log
for rep in 1 2; do
  for t in 16 15; do
    for v in base new; do
      lib=""; [ $v = base ] && lib="FLACGPU_LIB=$PWD/zig-flac_amd/build_ab/libflacgpu.so"
      out=gpurun_out/r4ze_${v}_t${t}_$rep.json
      env $lib FLACGPU_MD5_THREADS=$t timeout -k 10 300 python bench.py --steps 3 --warmup 1 --frames 16384 --configs= --no-cpu --no-curve \
        --no-sharded --verify-streams 4 --e2e-files 64,72 > $out 2> $out.err || { tail -5 $out.err; exit 1; }
      python3 -c "
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); e = d['end_to_end']
print(*sys.argv[2:], [(c['files'], c['batch']['value'], c['batch']['frac_of_md5_bound'], c['md5_pool_alone_ms'], c['batch']['wall_ms']) for c in e['curve']])" $out $v threads=$t rep=$rep
    done
  done
done
