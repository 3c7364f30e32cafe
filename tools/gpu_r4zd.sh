#!/bin/bash
# r4zd: end-to-end file batches (64 and 32 files from host memory) with the MD5 pool at 16 / 15 / 14
# workers (FLACGPU_MD5_THREADS; the pipeline's upload, download and caller threads share the cores)
set -o pipefail
mkdir -p gpurun_out
for rep in 1 2; do
  for t in 16 15 14; do
    out=gpurun_out/r4zd_t${t}_$rep.json
    FLACGPU_MD5_THREADS=$t timeout -k 10 300 python bench.py --steps 3 --warmup 1 --frames 16384 --configs= --no-cpu --no-curve \
      --no-sharded --verify-streams 4 --e2e-files 32,64 > $out 2> $out.err || { tail -5 $out.err; exit 1; }
    python3 -c "
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); e = d['end_to_end']
print('threads', sys.argv[2], 'rep', sys.argv[3], [(c['files'], c['batch']['value'], c['batch']['frac_of_md5_bound'], c['md5_pool_alone_ms']) for c in e['curve']])" $out $t $rep
  done
done
