#!/bin/bash
# r4zf: what binds the 64-file batch -- flacgpu_encode_files with its MD5s (default) against the
# same call with FLACGPU_FILES_MD5=0 (the GPU / PCIe schedule alone), 16 and 14 pool workers
set -o pipefail
mkdir -p gpurun_out
for rep in 1 2; do
  for v in "md5 16" "nomd5 16" "md5 14"; do
    set -- $v
    extra=""; [ $1 = nomd5 ] && extra="FLACGPU_FILES_MD5=0"
    out=gpurun_out/r4zf_$1_t$2_$rep.json
    env $extra FLACGPU_MD5_THREADS=$2 timeout -k 10 300 python bench.py --steps 3 --warmup 1 --frames 16384 --configs= --no-cpu --no-curve \
      --no-sharded --verify-streams 4 --e2e-files 32,64 > $out 2> $out.err || { tail -5 $out.err; exit 1; }
    python3 -c "
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); e = d['end_to_end']
print(*sys.argv[2:], [(c['files'], c['batch']['value'], c['batch']['wall_ms'], c['md5_pool_alone_ms'], c['frames_alone_ms']) for c in e['curve']])" $out $1 threads=$2 rep=$rep
  done
done
