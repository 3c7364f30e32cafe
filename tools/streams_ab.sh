#!/bin/bash
# Default C2 bench at several stream counts (plus the encode alone), short lines.
set -o pipefail
mkdir -p gpurun_out
for s in 16384 32768 65536; do
  timeout -k 10 200 python bench.py --streams $s --no-cpu --no-curve --no-e2e --verify-streams 8 > gpurun_out/sab_$s.json 2> gpurun_out/sab_$s.err || { echo FAIL $s; tail -5 gpurun_out/sab_$s.err; exit 1; }
  python3 -c "import json;d=json.loads(open('gpurun_out/sab_$s.json').read().strip().splitlines()[-1]);print($s,d['value'],d['kernel_ms_per_step'],d['output_ok'])"
done
timeout -k 10 200 python bench.py --no-md5 --no-cpu --no-curve --no-e2e --verify-streams 8 > gpurun_out/sab_nomd5.json 2> gpurun_out/sab_nomd5.err || { echo FAIL nomd5; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/sab_nomd5.json').read().strip().splitlines()[-1]);print('nomd5',d['value'],d['kernel_ms_per_step'],d['output_ok'])"
