#!/bin/bash
# r4j: file-level GPU tests (flacgpu_encode_files), then the e2e curve (per-file vs batch)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_file_host.py tests/test_golden.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r4j_parity.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; tail -2 gpurun_out/r4j_parity.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/r4j_parity.log | head; exit $rc; }
timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --configs= --no-sharded --no-cpu --no-curve > gpurun_out/r4j.json 2> gpurun_out/r4j.err || { echo "bench failed"; tail -5 gpurun_out/r4j.err; exit 1; }
python3 -c "
import json,sys; d=json.load(open(sys.argv[1])); e=d['end_to_end']
print(e['value'], e['mode'], e['files'], e['output_ok'])
for c in e['curve']: print(c['files'], c['value'], c['wall_ms'], c['md5_pool_alone_ms'], c['frames_alone_ms'], c['batch'])" gpurun_out/r4j.json
