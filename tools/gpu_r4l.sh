#!/bin/bash
# r4l: split-schedule parity + file tests, e2e (per-file vs batch), c4 A/B (just-in-time split
# tickets), c5 MD5 scheduling A/B -- all at the configs-block shape (65536 frames)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_file_host.py tests/test_golden.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r4l_parity.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; tail -2 gpurun_out/r4l_parity.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/r4l_parity.log | head; exit $rc; }
timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --configs= --no-sharded --no-cpu --no-curve > gpurun_out/r4l_e2e.json 2> gpurun_out/r4l_e2e.err || { echo "bench failed"; tail -5 gpurun_out/r4l_e2e.err; exit 1; }
python3 -c "
import json,sys; d=json.load(open(sys.argv[1])); e=d['end_to_end']
print('e2e', e['value'], e['mode'], e['files'], e['output_ok'])
for c in e['curve']: print(c['files'], c['value'], c['wall_ms'], c['md5_pool_alone_ms'], c['frames_alone_ms'], c['batch'])" gpurun_out/r4l_e2e.json
AB_REPS=2 AB_ARGS="--frames 65536" tools/ab.sh r4l "c4" base:- jit:FLACGPU_SPLIT_JIT=1 || exit 1
AB_REPS=1 AB_ARGS="--frames 65536" tools/ab.sh r4l "c5" base:- prio1:FLACGPU_MD5_PRIO=1 prio3:FLACGPU_MD5_PRIO=3 k2:FLACGPU_MD5_KERNEL=2 rsv:FLACGPU_MD5_RESERVE=1
timeout -k 10 900 bash tools/run_stamps.sh
