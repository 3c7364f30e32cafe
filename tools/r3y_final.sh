#!/bin/bash
# r3y: the default line at 262144 blocks per step (16384 streams x 16): rocprofv3 trace + PMC of that
# workload first (roofline.traffic), then the full default bench line
set -o pipefail
mkdir -p gpurun_out
bash tools/profile.sh r3y_c2 c2 262144 16384 || exit 1
head -12 profiles/r3y_c2_summary.md
timeout -k 10 900 python bench.py > gpurun_out/r3y_bench.json 2> gpurun_out/r3y_bench.err || { tail -5 gpurun_out/r3y_bench.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r3y_bench.json')); print('C2', d['value'], d['ms_per_step'], d['output_ok'], d['kernel_ms_per_step'], d['roofline']['frac'], d['roofline']['traffic']); c=d['cpu_baseline']; print('CPU', c['value'], c['single_core']['value'], c['single_socket_estimate']); print([(x['streams'], x['value']) for x in d['stream_curve']])"
