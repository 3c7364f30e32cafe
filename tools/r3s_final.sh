#!/bin/bash
# r3s: the default line at the round-3 batch shape (131072 blocks/step as 16384 streams x 8) and its
# rocprofv3 trace + PMC (roofline.traffic of that workload).
set -o pipefail
mkdir -p gpurun_out
echo "bench (default line) ..."
timeout -k 10 900 python bench.py > gpurun_out/r3s_bench.json 2> gpurun_out/r3s_bench.err || { tail -5 gpurun_out/r3s_bench.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r3s_bench.json')); print('C2', d['value'], d['ms_per_step'], d['output_ok'], d['kernel_ms_per_step'], d['roofline']['frac'], d['roofline']['traffic'])"
echo "profile ..."
bash tools/profile.sh r3s_c2 c2 131072 16384 && head -12 profiles/r3s_c2_summary.md
