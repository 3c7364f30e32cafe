#!/bin/bash
# Round-2 evidence run: keyed C2 profile at the bench default (16384 streams), then the
# default bench line (reads that PMC for roofline.traffic).  GPU box, repo root.
set -o pipefail
mkdir -p gpurun_out
bash tools/profile.sh r2c_c2 c2 65536 16384 || { echo PROFILE_FAIL; exit 1; }
cat profiles/r2c_c2_summary.md
timeout -k 10 600 python -u bench.py > gpurun_out/bench_r2c.json 2> gpurun_out/bench_r2c.err || { echo BENCH_FAIL; tail -20 gpurun_out/bench_r2c.err; exit 1; }
tail -1 gpurun_out/bench_r2c.json | cut -c1-1500
