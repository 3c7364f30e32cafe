#!/bin/bash
# Kernel trace + stats of short bench runs (one per config).  Usage: tools/ktrace.sh <tag> "<configs>"
set -o pipefail
TAG=$1; CFGS=$2
REPO=$(pwd); mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
for C in $CFGS; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $REPO/gpurun_out/kt_${TAG}_$C -o kt -- python3 $REPO/bench.py --config $C --steps 5 --warmup 2 --no-cpu --no-curve --no-e2e --verify-streams 4 > $REPO/gpurun_out/kt_${TAG}_$C.log 2>&1 || { echo FAIL $C; tail -5 $REPO/gpurun_out/kt_${TAG}_$C.log; exit 1; }
  echo "== $C"; python3 -c "
import csv,sys
for r in csv.DictReader(open(sys.argv[1])):
    if float(r['TotalDurationNs'])>1e6: print('  %-60s %5s %10.1f us' % (r['Name'][:60], r['Calls'], float(r['AverageNs'])/1e3))
" $REPO/gpurun_out/kt_${TAG}_$C/kt_kernel_stats.csv
done
