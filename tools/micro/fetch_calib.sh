#!/bin/bash
# FETCH_SIZE calibration for the encode kernels' access widths (tools/micro/fetch_micro.hip):
# plain run (timings), kernel trace + stats, then one FETCH_SIZE pass; joined by tools/fetch_calib.py
# into profiles/<tag>_fetch_calib.{json,md} (mirrored under gpurun_out/profiles/).
# Usage (GPU box, repo root): tools/micro/fetch_calib.sh <tag>
set -o pipefail
TAG=${1:-r4}
REPO=$(pwd)
OUT=$REPO/gpurun_out/fetch_$TAG
mkdir -p $OUT
BIN=$REPO/tools/micro/fetch_micro
timeout -k 10 120 $BIN 32768 3 > $OUT/run.jsonl || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o kt -- $BIN 32768 3 > $OUT/kt.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc1 -o pmc -- $BIN 32768 3 > $OUT/pmc1.log 2>&1 || exit 1
cd $REPO
python3 tools/micro/fetch_calib.py $OUT $TAG
