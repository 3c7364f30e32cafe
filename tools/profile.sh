#!/bin/bash
# rocprofv3 passes over bench.py (run on the GPU box from the repo root).
# Usage: tools/profile.sh <tag> <config> <frames> <streams> [bench args...]
# Writes gpurun_out/prof_<tag>/...: kernel trace + stats first, then PMC passes
# (one counter group per pass, never combined with tracing domains), then
# profiles/<tag>_summary.md + profiles/<tag>_pmc.json via tools/pmc_summary.py,
# keyed by the bench workload "<config>:<frames>x<streams>".
set -e
TAG=${1:-r2}; shift || true
CFG=${1:-c2}; shift || true
FRAMES=${1:-65536}; shift || true
STREAMS=${1:-16384}; shift || true
ARGS="--config $CFG --frames $FRAMES --streams $STREAMS --steps 5 --warmup 2 --no-cpu --no-curve --no-e2e --no-sharded --configs= --verify-streams 4 $@"
REPO=$(pwd)
OUT=$REPO/gpurun_out/prof_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o kt -- python3 $REPO/bench.py $ARGS > $OUT/kt.log 2>&1
i=0
for PMC in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES" "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 180 rocprofv3 --pmc $PMC --output-format csv -d $OUT/pmc$i -o pmc -- python3 $REPO/bench.py $ARGS > $OUT/pmc$i.log 2>&1 || { echo "PMC pass $i ($PMC) failed: no further GPU passes"; break; }
done
cd $REPO
KEY="$CFG:${FRAMES}x${STREAMS}"  # bench.py workload_key
[ "${FLACGPU_FUSED:-0}" = 1 ] && KEY="$KEY+fused"
case "${FLACGPU_ANA1:-0}" in 1|2) [ "$CFG" = c2 ] && KEY="$KEY+ana1v$FLACGPU_ANA1" ;; esac
python3 tools/pmc_summary.py $OUT $TAG $FRAMES "$KEY"
cp $OUT/kt/kt_kernel_stats.csv profiles/${TAG}_kernel_stats.csv
# profiles/ does not travel back from the GPU box: mirror the summaries under gpurun_out/
mkdir -p $REPO/gpurun_out/profiles && cp profiles/${TAG}_* $REPO/gpurun_out/profiles/
