#!/bin/bash
# r4s: which descriptor-store coalescing pays at C2: all (default build), no FrameDesc one-store
# (build_x), no SubDesc one-store (build_y), previous commit (build_ab); then WRITE_SIZE per variant
set -o pipefail
mkdir -p gpurun_out
AB_REPS=2 tools/ab.sh r4s "c2" all:- noframe:lib=zig-flac_amd/build_x nosub:lib=zig-flac_amd/build_y old:lib=zig-flac_amd/build_ab || exit 1
REPO=$(pwd)
cd /tmp && export TMPDIR=/tmp
for v in build build_x build_y build_ab; do
  FLACGPU_LIB=$REPO/zig-flac_amd/$v/libflacgpu.so timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $REPO/gpurun_out/r4s_w_$v -o pmc -- python3 $REPO/bench.py --frames 262144 --streams 16384 --steps 3 --warmup 1 --no-cpu --no-curve --no-e2e --no-sharded --configs= --verify-streams 4 > $REPO/gpurun_out/r4s_w_$v.log 2>&1 || { echo "pmc $v failed"; exit 1; }
  python3 -c "
import csv,glob,sys
v=[float(r['Counter_Value']) for f in glob.glob(sys.argv[1]+'/**/*counter_collection.csv',recursive=True) for r in csv.DictReader(open(f)) if 'k_analyze<2, 16, true' in r['Kernel_Name']]
print(sys.argv[2], 'analysis WRITE GB/launch %.3f'%(sum(v)/len(v)*1024/1e9))" $REPO/gpurun_out/r4s_w_$v $v
done
