#!/bin/bash
# A/B of the split analysis's per-XCD item queues (FLACGPU_XCD_QUEUE) on the c4 bench line:
# bench lines alternating, then one FETCH_SIZE pass per setting (analysis FETCH per launch).
# Usage (GPU box, repo root): tools/ab_xcd.sh <tag> [lib dir]
set -o pipefail
TAG=${1:-xcd}; LIB=${2:-zig-flac_amd/build}
mkdir -p gpurun_out
export FLACGPU_LIB=$PWD/$LIB/libflacgpu.so
ARGS="--config c4 --steps 10 --warmup 2 --no-cpu --no-curve --no-e2e --no-sharded --verify-streams 8"
for rep in 1 2; do
  for XQ in 0 1; do
    out=gpurun_out/ab_${TAG}_xq${XQ}_$rep.json
    FLACGPU_XCD_QUEUE=$XQ timeout -k 10 200 python bench.py $ARGS > $out 2> $out.err || { echo "FAIL xq$XQ"; tail -5 $out.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['ms_per_step'], d['output_ok'], d['kernel_ms_per_step'])" $out xq$XQ
  done
done
REPO=$PWD
cd /tmp && export TMPDIR=/tmp
for XQ in 0 1; do
  D=$REPO/gpurun_out/prof_${TAG}_xq$XQ
  mkdir -p $D
  FLACGPU_XCD_QUEUE=$XQ timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $D/pmc1 -o pmc -- python3 $REPO/bench.py --config c4 --steps 3 --warmup 1 --no-cpu --no-curve --no-e2e --no-sharded --verify-streams 2 > $D/pmc1.log 2>&1 || { echo "PMC xq$XQ failed"; exit 1; }
  python3 - $D/pmc1 $XQ <<'EOF'
import csv, glob, sys, collections
v = collections.defaultdict(list)
for f in glob.glob(sys.argv[1] + "/**/pmc_counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        n = r["Kernel_Name"]
        k = "analyze" if "k_analyze" in n else "pack" if "k_pack" in n else "md5" if "md5" in n else None
        if k and r["Counter_Name"] == "FETCH_SIZE":
            v[k].append(float(r["Counter_Value"]))
for k, xs in sorted(v.items()):
    print("xq%s %s FETCH GB/launch (x1024 x2): %.3f  (n=%d)" % (sys.argv[2], k, sum(xs) / len(xs) * 2048 / 1e9, len(xs)))
EOF
done
