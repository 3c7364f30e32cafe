# A/B of library builds on the c2 bench: tools/exp_ab.sh <build dir>...
set -o pipefail
mkdir -p gpurun_out
for lib in "$@"; do
 for md in "" "--no-md5"; do
  FLACGPU_LIB=zig-flac_amd/$lib/libflacgpu.so timeout -k 10 200 python bench.py --no-cpu $md > gpurun_out/bench_ab.log 2>&1 || { tail -5 gpurun_out/bench_ab.log; exit 1; }
  tail -1 gpurun_out/bench_ab.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$lib $md', d['value'], d['ms_per_step'], d['kernel_ms_per_step'], d['output_ok'])"
 done
done
