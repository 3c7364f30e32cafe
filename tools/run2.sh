set -o pipefail
mkdir -p gpurun_out
export FLACGPU_LIB=$PWD/zig-flac_amd/build_w2/libflacgpu.so
timeout -k 10 400 python -m pytest tests -m gpu -q -x > gpurun_out/pytest3.log 2>&1 || { echo PYTEST_FAIL; tail -30 gpurun_out/pytest3.log; exit 1; }
tail -2 gpurun_out/pytest3.log
for w in 2 3 4; do
  FLACGPU_LIB=$PWD/zig-flac_amd/build_w$w/libflacgpu.so timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu --no-md5 --verify > gpurun_out/bench_w$w.log 2>&1 || { echo BENCH_FAIL $w; tail -5 gpurun_out/bench_w$w.log; exit 1; }
  echo w$w; tail -1 gpurun_out/bench_w$w.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['kernel_ms_per_step'], d['output_ok'])"
done
for S in 1024 4096; do
  timeout -k 10 200 python bench.py --steps 5 --warmup 1 --no-cpu --streams $S > gpurun_out/bench_s$S.log 2>&1 || { echo BENCH_FAIL s$S; tail -5 gpurun_out/bench_s$S.log; exit 1; }
  echo s$S; tail -1 gpurun_out/bench_s$S.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['kernel_ms_per_step'], d['output_ok'])"
done
