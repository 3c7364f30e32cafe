set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests -m gpu -q -x > gpurun_out/pytest4.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/pytest4.log; exit 1; }
tail -2 gpurun_out/pytest4.log
timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu --no-md5 --verify > gpurun_out/bench_n.log 2>&1 || { echo BENCH_FAIL; tail -5 gpurun_out/bench_n.log; exit 1; }
tail -1 gpurun_out/bench_n.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['kernel_ms_per_step'], d['output_ok'])"
for v in st st128; do
 echo == $v
 FLACGPU_LIB=$PWD/zig-flac_amd/build_$v/libflacgpu.so timeout -k 10 200 python tools/stamps.py 2>&1 | grep -v amdgpu.ids
done
