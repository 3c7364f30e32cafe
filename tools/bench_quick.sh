set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu --verify > gpurun_out/bench_prio.log 2>&1 || { echo BENCH_FAIL; tail -5 gpurun_out/bench_prio.log; exit 1; }
tail -1 gpurun_out/bench_prio.log
