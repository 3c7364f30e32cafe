#!/bin/bash
# r3w: HEAD validation -- GPU suite, smoke, and the default bench line (CPU baseline with the
# table CRC-16, unrolled MD5 and per-order residual loops of the oracle port)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r3w_pytest_gpu.log 2>&1 || { tail -30 gpurun_out/r3w_pytest_gpu.log; exit 1; }
tail -1 gpurun_out/r3w_pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3w_smoke.log 2>&1 || { tail -20 gpurun_out/r3w_smoke.log; exit 1; }
tail -2 gpurun_out/r3w_smoke.log
timeout -k 10 900 python bench.py > gpurun_out/r3w_bench.json 2> gpurun_out/r3w_bench.err || { tail -5 gpurun_out/r3w_bench.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r3w_bench.json')); print('C2', d['value'], d['ms_per_step'], d['output_ok'], d['kernel_ms_per_step'], d['roofline']['frac'], d['roofline']['traffic']); c=d['cpu_baseline']; print('CPU', c['value'], c['single_core'], c['single_socket_estimate'])"
for C in c3 c4 c5; do
  timeout -k 10 600 python bench.py --config $C --frames 65536 --no-curve --no-e2e --no-sharded > gpurun_out/r3w_cfg_$C.json 2> gpurun_out/r3w_cfg_$C.err || { tail -5 gpurun_out/r3w_cfg_$C.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); c=d['cpu_baseline']; print(sys.argv[2], d['value'], d['output_ok'], 'CPU', c['value'], c['single_core']['value'], (c.get('fixed_only') or {}).get('value'), c['single_socket_estimate'])" gpurun_out/r3w_cfg_$C.json $C
done
