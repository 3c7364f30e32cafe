#!/bin/bash
# r4v: the final state after the LDS job ring: GPU tests, smoke, profiles of every config at its bench workload
# (so the line's roofline.traffic / step_issue_frac come from this code), then the default bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r4v_parity.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; tail -2 gpurun_out/r4v_parity.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/r4v_parity.log | head; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4v_smoke.log 2>&1 || { echo smoke failed; tail -5 gpurun_out/r4v_smoke.log; exit 1; }
echo smoke ok
tools/profile.sh r4v_c2 c2 262144 16384 > gpurun_out/r4v_prof_c2.log 2>&1 || { echo profile c2 failed; exit 1; }
for c in c3 c4 c5; do tools/profile.sh r4v_$c $c 65536 16384 > gpurun_out/r4v_prof_$c.log 2>&1 || { echo profile $c failed; exit 1; }; done
s=$(date +%s)
timeout -k 10 600 python -u bench.py > gpurun_out/r4v_bench.json 2> gpurun_out/r4v_bench.err || { echo "bench failed"; tail -5 gpurun_out/r4v_bench.err; exit 1; }
echo "bench wall $(( $(date +%s) - s )) s"
python3 -c "
import json,sys; d=json.load(open(sys.argv[1]))
print(d['value'], d['ms_per_step'], d['output_ok'], d['kernel_ms_per_step'])
print({k: d['roofline'].get(k) for k in ('bound','frac','step_issue_frac','traffic','traffic_source')})
for c in d.get('configs', []): print(c['config'], c['value'], c['ms_per_step'], c['output_ok'], c['kernel_ms_per_step'], c['roofline'].get('step_issue_frac'))
e=d['end_to_end']; print('e2e', e['value'], e['mode'], e['files'])
print('curve', [(c['streams'], c['md5_engine'], c['value']) for c in d['stream_curve']])
print('cpu', d['cpu_baseline']['value'], d.get('sharded_stream', {}).get('value') if isinstance(d.get('sharded_stream'), dict) else None)" gpurun_out/r4v_bench.json
