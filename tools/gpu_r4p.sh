#!/bin/bash
# r4p: smoke, the default bench line (timed), the C2 profile at the headline shape
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4p_smoke.log 2>&1 || { echo smoke failed; tail -5 gpurun_out/r4p_smoke.log; exit 1; }
echo smoke ok
s=$(date +%s)
timeout -k 10 600 python -u bench.py > gpurun_out/r4p_bench.json 2> gpurun_out/r4p_bench.err || { echo "bench failed"; tail -5 gpurun_out/r4p_bench.err; exit 1; }
echo "bench wall $(( $(date +%s) - s )) s"
python3 -c "
import json,sys; d=json.load(open(sys.argv[1]))
print(d['value'], d['ms_per_step'], d['output_ok'], d['kernel_ms_per_step'])
print({k: d['roofline'][k] for k in ('bound','frac','step_issue_frac','traffic')})
for c in d.get('configs', []): print(c['config'], c['value'], c['ms_per_step'], c['output_ok'], c['kernel_ms_per_step'])
print('e2e', d['end_to_end']['value'], d['end_to_end']['mode'])
print('cpu', d['cpu_baseline']['value'])" gpurun_out/r4p_bench.json
tools/profile.sh r4p_c2 c2 262144 16384 > gpurun_out/r4p_prof.log 2>&1 || { echo profile failed; tail -5 gpurun_out/r4p_prof.log; exit 1; }
head -12 profiles/r4p_c2_summary.md
