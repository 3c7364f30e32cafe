#!/bin/bash
# r4z: final check of the committed tree -- the whole GPU suite, smoke(), and the default bench line
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r4z_pytest.log 2>&1 || { tail -30 gpurun_out/r4z_pytest.log; exit 1; }
tail -3 gpurun_out/r4z_pytest.log
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r4z_smoke.log 2>&1 || { tail -30 gpurun_out/r4z_smoke.log; exit 1; }
tail -1 gpurun_out/r4z_smoke.log
timeout -k 10 300 python -u bench.py > gpurun_out/r4z_bench.json 2> gpurun_out/r4z_bench.err || { tail -30 gpurun_out/r4z_bench.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/r4z_bench.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['roofline']['frac'], [(c.get('config'), c.get('value')) for c in d.get('configs', [])])"
