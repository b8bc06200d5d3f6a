#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
timeout -k 10 600 python -m pytest tests -m gpu -q -x > gpurun_out/gpu_tests.log 2>&1; tail -1 gpurun_out/gpu_tests.log
for rep in 1 2; do for sp in 1 0; do for nwf in "" "--nwf"; do
PIN_QUERY_SPLIT=$sp timeout -k 10 200 python bench.py --no-mapper --no-cpu-baseline --no-tracker --no-mesher $nwf > gpurun_out/t.json 2>/dev/null || exit 1
python3 -c "import json;d=json.load(open('gpurun_out/t.json'));print('split=$sp $nwf', round(d['value']/1e9,3), 'Gq/s', round(d['ms_per_step']*1e3,1), 'us/step kernel', round(d['roofline']['kernel_ms']*1e3,1))"
done; done; done
