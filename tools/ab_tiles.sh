#!/bin/bash
# tiles on/off, alternating, same box
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for rep in 1 2; do for t in 1 0; do
PIN_QUERY_TILES=$t timeout -k 10 200 python bench.py --no-mapper --no-cpu-baseline > gpurun_out/t.json 2>/dev/null || exit 1
python3 -c "import json;d=json.load(open('gpurun_out/t.json'));print('tiles=$t', round(d['value']/1e9,3), 'Gq/s', round(d['ms_per_step']*1e3,1), 'us/step kernel', round(d['roofline']['kernel_ms']*1e3,1))"
done; done
