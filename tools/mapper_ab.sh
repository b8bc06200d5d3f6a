#!/bin/bash
# Mapper-leg A/B (configs[3], WF frozen + per-neighbour): bench.py's mapper legs only, once per
# environment setting given as arguments, alternating twice.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for rep in 1 2; do
for setting in "$@"; do
    env $setting timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-tracker --no-mesher \
        --no-map-update --no-process-frame --no-nwf-leg --no-slam --no-input-order > /tmp/mab.json 2> /tmp/mab.err \
        || { tail -5 /tmp/mab.err; exit 1; }
    python3 -c "
import json,sys;d=json.loads(open('/tmp/mab.json').read().strip().splitlines()[-1])
m=d.get('mapper',{});n=d.get('mapper_nwf',{})
print('$setting', 'mapper', round(m.get('value',0),1), 'it/s', 'nwf', round(n.get('value',0),1), 'it/s', flush=True)"
done
done
