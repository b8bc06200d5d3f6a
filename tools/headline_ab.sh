#!/bin/bash
# Headline A/B: bench.py's headline leg only, once per environment setting given as arguments,
# alternating three times; prints q/s and the kernel's HIP-event time.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for rep in 1 2 3; do
for setting in "$@"; do
    env $setting timeout -k 10 300 python3 bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-mapper --no-tracker \
        --no-mesher --no-map-update --no-process-frame --no-nwf-leg --no-slam --no-input-order > /tmp/hab.json 2> /tmp/hab.err \
        || { tail -5 /tmp/hab.err; exit 1; }
    python3 -c "
import json;d=json.loads(open('/tmp/hab.json').read().strip().splitlines()[-1])
print('$setting', round(d['value']/1e9,3), 'Gq/s kernel', round(d['roofline']['kernel_ms']*1e3,2), 'us', flush=True)"
done
done
