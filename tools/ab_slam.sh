#!/bin/bash
# A/B of the whole-frame leg on one box: each ENV=VALUE argument runs bench.py's SLAM leg twice
# with that environment (e.g. PIN_TRAIN_ROW_DECODE=0 PIN_TRAIN_ROW_DECODE=1).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for rep in 0 1; do
  for kv in "$@"; do
    (export $kv; timeout -k 10 300 python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-mapper --no-tracker \
        --no-mesher --no-map-update --no-process-frame --no-nwf-leg --no-input-order > /tmp/ab.json 2>/dev/null) || exit 1
    python3 -c "
import json, sys; d = json.loads(open('/tmp/ab.json').read().strip().splitlines()[-1])['slam_frame']
print('rep$rep', '$kv', round(d['value'], 1), 'fps', {k: round(v, 3) for k, v in d['parts_mean_ms'].items()})"
  done
done
