#!/bin/bash
# bench.py's whole-frame leg (configs[0]) once per tools/exp_libs variant (PIN_LIB): frames/s and
# the mean part times, plus the headline step for reference.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for l in tools/exp_libs/*.so; do
    PIN_LIB=$PWD/$l timeout -k 10 150 python3 bench.py --steps 20 --no-cpu-baseline --no-mapper --no-tracker \
        --no-mesher --no-map-update --no-process-frame --no-nwf-leg --no-input-order > /tmp/sv.json 2>/dev/null || exit 1
    python3 -c "
import json; d = json.load(open('/tmp/sv.json')); s = d['slam_frame']
print('$(basename $l)', round(d['value'] / 1e9, 3), 'Gq/s', round(s['value'], 1), 'frames/s', s['parts_mean_ms'], 'err', round(s['max_pose_error_m'], 4))"
done
