#!/bin/bash
# SLAM-leg A/B: the whole-frame leg's mapping time and one steady-state iteration's kernel timeline,
# once per environment setting given as arguments (e.g. "PIN_TRAIN_TILE_MIN=1024").
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for setting in "$@"; do
    echo "=== $setting"
    env $setting bash tools/prof_slam.sh > /tmp/slam_ab.txt 2>&1 || { tail -5 /tmp/slam_ab.txt; exit 1; }
    grep -E "k_train|k_adam|k_mlp|k_tile|span" /tmp/slam_ab.txt
    python3 -c "import json;d=json.loads(open('/tmp/profs/bench.json').read().strip().splitlines()[-1]);print('slam parts', d['slam_frame']['parts_mean_ms'], 'fps', round(d['slam_frame']['value'],1))"
done
