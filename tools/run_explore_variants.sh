#!/bin/bash
# tools/explore_mapper.py (WFS, default weighted_first) once per tools/exp_libs variant, on one box.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for l in tools/exp_libs/*.so; do
    echo "$(basename $l) $(PIN_LIB=$PWD/$l WFS=${WFS:-1} timeout -k 10 200 python3 tools/explore_mapper.py 2>&1 | grep wf=)" || exit 1
done
