#!/bin/bash
# tools/explore_mapper.py (weighted_first) with the default library, then every tools/exp_libs variant.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
WFS=${WFS:-1} timeout -k 10 200 python3 tools/explore_mapper.py 2>&1 | grep wf= || exit 1
for l in tools/exp_libs/*.so; do
    echo "$l"; PIN_LIB=$PWD/$l WFS=${WFS:-1} timeout -k 10 200 python3 tools/explore_mapper.py 2>&1 | grep wf= || exit 1
done
