#!/bin/bash
# tools/explore_mapper.py once per library variant in tools/exp_libs (WFS etc. passed through).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for so in tools/exp_libs/*.so; do
    echo "== $(basename "$so")"
    PIN_LIB=$so timeout -k 10 150 python -u tools/explore_mapper.py || exit $?
done
