#!/bin/bash
# The SLAM-frame leg's mapping-iteration kernel timeline (tools/prof_slam.sh) once per
# tools/exp_libs variant (PIN_LIB), on one box.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for l in tools/exp_libs/*.so; do
    echo "== $(basename $l)"
    PIN_LIB=$PWD/$l bash tools/prof_slam.sh 2>&1 | grep -E "k_train|k_adam|k_mlp|iteration span" || exit 1
done
