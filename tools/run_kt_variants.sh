#!/bin/bash
# tools/kernel_times.py (grad variants) for every library in tools/exp_libs (tools/variants.py build).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for l in tools/exp_libs/*.so; do
    KT_SIZES=${KT_SIZES:-262144} KT_WF=${KT_WF:-1,0} PIN_LIB=$PWD/$l timeout -k 10 200 python3 tools/kernel_times.py 2>&1 \
        | grep "grad=1" || exit 1
done
