#!/bin/bash
# tools/kernel_times.py for the default library and every tools/exp_libs variant
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
timeout -k 10 200 python3 tools/kernel_times.py || exit 1
for lib in tools/exp_libs/*.so; do
    PIN_LIB=$PWD/$lib timeout -k 10 200 python3 tools/kernel_times.py || exit 1
done
