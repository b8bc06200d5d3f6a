#!/bin/bash
# Run GPU steps in order, each under its own time limit; stop at the first step that ends in a
# fault, abort, signal or time limit (anything but 0 = ok / 1 = ordinary test failure).
#   tools/gpu_steps.sh NAME:SECONDS:COMMAND [NAME:SECONDS:COMMAND ...]
# Output of step NAME goes to gpurun_out/NAME.log; a summary to gpurun_out/steps.txt.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
echo "start $(date)" > gpurun_out/steps.txt
for spec in "$@"; do
    name=${spec%%:*}
    rest=${spec#*:}
    secs=${rest%%:*}
    cmd=${rest#*:}
    timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
    rc=$?
    echo "$name rc=$rc" | tee -a gpurun_out/steps.txt
    tail -3 "gpurun_out/$name.log" >> gpurun_out/steps.txt
    case $rc in
        0|1) ;;
        *) echo "stopping after $name (rc=$rc)" | tee -a gpurun_out/steps.txt; exit "$rc" ;;
    esac
done
