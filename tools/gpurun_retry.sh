#!/bin/bash
# gpurun, retried while no box / slot is free (exit 3, or a transient status); any other outcome
# ends it.  Usage: tools/gpurun_retry.sh OUTFILE TIMEOUT 'command'
out=$1; to=$2; cmd=$3
for i in $(seq 1 30); do
    /usr/local/graft/bin/gpurun --timeout "$to" -- "$cmd" > "$out" 2>&1
    rc=$?
    if [ $rc -eq 3 ] || grep -q "status=transient" "$out"; then sleep 60; continue; fi
    exit $rc
done
exit 3
