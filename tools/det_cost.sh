#!/bin/bash
# Cost of the deterministic training mode: the mapper legs and the SLAM frame with and without
# PIN_DETERMINISTIC=1, alternating (two rounds).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for r in 1 2; do
  for d in 0 1; do
    echo "== PIN_DETERMINISTIC=$d"
    PIN_DETERMINISTIC=$d TAG=det$d LEGS=slam,mapper,nwf tools/bench_legs.sh || exit $?
  done
done
