#!/bin/bash
# HBM-side traffic per launch of the bench kernels: two PMC passes (FETCH_SIZE, WRITE_SIZE: they
# do not fit one TCC pass), kernel-trace only, then tools/traffic.py -> gpurun_out/traffic.json.
# Default: the headline legs only (the per-kernel means are then the headline launches'); set
# BENCH_ARGS to profile other legs.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TRAFFIC_NAME:-traffic}
rm -rf $OUT; mkdir -p $OUT
for c in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 300 rocprofv3 --kernel-trace --pmc $c --output-format csv -d $OUT/$c -o run -- \
        python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline ${BENCH_ARGS:---no-mapper --no-tracker --no-mesher --no-map-update --no-process-frame --no-nwf-leg --no-slam --no-input-order} > $OUT/$c.log 2>&1 || exit $?
done
python3 tools/traffic.py $OUT > gpurun_out/${TRAFFIC_NAME:-traffic}.json
