#!/bin/bash
# rocprofv3 kernel stats of the headline leg only (query order + SDF+grad kernel).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/profq
rm -rf $OUT; mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o run -- \
    python3 bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-mapper --no-tracker --no-mesher --no-map-update --no-process-frame --no-nwf-leg --no-slam --no-input-order \
    ${BENCH_ARGS:-} > $OUT/bench.json 2> $OUT/bench.err || exit $?
f=$(find $OUT -name "*kernel_stats.csv" | head -1)
cp $f gpurun_out/query_kernel_stats.csv
cut -d, -f1-4 $f | head -12
tail -1 $OUT/bench.json | cut -c1-300
