#!/bin/bash
# Round-4 evidence, part B: headline kernel stats, matrix-core PMC, HBM traffic of the headline and
# mapper legs, the mapper timeline, the per-neighbour mapper's kernel stats.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r04; mkdir -p $OUT; export TMPDIR=/tmp
bash tools/prof_query.sh > $OUT/prof_query.txt 2>&1 || { tail -5 $OUT/prof_query.txt; exit 1; }
cp gpurun_out/query_kernel_stats.csv $OUT/ && echo query-ok
bash tools/mfma_pmc.sh || exit 1
cp gpurun_out/mfma.json $OUT/ && echo mfma-ok
bash tools/traffic.sh || exit 1
cp gpurun_out/traffic.json $OUT/traffic_headline.json && echo traffic-ok
bash tools/prof_mapper.sh > $OUT/mapper_timeline.txt 2>&1 || { tail -5 $OUT/mapper_timeline.txt; exit 1; }
cp gpurun_out/profm/run_kernel_stats.csv $OUT/mapper_kernel_stats.csv && echo mapper-ok
TRAFFIC_NAME=mapper_traffic BENCH_ARGS="--no-tracker --no-mesher --no-map-update --no-process-frame --no-nwf-leg --no-slam --no-input-order --no-mapper-nwf --mapper-steps 5" bash tools/traffic.sh || exit 1
cp gpurun_out/mapper_traffic.json $OUT/ && echo mapper-traffic-ok
D=$OUT/profnwf; rm -rf $D; mkdir -p $D
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D -o run -- \
    python3 bench.py --nwf --steps 5 --warmup 2 --no-cpu-baseline --no-tracker --no-mesher --no-map-update \
    --no-process-frame --no-slam --mapper-steps 5 > $D/bench.json 2> $D/bench.err || exit 1
cp $D/run_kernel_stats.csv $OUT/mapper_nwf_kernel_stats.csv && echo nwf-ok
