#!/bin/bash
# For every library in tools/exp_libs: the timed headline leg (tools/variants.py run; NO_TIME=1
# skips it) and one PMC pass per counter group (CTR_GROUPS, ';'-separated) of the query kernel.
# Each GPU step has its own time limit.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/exp; rm -rf $OUT; mkdir -p $OUT
if [ -z "$NO_TIME" ]; then
    timeout -k 10 500 python3 tools/variants.py run > $OUT/times.txt 2>&1 || { cat $OUT/times.txt; exit 1; }
    cat $OUT/times.txt
fi
GROUPS_STR=${CTR_GROUPS:-"SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU"}
IFS=';' read -ra GROUPS_ARR <<< "$GROUPS_STR"
for lib in tools/exp_libs/*.so; do
    n=$(basename $lib .so)
    g=0
    for grp in "${GROUPS_ARR[@]}"; do
        g=$((g+1))
        PIN_LIB=$PWD/$lib timeout -k 10 120 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d $OUT/$n/g$g -o run -- \
            python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-mapper --no-tracker --no-mesher --no-map-update \
            --no-process-frame --no-nwf-leg > $OUT/$n.g$g.log 2>&1 || { echo "pmc $n g$g failed"; tail -5 $OUT/$n.g$g.log; exit 1; }
    done
    echo "== $n"; python3 tools/pmc_summary.py $OUT/$n ${KMATCH:-k_query_sdf_grid} | sed 's/^.*> *//'
done
