#!/bin/bash
# For every library in tools/exp_libs: the timed headline leg (tools/variants.py run) and one
# SQ counter pass of the query kernel per variant.  Each GPU step has its own time limit.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/exp; rm -rf $OUT; mkdir -p $OUT
timeout -k 10 500 python3 tools/variants.py run > $OUT/times.txt 2>&1 || { cat $OUT/times.txt; exit 1; }
cat $OUT/times.txt
CTR=${CTR:-"SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU"}
for lib in tools/exp_libs/*.so; do
    n=$(basename $lib .so)
    PIN_LIB=$PWD/$lib timeout -k 10 120 rocprofv3 --kernel-trace --pmc $CTR --output-format csv -d $OUT/$n -o run -- \
        python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-mapper --no-tracker --no-mesher --no-map-update \
        --no-process-frame --no-nwf-leg > $OUT/$n.log 2>&1 || { echo "pmc $n failed"; tail -5 $OUT/$n.log; exit 1; }
    echo "== $n"; python3 tools/pmc_summary.py $OUT/$n k_query_sdf_grid | sed 's/^.*> *//'
done
