#!/bin/bash
# PMC passes (one counter group per run, kernel-trace only), for the roofline traffic figure.
# PMC_GROUPS: groups separated by ';', counters inside a group by spaces.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${PMC_OUT:-gpurun_out/pmc}
rm -rf $OUT
mkdir -p $OUT
export TMPDIR=/tmp
rocprofv3 -L > $OUT/counters_list.txt 2>&1 || true
GROUPS_STR=${PMC_GROUPS:-"FETCH_SIZE;WRITE_SIZE;TCC_HIT_sum TCC_MISS_sum;TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum"}
IFS=';' read -ra GROUPS_ARR <<< "$GROUPS_STR"
i=0
for grp in "${GROUPS_ARR[@]}"; do
    i=$((i+1))
    timeout -k 10 300 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d $OUT/p$i -o run -- \
        python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline ${BENCH_ARGS:-} > $OUT/p$i.log 2>&1
    rc=$?
    echo "group $i ($grp) rc=$rc" >> $OUT/summary.txt
    case $rc in 0) ;; *) echo "stopping"; exit $rc ;; esac
done
python3 tools/pmc_summary.py $OUT > $OUT/pmc_summary.txt 2>&1 || true
