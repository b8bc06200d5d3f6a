#!/bin/bash
# Round-6 evidence.  STEPS (default all): smoke, tests, bench, stats (rocprof kernel stats of every
# query leg -- headline, per-neighbour, mesher, tracker -- and of both mapper legs), qpmc (HBM
# traffic of the headline / per-neighbour / mesher kernels), tpmc (tracker kernel), mpmc (mapper
# kernels, both decoding modes).  Every GPU step has its own time limit; a fault ends the script.
# Outputs under gpurun_out/r06/; copy what is judged into profiles/r06/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r06; mkdir -p $OUT; export TMPDIR=/tmp
S=${STEPS:-smoke,tests,bench,stats,qpmc,tpmc,mpmc}
run() {   # name seconds command...
    local name=$1 secs=$2; shift 2
    timeout -k 10 "$secs" "$@" > $OUT/$name.log 2>&1
    local rc=$?
    echo "$name rc=$rc" | tee -a $OUT/summary.txt
    case $rc in 0|1) return 0 ;; *) echo "stopping after $name"; exit $rc ;; esac
}
NOLEGS="--no-cpu-baseline --no-map-update --no-process-frame --no-slam --no-input-order"
pmc() {   # name bench-args...: FETCH_SIZE and WRITE_SIZE passes, then bytes per launch
    local name=$1; shift
    for c in FETCH_SIZE WRITE_SIZE; do
        run ${name}_$c 420 rocprofv3 --kernel-trace --pmc $c --output-format csv -d $OUT/$name/$c -o run -- \
            python3 bench.py --steps 10 --warmup 3 $NOLEGS "$@"
    done
    python3 tools/traffic.py $OUT/$name > $OUT/${name}_traffic.json
}
echo "start $(date)" >> $OUT/summary.txt
[[ $S == *smoke* ]] && run smoke 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
[[ $S == *tests* ]] && run gpu_tests 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread
[[ $S == *bench* ]] && { run bench 600 python -u bench.py; grep '^{' $OUT/bench.log > $OUT/bench.json; }
if [[ $S == *stats* ]]; then
    run stats_query 420 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats_query -o run -- \
        python3 bench.py --steps 20 --warmup 5 $NOLEGS --no-mapper
    run stats_mapper 420 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats_mapper -o run -- \
        python3 bench.py --steps 20 --warmup 5 $NOLEGS --no-tracker --no-mesher --no-nwf-leg --mapper-steps 10 \
        --mapper-warmup 2
fi
[[ $S == *qpmc* ]] && pmc query --no-mapper --no-tracker
[[ $S == *tpmc* ]] && pmc tracker --no-mapper --no-mesher --no-nwf-leg
[[ $S == *mpmc* ]] && pmc mapper --no-tracker --no-mesher --no-nwf-leg --mapper-steps 5 --mapper-warmup 1
echo "done $(date)" >> $OUT/summary.txt
