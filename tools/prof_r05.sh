#!/bin/bash
# Round-5 evidence.  STEPS (default all): smoke, tests, bench, prof (kernel stats of the headline
# and mapper legs), nwf_pmc (HBM traffic of the per-neighbour mapper kernels), dbwd (rocprof of
# the drop-in double backward).  Every GPU step has its own time limit; a fault ends the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r05; mkdir -p $OUT; export TMPDIR=/tmp
S=${STEPS:-smoke,tests,bench,prof,nwf_pmc,wf_pmc,dbwd}
run() {   # name seconds command...
    local name=$1 secs=$2; shift 2
    timeout -k 10 "$secs" "$@" > $OUT/$name.log 2>&1
    local rc=$?
    echo "$name rc=$rc" | tee -a $OUT/summary.txt
    case $rc in 0|1) return 0 ;; *) echo "stopping after $name"; exit $rc ;; esac
}
echo "start $(date)" > $OUT/summary.txt
[[ $S == *smoke* ]] && run smoke 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
[[ $S == *tests* ]] && run gpu_tests 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread
[[ $S == *bench* ]] && { run bench 600 python -u bench.py; cp $OUT/bench.log $OUT/bench_full.log; grep '^{' $OUT/bench.log > $OUT/bench.json; }
if [[ $S == *prof* ]]; then
    run prof 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- \
        python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-tracker --no-mesher --no-map-update \
        --no-process-frame --no-nwf-leg --no-slam --mapper-steps 5 --mapper-warmup 2
fi
if [[ $S == *nwf_pmc* ]]; then
    for c in FETCH_SIZE WRITE_SIZE; do
        run nwf_$c 300 rocprofv3 --kernel-trace --pmc $c --output-format csv -d $OUT/nwf_pmc/$c -o run -- \
            python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --nwf --no-tracker --no-mesher --no-map-update \
            --no-process-frame --no-slam --no-input-order --mapper-steps 3 --mapper-warmup 1
    done
    python3 tools/traffic.py $OUT/nwf_pmc > $OUT/mapper_nwf_traffic.json 2>&1
fi
if [[ $S == *wf_pmc* ]]; then   # HBM traffic of the weighted-first mapper kernels (sorted-run scatter)
    for c in FETCH_SIZE WRITE_SIZE; do
        run wf_$c 300 rocprofv3 --kernel-trace --pmc $c --output-format csv -d $OUT/wf_pmc/$c -o run -- \
            python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-tracker --no-mesher --no-map-update \
            --no-process-frame --no-slam --no-input-order --no-mapper-nwf --no-nwf-leg --mapper-steps 3 --mapper-warmup 1
    done
    python3 tools/traffic.py $OUT/wf_pmc > $OUT/mapper_wf_traffic.json 2>&1
fi
if [[ $S == *dbwd* ]]; then
    run dbwd 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/dbwd -o run -- \
        python3 -m pytest -q tests/test_gpu_mapper.py -k "double_backward_matches_reference and grid"
fi
if [[ $S == *dbloop* ]]; then
    run dbloop 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/dbloop -o run -- \
        python3 tools/dbwd_loop.py
fi
echo "end $(date)" >> $OUT/summary.txt
