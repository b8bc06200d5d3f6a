#!/bin/bash
# One GPU-box session: parity tests, a bench line, a rocprofv3 kernel-trace summary.
# Every GPU step has its own time limit; a crash/fault/timeout ends the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp

stop_on_fatal() {  # $1 = rc, $2 = step
    case $1 in
        0|1) return 0 ;;   # ok / ordinary test failure
        *) echo "FATAL rc=$1 in $2; stopping" | tee -a $OUT/summary.txt; exit $1 ;;
    esac
}

STEPS=${STEPS:-tests,bench,prof}
echo "start $(date)" > $OUT/summary.txt
if [[ $STEPS == *tests* ]]; then
    timeout -k 10 900 python -m pytest tests -m gpu -q -rf ${PYTEST_ARGS:-} > $OUT/gpu_tests.log 2>&1
    rc=$?; echo "tests rc=$rc" >> $OUT/summary.txt; tail -5 $OUT/gpu_tests.log >> $OUT/summary.txt
    stop_on_fatal $rc tests
fi
if [[ $STEPS == *bench* ]]; then
    timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > $OUT/bench.json 2> $OUT/bench.err
    rc=$?; echo "bench rc=$rc" >> $OUT/summary.txt; cat $OUT/bench.json >> $OUT/summary.txt
    stop_on_fatal $rc bench
fi
if [[ $STEPS == *prof* ]]; then
    timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- \
        python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline ${BENCH_ARGS:-} > $OUT/prof.log 2>&1
    rc=$?; echo "prof rc=$rc" >> $OUT/summary.txt
    stop_on_fatal $rc prof
    find $OUT/prof -name "*kernel_stats.csv" -exec cp {} $OUT/kernel_stats.csv \;
    cat $OUT/kernel_stats.csv >> $OUT/summary.txt 2>/dev/null
fi
echo "done $(date)" >> $OUT/summary.txt
