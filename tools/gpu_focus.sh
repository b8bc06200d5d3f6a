#!/bin/bash
# Focused GPU session: selected GPU tests (PYTEST_K), then the bench with BENCH_ARGS.
# Every GPU step has its own time limit; a failing step ends the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
if [ -n "$PYTEST_K" ]; then
    timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "$PYTEST_K" \
        > $OUT/focus_tests.log 2>&1 || { tail -40 $OUT/focus_tests.log; exit 1; }
    tail -2 $OUT/focus_tests.log
fi
if [ -n "$BENCH_ARGS" ]; then
    timeout -k 10 500 python bench.py $BENCH_ARGS > $OUT/focus_bench.json 2> $OUT/focus_bench.err \
        || { tail -20 $OUT/focus_bench.err; exit 1; }
    cat $OUT/focus_bench.json
fi
echo done
