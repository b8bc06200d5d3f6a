#!/bin/bash
# Round checkpoint on the GPU box: smoke(), GPU parity tests, the default bench line, and the
# rocprofv3 kernel-trace summary of the headline leg.  Every GPU step has its own time limit.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 400 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -30 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
bash tools/prof_query.sh > $OUT/prof.log 2>&1 || { tail -20 $OUT/prof.log; exit 1; }
echo done
