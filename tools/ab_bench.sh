#!/bin/bash
# A/B of the grid query variants on the headline workload (+ parity tests first).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
if [ -z "$NO_TESTS" ]; then
    timeout -k 10 600 python -m pytest tests -m gpu -q -x > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
    tail -1 gpurun_out/gpu_tests.log
fi
for split in 1 0; do  # PIN_QUERY_BIN
for v in window cells; do
    PIN_QUERY_TILES=$split PIN_GRID_SCAN=$v timeout -k 10 300 python bench.py --no-mapper --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/ab_${split}_$v.json 2>gpurun_out/ab_${split}_$v.err || exit 1
    python3 -c "import json;d=json.load(open('gpurun_out/ab_${split}_$v.json'));print('tiles=$split $v', round(d['value']/1e9,3),'Gq/s kernel_ms', round(d['roofline']['kernel_ms'],4))"
done
done
