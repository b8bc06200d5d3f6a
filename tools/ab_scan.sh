#!/bin/bash
# A/B of the grid scan variants (PIN_GRID_SCAN=bricks|cells vs the default column scan) on the
# headline bench leg, after the GPU parity tests.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
for rep in 1 2; do
for v in columns bricks; do
    PIN_GRID_SCAN=$v timeout -k 10 120 python bench.py --no-mapper --no-tracker --no-mesher --no-map-update --no-process-frame --no-nwf-leg --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/ab_$v.json 2>gpurun_out/ab_$v.err || exit 1
    python - "$v" <<'PY'
import json, sys
d = json.loads(open(f"gpurun_out/ab_{sys.argv[1]}.json").read().strip().splitlines()[-1])
print(f"{sys.argv[1]:8s} {d['value']/1e9:.3f} Gq/s kernel {d['roofline']['kernel_ms']*1e3:.1f} us frac {d['roofline']['frac']:.3f}")
PY
done
done
