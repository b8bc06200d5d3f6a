#!/bin/bash
# rocprofv3 kernel trace + stats of the mapper leg (headline leg kept short, other legs off),
# then the per-iteration kernel timeline of one steady-state iteration.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/profm; rm -rf $OUT; mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o run -- \
    python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-tracker --no-mesher --no-map-update \
    --no-process-frame --no-nwf-leg --no-slam --no-mapper-nwf ${BENCH_ARGS:-} > $OUT/bench.json 2> $OUT/bench.err || exit $?
python3 - <<'PY'
import csv
rows = list(csv.DictReader(open("gpurun_out/profm/run_kernel_trace.csv")))
ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
# the last k_adam marks the end of the timed mapping(); print the kernels of the iteration before it
idx = [i for i, e in enumerate(ev) if "k_adam" in e[2]]
a, b = idx[-3], idx[-2]
prev = None
for s, e, n in ev[a + 1:b + 1]:
    short = n.replace("(anonymous namespace)::", "").replace("void ", "")[:70]
    gap = (s - prev) / 1e3 if prev else 0.0
    print(f"{short:70s} {(e - s) / 1e3:8.2f} us  gap {gap:6.2f}")
    prev = e
print("iteration span", (ev[b][1] - ev[a][1]) / 1e3, "us")
PY
