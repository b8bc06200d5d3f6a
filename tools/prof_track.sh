#!/bin/bash
# rocprofv3 kernel trace of the tracker leg only; prints the kernel timeline of the last tracking()
# call (GPU busy vs gaps per registration iteration).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=/tmp/proft; rm -rf $OUT; mkdir -p $OUT gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d $OUT -o run -- \
    python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-mapper --no-slam --no-mesher --no-map-update \
    --no-process-frame --no-nwf-leg --no-input-order > $OUT/bench.json 2> $OUT/bench.err || { tail -5 $OUT/bench.err; exit 1; }
python3 - <<'PY'
import csv, glob
f = glob.glob("/tmp/proft/**/*kernel_trace.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
ev = ev[-40:]
t0 = ev[0][0]
prev = None
for s, e, n in ev:
    gap = (s - prev) / 1e3 if prev else 0.0
    print(f"{(s - t0) / 1e3:9.1f} {(e - s) / 1e3:7.1f} gap {gap:6.1f}  {n[:70]}")
    prev = e
PY
