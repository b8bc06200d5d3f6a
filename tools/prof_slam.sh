#!/bin/bash
# rocprofv3 kernel trace of the whole-frame leg only; prints the kernel timeline of one steady-state
# mapping iteration (GPU busy vs gaps) and the per-kernel totals of the timed frames.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=/tmp/profs; rm -rf $OUT; mkdir -p $OUT gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o run -- \
    python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-mapper --no-tracker --no-mesher --no-map-update \
    --no-process-frame --no-nwf-leg > $OUT/bench.json 2> $OUT/bench.err || { tail -5 $OUT/bench.err; exit 1; }
cp $(find $OUT -name "*kernel_stats.csv" | head -1) gpurun_out/slam_kernel_stats.csv
python3 - <<'PY'
import csv, glob
f = glob.glob("/tmp/profs/**/*kernel_trace.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
# steady-state mapping iterations: the decoder Adam launch marks each iteration's end (k_adam_segments,
# or k_adam_step_segments when the feature and decoder steps share one launch)
idx = [i for i, e in enumerate(ev) if "k_adam_segments" in e[2] or "k_adam_step_segments" in e[2] or "k_adam_train" in e[2]]
print("mapping iterations seen:", len(idx))
a, b = idx[-8], idx[-7]
prev = None
busy = 0
for s, e, n in ev[a + 1:b + 1]:
    short = n.replace("(anonymous namespace)::", "").replace("void ", "")[:70]
    gap = (s - prev) / 1e3 if prev else 0.0
    busy += e - s
    print(f"{short:70s} {(e - s) / 1e3:8.2f} us  gap {gap:6.2f}")
    prev = e
print("iteration span", (ev[b][1] - ev[a][1]) / 1e3, "us, kernels busy", busy / 1e3, "us")
PY
