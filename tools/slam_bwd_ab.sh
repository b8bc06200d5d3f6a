#!/bin/bash
# SLAM-frame mapping kernels, default library vs a variant (LIB): rocprofv3 kernel stats of the
# whole-frame leg, the training kernels' averages side by side.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
V=${LIB:-$(ls tools/exp_libs/*.so | head -1)}
for tag in def var; do
  OUT=gpurun_out/slamab_$tag; rm -rf $OUT; mkdir -p $OUT
  if [ $tag = var ]; then export PIN_LIB=$V; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o run -- \
    python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-mapper --no-tracker --no-mesher --no-map-update \
    --no-process-frame --no-nwf-leg --no-input-order > $OUT/bench.json 2> $OUT/bench.err || exit 1
done
python3 - <<'PY'
import csv
for tag in ("def", "var"):
    rows = list(csv.DictReader(open(f"gpurun_out/slamab_{tag}/run_kernel_stats.csv")))
    for r in rows:
        if "k_train" in r["Name"] or "k_adam" in r["Name"] or "k_mlp" in r["Name"]:
            print(tag, r["Calls"], round(float(r["AverageNs"]) / 1e3, 2), r["Name"][:90])
PY
