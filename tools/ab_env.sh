#!/bin/bash
# A/B of an environment switch on the bench (same box, alternating): AB_VAR=NAME, values AB_A / AB_B,
# bench arguments BENCH_ARGS; prints the headline, mapper, slam and tracker-loop numbers per run.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
for rep in 0 1; do
  for v in "$AB_A" "$AB_B"; do
    env $AB_VAR=$v timeout -k 10 300 python bench.py $BENCH_ARGS > $OUT/ab.json 2> $OUT/ab.err || { tail -5 $OUT/ab.err; exit 1; }
    python3 - "$AB_VAR=$v" <<'PY'
import json, sys
d = json.loads(open("gpurun_out/ab.json").read().strip().splitlines()[-1])
m = d.get("mapper") or {}
sl = d.get("slam_frame") or {}
tr = (d.get("tracker") or {}).get("tracking_loop") or {}
print(sys.argv[1], f"head {d['value']/1e9:.3f}G", f"mapper {m.get('value', 0):.1f} it/s", f"slam {sl.get('value', 0):.1f} fps",
      sl.get("parts_mean_ms"), f"track {tr.get('ms_per_iter', 0)*1e3:.1f} us/it", flush=True)
PY
  done
done
