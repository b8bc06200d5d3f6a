#!/bin/bash
# bench.py with only the legs named in LEGS (slam, mapper, nwf, map, pf, tracker, mesher); headline
# leg short.  Output: gpurun_out/legs_$TAG.json
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
L=${LEGS:-slam,mapper}
A="--no-cpu-baseline --no-nwf-leg --no-input-order --steps 20 --warmup 5"
[[ $L == *slam* ]] || A="$A --no-slam"
[[ $L == *mapper* ]] || A="$A --no-mapper"
[[ $L == *nwf* ]] || A="$A --no-mapper-nwf"
[[ $L == *map,* || $L == *map ]] || A="$A --no-map-update"
[[ $L == *pf* ]] || A="$A --no-process-frame"
[[ $L == *tracker* ]] || A="$A --no-tracker"
[[ $L == *mesher* ]] || A="$A --no-mesher"
timeout -k 10 400 python bench.py $A > gpurun_out/legs_${TAG:-x}.json || exit $?
python3 - <<PY
import json
d = json.loads(open("gpurun_out/legs_${TAG:-x}.json").read().strip().splitlines()[-1])
print("headline", round(d["value"] / 1e9, 3), "Gq/s")
for k in ("slam_frame", "mapper", "mapper_nwf", "map_update", "process_frame", "tracker", "mesher"):
    m = d.get(k)
    if m:
        print(k, round(m["value"], 2), m.get("unit"), {kk: m[kk] for kk in ("ms_per_frame", "median_ms_per_frame", "ms_per_iter", "parts_mean_ms") if kk in m})
PY
