#!/bin/bash
# SLAM-frame leg under environment variants (two runs each, interleaved); the variants are the
# arguments (VAR=value each), default: the replica count and the paired-lane forward
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
for rep in 1 2; do
VARS=("$@"); [ ${#VARS[@]} -eq 0 ] && VARS=("DEFAULT=1" "PIN_TRAIN_REPLICAS=4" "PIN_TRAIN_REPLICAS=1" "PIN_TRAIN_PAIR_ROWS=0")
for v in "${VARS[@]}"; do
  env $v timeout -k 10 200 python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-mapper --no-tracker --no-mesher \
     --no-map-update --no-process-frame --no-nwf-leg > gpurun_out/se.json 2> gpurun_out/se.err
  rc=$?; [ $rc -ne 0 ] && { echo "$v rc=$rc"; tail -3 gpurun_out/se.err; exit $rc; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/se.json').read().strip().splitlines()[-1])['slam_frame']; print(sys.argv[1], round(d['ms_per_frame'],3), d['parts_mean_ms'])" "$v"
done; done
