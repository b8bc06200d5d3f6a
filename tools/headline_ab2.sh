#!/bin/bash
# Headline step A/B: the fused one-launch tile sort against the two launches (PIN_SORT_FUSED=0),
# alternating, headline leg only.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
A="--no-cpu-baseline --no-nwf-leg --no-mesher --no-tracker --no-map-update --no-process-frame --no-slam --no-mapper"
for r in 1 2 3; do
  for f in 1 0; do  # PIN_SORT_FUSED=1: the opt-in one-launch sort
    PIN_SORT_FUSED=$f timeout -k 10 120 python bench.py $A --steps 200 --warmup 20 > gpurun_out/hab_$f.json || exit $?
    python3 -c "
import json;d=json.load(open('gpurun_out/hab_$f.json'))
print('fused=$f', round(d['value']/1e9,3), 'Gq/s step', round(d['ms_per_step']*1e3,2), 'us kernel', round(d['roofline']['kernel_ms']*1e3,2), 'order', round(d['roofline']['order_pass_ms']*1e3,2))"
  done
done
