#!/bin/bash
# Every profile the round's DESIGN.md / bench line cites, one GPU call: headline kernel stats,
# HBM traffic (two PMC passes over the whole bench), matrix-core counters, the mapper timeline.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/prof_query.sh > gpurun_out/prof_query.txt 2>&1 || { tail -5 gpurun_out/prof_query.txt; exit 1; }
bash tools/mfma_pmc.sh || exit 1
bash tools/traffic.sh || exit 1
bash tools/prof_mapper.sh > gpurun_out/prof_mapper.txt 2>&1 || { tail -5 gpurun_out/prof_mapper.txt; exit 1; }
echo done
