#!/bin/bash
# Matrix-core evidence for the headline SDF+grad kernel: one PMC pass (SQ_VALU_MFMA_BUSY_CYCLES,
# SQ_INSTS_VALU_MFMA_MOPS_F16, SQ_INSTS_MFMA, GRBM_GUI_ACTIVE; kernel-trace only) over the
# headline leg, then tools/mfma_pmc.py -> gpurun_out/mfma.json.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/mfma; rm -rf $OUT; mkdir -p $OUT
timeout -k 10 180 rocprofv3 --kernel-trace \
    --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F16 SQ_INSTS_MFMA GRBM_GUI_ACTIVE \
    --output-format csv -d $OUT/p -o run -- \
    python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-mapper --no-tracker --no-mesher \
    --no-map-update --no-process-frame --no-slam --no-input-order ${BENCH_ARGS:-} > $OUT/bench.log 2>&1 || exit $?
python3 tools/mfma_pmc.py $OUT > gpurun_out/mfma.json
