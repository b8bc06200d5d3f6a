#!/bin/bash
# Memory-pipeline counters (TA / TD / TCP) of the headline query kernel, one group per pass:
# is the fused kernel bound by the per-CU address / data path of its gathers?
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
G="GRBM_GUI_ACTIVE TA_TA_BUSY TA_ADDR_STALLED_BY_TC_CYCLES TD_TD_BUSY TD_TC_STALL SQ_WAVES SQ_INSTS_VMEM_RD SQ_BUSY_CYCLES;TCP_TOTAL_CACHE_ACCESSES TCP_TCC_READ_REQ TCP_PENDING_STALL_CYCLES TCP_TCP_TA_DATA_STALL_CYCLES TA_FLAT_READ_WAVEFRONTS TA_DATA_STALLED_BY_TC_CYCLES;TCP_READ_TAGCONFLICT_STALL_CYCLES TCP_TCR_TCP_STALL_CYCLES TCP_TCC_READ_REQ_LATENCY TCP_TCP_LATENCY SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU"
BENCH_ARGS="--no-mapper --no-tracker --no-mesher --no-map-update --no-process-frame --no-nwf-leg" PMC_OUT=gpurun_out/pmc_ta PMC_GROUPS="$G" bash tools/gpu_pmc.sh
