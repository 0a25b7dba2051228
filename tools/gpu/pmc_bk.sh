#!/bin/bash
# PMC of the bucketed-round kernels on the grid workloads (one rocprofv3 pass per counter group).
set -o pipefail
for wl in ${WLS:-grid grid-gradient}; do
  TAG=${TAG:-pmcbk}/$wl KRE="${KRE:-k_bmin|k_bucket}" BENCH_ARGS="--workload $wl --no-scaling-base" \
  PMC_GROUPS="${PMC_GROUPS:-SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES|FETCH_SIZE GRBM_GUI_ACTIVE|WRITE_SIZE TCC_HIT_sum TCC_MISS_sum|SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS}" \
  bash tools/gpu/pmc.sh || exit 1
done
