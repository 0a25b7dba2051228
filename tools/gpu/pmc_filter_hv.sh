#!/bin/bash
# SQ counters of k_filter with and without the bucketed heavy passes (GHS_HV), R-MAT s24.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for hv in 0 1; do
  GHS_HV=$hv TAG=pmc_hv$hv KRE="k_filter|k_select" PMC_GROUPS="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES|SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_ACTIVE_INST_LDS|FETCH_SIZE GRBM_GUI_ACTIVE|WRITE_SIZE TCC_HIT_sum TCC_MISS_sum" BENCH_ARGS="--no-scaling-base" bash tools/gpu/pmc.sh > /dev/null || exit 1
done
for hv in 0 1; do echo "== GHS_HV=$hv"; cat gpurun_out/pmc_hv$hv/pmc.md; done
