#!/bin/bash
# PMC passes (one rocprofv3 run per counter group, as the pool requires) over the bench's
# kernels matching $KRE; summary per kernel and counter with tools/pmc_summary.py.
set -o pipefail
OUT=gpurun_out/${TAG:-pmc}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
KRE=${KRE:-k_canon_pass|k_minedge|k_level_pass}
i=0
IFS='|' read -ra GS <<< "${PMC_GROUPS:-SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES|FETCH_SIZE GRBM_GUI_ACTIVE|WRITE_SIZE TCC_HIT_sum TCC_MISS_sum|SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_ACTIVE_INST_LDS}"
for g in "${GS[@]}"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $g --kernel-include-regex "$KRE" -d "$OUT/p$i" -o run -- python3 bench.py --no-cpu-baseline --steps 1 --warmup 0 ${BENCH_ARGS} > "$OUT/p$i.json" 2> "$OUT/p$i.err" || { echo "pmc pass $i ($g) failed"; tail -5 "$OUT/p$i.err"; exit 1; }
done
python3 tools/pmc_summary.py "$OUT" | tee "$OUT/pmc.md"
# the raw rocprofv3 databases stay on the box (gpurun copies back at most 64 MiB)
for d in "$OUT"/p*/; do rm -rf "$d"; done
