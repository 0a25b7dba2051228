#!/bin/bash
# parity suite + same-box A/B of the working tree (new) vs lib/exp/base.so (HEAD): s24, s26, grid
set -o pipefail
mkdir -p gpurun_out/abb
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 250 --timeout-method thread > gpurun_out/abb/pytest.log 2>&1 || { tail -30 gpurun_out/abb/pytest.log; exit 1; }
tail -1 gpurun_out/abb/pytest.log
TAG=abb REPS=3 VARIANTS="base:GHS_MST_LIB=distributed_ghs_implementation_amd/lib/exp/base.so new:" TOPK=4 bash tools/gpu/ab.sh
TAG=abb_s26 REPS=2 BENCH_ARGS="--scale 26 --steps 3 --warmup 1" VARIANTS="base:GHS_MST_LIB=distributed_ghs_implementation_amd/lib/exp/base.so new:" TOPK=4 bash tools/gpu/ab.sh
TAG=abb_grid REPS=1 BENCH_ARGS="--workload grid --steps 4 --warmup 1" VARIANTS="base:GHS_MST_LIB=distributed_ghs_implementation_amd/lib/exp/base.so new:" TOPK=4 bash tools/gpu/ab.sh
