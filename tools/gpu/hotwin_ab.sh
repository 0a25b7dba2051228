#!/bin/bash
# windowed fragment-min cache: parity with a small window, then A/B of GHS_HOT_WINDOW
set -o pipefail
mkdir -p gpurun_out/hotwin
GHS_HOT_WINDOW=2 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -q --timeout 250 --timeout-method thread -k "grid or rmat_device or tie or s24_full or 16k or emulated or partitioned" > gpurun_out/hotwin/pytest.log 2>&1 || { tail -30 gpurun_out/hotwin/pytest.log; exit 1; }
tail -1 gpurun_out/hotwin/pytest.log
TAG=hotwin_grid REPS=1 BENCH_ARGS="--workload grid --steps 4 --warmup 1" VARIANTS="w0:GHS_HOT_WINDOW=0 w4:GHS_HOT_WINDOW=4 w16:GHS_HOT_WINDOW=16 w64:GHS_HOT_WINDOW=64" TOPK=5 bash tools/gpu/ab.sh
TAG=hotwin_rmat REPS=1 VARIANTS="w0:GHS_HOT_WINDOW=0 w4:GHS_HOT_WINDOW=4 w16:GHS_HOT_WINDOW=16 w64:GHS_HOT_WINDOW=64" TOPK=5 bash tools/gpu/ab.sh
