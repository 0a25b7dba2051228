#!/bin/bash
# parity subset + same-box A/B of the working tree (new) vs lib/exp/base.so (HEAD), R-MAT s24
set -o pipefail
mkdir -p gpurun_out/absel
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -q --timeout 200 --timeout-method thread -k "rmat_device or s24_full or noncanonical or tie or golden or native_loop_emulated" > gpurun_out/absel/pytest.log 2>&1 || { tail -30 gpurun_out/absel/pytest.log; exit 1; }
tail -1 gpurun_out/absel/pytest.log
TAG=absel REPS=3 VARIANTS="base:GHS_MST_LIB=distributed_ghs_implementation_amd/lib/exp/base.so new:" TOPK=5 bash tools/gpu/ab.sh
