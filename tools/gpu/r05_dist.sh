#!/bin/bash
# the device-side MSF compaction test, the distributed GPU tests, then the N=4 gloo bench rehearsal
# at s26 (ranks sharing the box's GPU)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r05dist
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -k "flags_to_eids or distributed or cache or fault" > gpurun_out/r05dist/pytest.log 2>&1; rc=$?
grep -E "FAILED|passed|failed" gpurun_out/r05dist/pytest.log | tail -8
case $rc in 0) ;; *) exit 1;; esac
NS="${NS:-4}" STEPS=2 TAG=r05dist timeout -k 10 500 bash tools/gpu/dist_bench_rehearsal.sh
