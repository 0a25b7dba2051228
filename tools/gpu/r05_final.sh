#!/bin/bash
# Round-5 final tree: the GPU suite, then the evidence set (tools/gpu/r05_evidence.sh).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${TAG:-r05final} LIMIT=600 bash tools/gpu/pytest_gpu.sh > /dev/null; rc=$?
tail -2 gpurun_out/${TAG:-r05final}/pytest_gpu.log
[ $rc = 0 ] || exit 1
TAG=${TAG:-r05final}/evidence bash tools/gpu/r05_evidence.sh
