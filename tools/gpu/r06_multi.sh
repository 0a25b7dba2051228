#!/bin/bash
# Round 6: the multi-rank loop's tests (emulated ranks, the RCCL stub), then the s26 x 8 emulation.
set -o pipefail
OUT=gpurun_out/${TAG:-r06multi}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_rccl_stub.py tests/test_gpu_csr.py tests/test_gpu_distributed.py -m gpu -x -v --timeout 300 --timeout-method thread -k "${PYK:-emulated or native_loop or rccl or multi or distributed or partitioned}" > "$OUT/pytest.log" 2>&1
rc=$?; tail -3 "$OUT/pytest.log"; [ $rc -ne 0 ] && { grep -E "FAILED|Error" "$OUT/pytest.log" | head -20; exit 1; }
[ -n "$NOEMU" ] && exit 0
TAG=${TAG:-r06multi} EMUS="${EMUS:-tail:}" bash tools/gpu/r06_emu.sh
