#!/bin/bash
# s26 x8 per-rank emulation with every rank's kernels in the level-opening rounds
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-r05emu}
mkdir -p $OUT
timeout -k 10 400 python -u tools/dist_emulate.py --scale ${SCALE:-26} --world ${W:-8} --reps 2 --profile --per-rank $EARGS > $OUT/emu.txt 2> $OUT/emu.err
