#!/bin/bash
# Build libghs_mst.so from a git revision into distributed_ghs_implementation_amd/lib/exp/<name>.so
# (same-box A/B runs: tools/gpu/ab.sh with GHS_MST_LIB=...). Usage: tools/build_rev.sh REV NAME
set -e
REV=${1:-HEAD}; NAME=${2:-base}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
T=$(mktemp -d)
mkdir -p "$T/x/csrc" "$T/include"
git -C "$ROOT" show "$REV:include/ghs_mst.h" > "$T/include/ghs_mst.h"
for f in $(git -C "$ROOT" ls-tree --name-only "$REV" distributed_ghs_implementation_amd/csrc/); do
  git -C "$ROOT" show "$REV:$f" > "$T/x/csrc/$(basename "$f")"
done
cd "$T/x/csrc"
F="-O3 -std=c++17 -fPIC --offload-arch=gfx950"
for s in boruvka ingest host multi; do [ -f $s.hip ] && { /opt/rocm/bin/hipcc $F -c -o $s.o $s.hip 2>&1 | grep -v hip-link || true; }; done
mkdir -p "$ROOT/distributed_ghs_implementation_amd/lib/exp"
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o "$ROOT/distributed_ghs_implementation_amd/lib/exp/$NAME.so" *.o -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
rm -rf "$T"
echo "built $NAME.so from $REV"
