#!/bin/bash
# Build libghs_mst.so from the working tree with extra compile flags into
# distributed_ghs_implementation_amd/lib/exp/<name>.so (same-box A/B: tools/gpu/ab.sh with
# GHS_MST_LIB=...). Usage: tools/build_variant.sh NAME "-DGHS_X=1 ..."
set -e
NAME=$1; EXTRA=$2
ROOT=$(cd "$(dirname "$0")/.." && pwd)
T=$(mktemp -d)
cd "$ROOT/distributed_ghs_implementation_amd/csrc"
F="-O3 -std=c++17 -fPIC --offload-arch=gfx950 $EXTRA"
for s in boruvka ingest host multi; do /opt/rocm/bin/hipcc $F -c -o $T/$s.o $s.hip 2>&1 | grep -v hip-link || true; done
mkdir -p "$ROOT/distributed_ghs_implementation_amd/lib/exp"
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o "$ROOT/distributed_ghs_implementation_amd/lib/exp/$NAME.so" $T/boruvka.o $T/ingest.o $T/host.o $T/multi.o -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
rm -rf "$T"
echo "built $NAME.so with $EXTRA"
