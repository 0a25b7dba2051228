#!/bin/bash
# Round 6: the CSR entry — its parity tests, then the s24 line in both input forms (same box), and
# variant libraries (VARIANTS="name:lib.so:form ...").
set -o pipefail
OUT=gpurun_out/${TAG:-r06csr}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
if [ -z "$NOTEST" ]; then
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_csr.py ${PYARGS:--x} -v --timeout 300 --timeout-method thread > "$OUT/pytest_csr.log" 2>&1
rc=$?; tail -3 "$OUT/pytest_csr.log"; [ $rc -ne 0 ] && { echo "csr tests rc=$rc"; grep -E "FAILED|Error|error" "$OUT/pytest_csr.log" | head -20; exit 1; }
fi
L=distributed_ghs_implementation_amd/lib
for rep in $(seq 1 ${REPS:-2}); do
for v in ${VARIANTS:-coo:libghs_mst.so:coo csr:libghs_mst.so:csr}; do
  name=${v%%:*}; rest=${v#*:}; lib=${rest%%:*}; form=${rest#*:}
  GHS_MST_LIB=$L/$lib timeout -k 10 240 python3 -u bench.py --no-cpu-baseline --no-scaling-base --input $form $BARGS > "$OUT/bench_$name.$rep.json" 2> "$OUT/bench_$name.$rep.err" || { echo "bench $name failed"; tail -5 "$OUT/bench_$name.$rep.err"; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/bench_$name.$rep.json'));k=d['kernels'];print('$name', d['ms_per_step'], 'sel', k['k_select']['ms_per_step'], 'filt', k['k_filter']['ms_per_step'], 'lp', k.get('k_level_pass',{}).get('ms_per_step'), 's1', d['stage1_roofline']['frac'])"
done
done
