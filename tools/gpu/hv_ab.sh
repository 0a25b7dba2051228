set -o pipefail
mkdir -p gpurun_out/hv5
GHS_HV=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q --timeout 200 --timeout-method thread -k "heavy_buckets or s24_full" > gpurun_out/hv5/pytest.log 2>&1 || { tail -30 gpurun_out/hv5/pytest.log; exit 1; }
tail -2 gpurun_out/hv5/pytest.log


TAG=hv5 REPS=2 VARIANTS="off:GHS_HV=0 on4:GHS_HV=1" TOPK=4 bash tools/gpu/ab.sh

