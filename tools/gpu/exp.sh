set -o pipefail
export TMPDIR=/tmp
for x in 0 1 2; do
GHS_EXP=$x timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/exp$x -o run -- python3 bench.py --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/exp$x.json 2>/dev/null || exit 1
python3 tools/prof_summary.py gpurun_out/exp$x/run_results.db | grep canon
done
