set -o pipefail
# round-4 final check of the committed tree: every GPU test, smoke, the full
# bench line (CPU baseline included), kernel stats and PMC traffic
mkdir -p gpurun_out/r04o
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 150 --timeout-method thread > gpurun_out/r04o/pytest_gpu.log 2>&1; RC=$?
tail -3 gpurun_out/r04o/pytest_gpu.log; [ $RC -eq 0 ] || exit $RC
grep "short PSNR gate" gpurun_out/r04o/pytest_gpu.log || true
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04o/smoke.txt 2>&1 || { tail -5 gpurun_out/r04o/smoke.txt; exit 1; }
tail -2 gpurun_out/r04o/smoke.txt
timeout -k 10 600 python bench.py > gpurun_out/r04o/bench_full.json 2> gpurun_out/r04o/bench_full.err || { tail -5 gpurun_out/r04o/bench_full.err; exit 1; }
cut -c1-300 gpurun_out/r04o/bench_full.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04o/prof -o prof -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r04o/prof.log 2>&1 || { tail -5 gpurun_out/r04o/prof.log; exit 1; }
F=$(find gpurun_out/r04o/prof -name "*kernel_trace.csv" | head -1)
python3 scripts/trace_tail_stats.py $F 10 > gpurun_out/r04o/kernel_stats_r04o.csv
S=$(find gpurun_out/r04o/prof -name "*kernel_stats.csv" | head -1); cp $S gpurun_out/r04o/rocprof_kernel_stats_r04o.csv; rm -rf gpurun_out/r04o/prof
cut -d, -f1,2,4 gpurun_out/r04o/kernel_stats_r04o.csv | head -8
PMC_PASSES="FETCH_SIZE;WRITE_SIZE" timeout -k 10 400 bash scripts/gpu_pmc.sh r04o > gpurun_out/r04o/pmc.txt 2>&1; echo "pmc rc=$?"
