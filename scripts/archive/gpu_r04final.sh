set -o pipefail
# final check of the committed tree (round-4 final library): GPU tests, smoke, bench line, 2-rank gloo
# rehearsal of the bench's data-parallel path
mkdir -p gpurun_out/r04f
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 150 --timeout-method thread > gpurun_out/r04f/pytest_gpu.log 2>&1; RC=$?
tail -2 gpurun_out/r04f/pytest_gpu.log; [ $RC -eq 0 ] || exit $RC
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04f/smoke.txt 2>&1 || { tail -5 gpurun_out/r04f/smoke.txt; exit 1; }
tail -1 gpurun_out/r04f/smoke.txt
timeout -k 10 600 python bench.py > gpurun_out/r04f/bench_full.json 2> gpurun_out/r04f/bench_full.err || { tail -5 gpurun_out/r04f/bench_full.err; exit 1; }
cut -c1-200 gpurun_out/r04f/bench_full.json
timeout -k 10 600 python bench.py --gpus 2 --backend gloo --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r04f/bench_gloo2.json 2> gpurun_out/r04f/bench_gloo2.err || { tail -5 gpurun_out/r04f/bench_gloo2.err; exit 1; }
cut -c1-200 gpurun_out/r04f/bench_gloo2.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04f/prof -o prof -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r04f/prof.log 2>&1 || { tail -5 gpurun_out/r04f/prof.log; exit 1; }
F=$(find gpurun_out/r04f/prof -name "*kernel_trace.csv" | head -1)
python3 scripts/trace_tail_stats.py $F 10 > gpurun_out/r04f/kernel_stats_r04f.csv
S=$(find gpurun_out/r04f/prof -name "*kernel_stats.csv" | head -1); cp $S gpurun_out/r04f/rocprof_kernel_stats_r04f.csv; rm -rf gpurun_out/r04f/prof
cut -d, -f1,2,4 gpurun_out/r04f/kernel_stats_r04f.csv | head -6
