set -o pipefail
# the library in the tree at the end of round 4: GPU tests, smoke, bench line
mkdir -p gpurun_out/r04last
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 150 --timeout-method thread > gpurun_out/r04last/pytest_gpu.log 2>&1; RC=$?
tail -2 gpurun_out/r04last/pytest_gpu.log; [ $RC -eq 0 ] || exit $RC
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04last/smoke.txt 2>&1 || { tail -5 gpurun_out/r04last/smoke.txt; exit 1; }
tail -1 gpurun_out/r04last/smoke.txt
timeout -k 10 600 python bench.py > gpurun_out/r04last/bench_full.json 2> gpurun_out/r04last/bench_full.err || { tail -5 gpurun_out/r04last/bench_full.err; exit 1; }
cut -c1-200 gpurun_out/r04last/bench_full.json
