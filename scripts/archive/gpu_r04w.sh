set -o pipefail
# final check of the committed tree (library as build() leaves it): GPU tests, smoke, bench line, 2-rank gloo
# rehearsal of the bench's data-parallel path
mkdir -p gpurun_out/r04w
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 150 --timeout-method thread > gpurun_out/r04w/pytest_gpu.log 2>&1; RC=$?
tail -2 gpurun_out/r04w/pytest_gpu.log; [ $RC -eq 0 ] || exit $RC
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04w/smoke.txt 2>&1 || { tail -5 gpurun_out/r04w/smoke.txt; exit 1; }
tail -1 gpurun_out/r04w/smoke.txt
timeout -k 10 600 python bench.py > gpurun_out/r04w/bench_full.json 2> gpurun_out/r04w/bench_full.err || { tail -5 gpurun_out/r04w/bench_full.err; exit 1; }
cut -c1-200 gpurun_out/r04w/bench_full.json
timeout -k 10 600 python bench.py --gpus 2 --backend gloo --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r04w/bench_gloo2.json 2> gpurun_out/r04w/bench_gloo2.err || { tail -5 gpurun_out/r04w/bench_gloo2.err; exit 1; }
cut -c1-200 gpurun_out/r04w/bench_gloo2.json
