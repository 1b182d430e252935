set -o pipefail
# the single all-gather of the segmented exchange: GPU DP tests, 8-rank gloo rehearsal
mkdir -p gpurun_out/r04v
timeout -k 10 600 python -u -m pytest tests/test_gpu_dp.py -x -q -rf --timeout 200 --timeout-method thread > gpurun_out/r04v/pytest_dp.log 2>&1; RC=$?
tail -2 gpurun_out/r04v/pytest_dp.log; [ $RC -eq 0 ] || exit $RC
timeout -k 10 600 python bench.py --gpus 8 --backend gloo --steps 2 --warmup 1 --pretrain 20 --no-cpu-baseline > gpurun_out/r04v/bench_gloo8.json 2> gpurun_out/r04v/bench_gloo8.err || { tail -8 gpurun_out/r04v/bench_gloo8.err; exit 1; }
cut -c1-200 gpurun_out/r04v/bench_gloo8.json
