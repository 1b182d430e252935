#!/bin/bash
# r03c: TV records / fused TV step tests, driver tests, SLP A/B, config 3
set -o pipefail
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_scatter.py tests/test_gpu_driver.py tests/test_gpu_dp.py -m gpu -v -rf --timeout 120 --timeout-method thread > $OUT/pytest_gpu_r03c.log 2>&1
RC=$?; echo "pytest rc=$RC"; grep -E "passed|failed" $OUT/pytest_gpu_r03c.log | tail -2
[ $RC -le 1 ] || exit $RC
for V in base noslp base noslp; do
  if [ $V = base ]; then L=hashnerf-pytorch_amd/lib/libhashnerf_amd.so; else L=hashnerf-pytorch_amd/build/var_$V.so; fi
  HN_LIB_PATH=$L timeout -k 10 300 python bench.py --no-cpu-baseline > $OUT/ab_$V.json 2> $OUT/ab_$V.err || exit 3
  python -c "import json;d=json.load(open('$OUT/ab_$V.json'));print('$V', d['value'], d['ms_per_step'], d['kernels']['render_fwd_ms'], d['kernels']['render_bwd_ms'])"
done
timeout -k 10 600 python bench.py --config 3 --no-cpu-baseline > $OUT/bench_config3_r03c.json 2> $OUT/bench_config3_r03c.err || exit 4
python -c "import json;d=json.load(open('$OUT/bench_config3_r03c.json'));print('config3', d['value'], d['ms_per_step'], d['kernels'])"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_r03c -o prof -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --config 3 > $OUT/prof_r03c.log 2>&1 || exit 5
python3 scripts/trace_tail_stats.py $OUT/prof_r03c/prof_kernel_trace.csv 10 > $OUT/prof_r03c/prof_kernel_stats_timed.csv; rm -f $OUT/prof_r03c/prof_kernel_trace.csv
head -16 $OUT/prof_r03c/prof_kernel_stats_timed.csv | cut -c1-110
