#!/bin/bash
# r03d: TV records inside the scatter kernel; config 3; default bench
set -o pipefail
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_scatter.py tests/test_gpu_driver.py tests/test_gpu_dp.py -m gpu -v -rf --timeout 120 --timeout-method thread > $OUT/pytest_gpu_r03d.log 2>&1
RC=$?; echo "pytest rc=$RC"; grep -E "passed|failed" $OUT/pytest_gpu_r03d.log | tail -2
[ $RC -le 1 ] || exit $RC
timeout -k 10 300 python bench.py --no-cpu-baseline > $OUT/bench_r03d.json 2> $OUT/bench_r03d.err || exit 3
python -c "import json;d=json.load(open('$OUT/bench_r03d.json'));print('config2', d['value'], d['ms_per_step'], d['kernels'])"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_r03d -o prof -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --config 3 > $OUT/prof_r03d.log 2>&1 || exit 5
python3 scripts/trace_tail_stats.py $OUT/prof_r03d/prof_kernel_trace.csv 10 > $OUT/prof_r03d/prof_kernel_stats_timed.csv; rm -f $OUT/prof_r03d/prof_kernel_trace.csv
head -12 $OUT/prof_r03d/prof_kernel_stats_timed.csv | cut -c1-110
timeout -k 10 600 python bench.py --config 3 --no-cpu-baseline > $OUT/bench_config3_r03d.json 2> $OUT/bench_config3_r03d.err || exit 4
python -c "import json;d=json.load(open('$OUT/bench_config3_r03d.json'));print('config3', d['value'], d['ms_per_step'], d['kernels'])"
for V in base lg4 base lg4; do
  if [ $V = base ]; then L=hashnerf-pytorch_amd/lib/libhashnerf_amd.so; else L=hashnerf-pytorch_amd/build/var_$V.so; fi
  HN_LIB_PATH=$L timeout -k 10 300 python bench.py --no-cpu-baseline > $OUT/ab_$V.json 2> $OUT/ab_$V.err || exit 6
  python -c "import json;d=json.load(open('$OUT/ab_$V.json'));print('$V', d['value'], d['ms_per_step'], d['kernels']['render_fwd_ms'], d['kernels']['render_bwd_ms'])"
done
HN_LIB_PATH=hashnerf-pytorch_amd/build/var_lg4.so timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_r03d_lg4 -o prof -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > $OUT/prof_r03d_lg4.log 2>&1 || exit 7
python3 scripts/trace_tail_stats.py $OUT/prof_r03d_lg4/prof_kernel_trace.csv 10 > $OUT/prof_r03d_lg4/prof_kernel_stats_timed.csv; rm -f $OUT/prof_r03d_lg4/prof_kernel_trace.csv
head -8 $OUT/prof_r03d_lg4/prof_kernel_stats_timed.csv | cut -c1-110
HN_LIB_PATH=hashnerf-pytorch_amd/build/var_lg4.so PMC_PASSES="WRITE_SIZE" timeout -k 10 300 bash scripts/gpu_pmc.sh r03d_lg4 > $OUT/pmc_r03d_lg4.out 2>&1 || exit 8
PMC_PASSES="WRITE_SIZE" timeout -k 10 300 bash scripts/gpu_pmc.sh r03d_base > $OUT/pmc_r03d_base.out 2>&1 || exit 9
grep -A2 "scatter_bins\|bin_reduce" $OUT/pmc_r03d_lg4.txt $OUT/pmc_r03d_base.txt
