set -o pipefail
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_blender_data.py tests/test_gpu_dp.py tests/test_gpu_driver.py tests/test_gpu_scatter.py tests/test_capi.py -m gpu -v -rf --timeout 120 --timeout-method thread > $OUT/pytest_gpu_r03b.log 2>&1
RC=$?; echo "pytest rc=$RC"; grep -E "passed|failed" $OUT/pytest_gpu_r03b.log | tail -2
[ $RC -le 1 ] || exit $RC
timeout -k 10 600 python bench.py --config 5 --no-cpu-baseline > $OUT/bench_config5_r03b.json 2> $OUT/bench_config5_r03b.err || exit 3
cat $OUT/bench_config5_r03b.json | cut -c1-400
timeout -k 10 600 python bench.py --config 3 --no-cpu-baseline > $OUT/bench_config3_r03b.json 2> $OUT/bench_config3_r03b.err || exit 4
cat $OUT/bench_config3_r03b.json | cut -c1-300
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_r03b -o prof -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > $OUT/prof_r03b.log 2>&1 && python3 scripts/trace_tail_stats.py $OUT/prof_r03b/prof_kernel_trace.csv 10 > $OUT/prof_r03b/prof_kernel_stats_timed.csv; rm -f $OUT/prof_r03b/prof_kernel_trace.csv; head -8 $OUT/prof_r03b/prof_kernel_stats_timed.csv | cut -c1-100
PMC_PASSES="SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE;SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU" timeout -k 10 400 bash scripts/gpu_pmc.sh r03b > $OUT/pmc_r03b.out 2>&1 || { tail $OUT/pmc_r03b.out; exit 5; }
grep -A12 "render_bwd_kernel\|render_fwd_kernel" $OUT/pmc_r03b.txt | head -40
